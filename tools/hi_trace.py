import sys, time, numpy as np
sys.path.insert(0, '.')
import bench, gocask_amd as g
ctx = g.ReplayContext()
info = ctx.encode(**bench.CONFIGS['c3'])
ctx.run()
nf = info['n_files']
sizes = [int(info['sizes'][info['walk_order'][w]]) for w in range(nf)]
host = np.empty(sum(sizes), dtype=np.uint8); g.host_register(host)
views, off = [], 0
for w, n in enumerate(sizes):
    views.append(ctx.read_file(w, 0, n, out=host[off:off+n])); off += n
reset = [w + 1 < nf for w in range(nf)]
recs = np.empty(ctx.stats()['n_recs'], dtype=g.REC_DTYPE); g.host_register(recs)
ctx.close()
for i in range(4):
    t0 = time.perf_counter(); st = g.replay_into(views, recs, reset); t1 = time.perf_counter()
    print('replay_into ms', round((t1-t0)*1e3, 2), st['n_recs'], flush=True)
