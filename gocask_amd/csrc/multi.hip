// multi.hip — several GPUs behind one C-ABI call.
//
// gck_replay_multi is gck_replay over a device list: the files (walk order)
// are cut into one contiguous shard per device, only after files that reset
// lastOffset (gck_plan_shards), so every shard replays exactly as the global
// walk would (core/db.go:110-138); each shard replays on its own device from a
// host thread; the first startup error in walk order ends the walk
// (core/db.go:134-138, internal/fs/disk.go:134-141): its shard's records
// before the error count, later shards contribute nothing.  The one exchange
// step is the keydir merge (keyDir.set / unset over all files in walk order,
// core/keydir.go:22-49):
//   1. per shard, the keydir with tombstones kept (a later shard's delete must
//      hide an earlier shard's Put), partitioned by key hash over the devices
//      (gck_ctx_keydir, gck_kd_pack_sizes, gck_kd_pack);
//   2. partition p of every shard moves to device p in shard order: RCCL
//      point-to-point over xGMI (ncclCommInitAll over the devices, grouped
//      ncclSend / ncclRecv; the counts are all known to this one process, so
//      no size exchange is needed);
//   3. per owner, the highest shard's entry of each key wins and a winning
//      tombstone drops the key (gck_kd_merge).
// The owners' live entries together are the global keydir; they come back as
// gck_recs with global file indices.
//
// RCCL is loaded at the first multi-GPU call (dlopen of librccl.so.1: the copy
// a host process such as torch already loaded, else the system's), so the
// library itself links only the HIP runtime.
#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include <rccl/rccl.h>  // types only: the entry points are resolved with dlsym

#include "gck_internal.h"

namespace {

struct Rccl {
    ncclResult_t (*init_all)(ncclComm_t *, int, const int *) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*group_start)() = nullptr;
    ncclResult_t (*group_end)() = nullptr;
    ncclResult_t (*send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    const char *(*err)(ncclResult_t) = nullptr;
    bool ok = false;
};

const Rccl &rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (!h) return;
        r.init_all = reinterpret_cast<decltype(r.init_all)>(dlsym(h, "ncclCommInitAll"));
        r.destroy = reinterpret_cast<decltype(r.destroy)>(dlsym(h, "ncclCommDestroy"));
        r.group_start = reinterpret_cast<decltype(r.group_start)>(dlsym(h, "ncclGroupStart"));
        r.group_end = reinterpret_cast<decltype(r.group_end)>(dlsym(h, "ncclGroupEnd"));
        r.send = reinterpret_cast<decltype(r.send)>(dlsym(h, "ncclSend"));
        r.recv = reinterpret_cast<decltype(r.recv)>(dlsym(h, "ncclRecv"));
        r.err = reinterpret_cast<decltype(r.err)>(dlsym(h, "ncclGetErrorString"));
        r.ok = r.init_all && r.destroy && r.group_start && r.group_end && r.send && r.recv && r.err;
    });
    return r;
}

// Communicators over a device list, kept for the next call with the same list
// (ncclCommInitAll costs far more than a replay of a small database).
std::mutex g_comm_mu;
std::vector<std::pair<std::vector<int>, std::vector<ncclComm_t>>> g_comms;

int comms_for(const std::vector<int> &devs, std::vector<ncclComm_t> &out) {
    const Rccl &R = rccl();
    if (!R.ok) {
        gck::set_error("dlopen librccl.so.1", hipErrorSharedObjectInitFailed, __FILE__, __LINE__);
        return GCK_EDEVICE;
    }
    std::lock_guard<std::mutex> lk(g_comm_mu);
    for (auto &e : g_comms)
        if (e.first == devs) {
            out = e.second;
            return GCK_OK;
        }
    std::vector<ncclComm_t> c(devs.size(), nullptr);
    const ncclResult_t r = R.init_all(c.data(), (int)devs.size(), devs.data());
    if (r != ncclSuccess) {
        gck::set_error(R.err(r), hipErrorUnknown, __FILE__, __LINE__);
        return GCK_EDEVICE;
    }
    g_comms.emplace_back(devs, c);
    out = c;
    return GCK_OK;
}

struct Shard {
    uint32_t a = 0, b = 0;  // files [a, b)
    gck_ctx *ctx = nullptr;
    int rc = GCK_OK;
    gck_stats st{};
    uint64_t counts[64] = {}, kbytes[64] = {};  // per owner
    void *d_ents = nullptr, *d_keys = nullptr;  // packed partitions (device of the shard)
    void *r_ents = nullptr, *r_keys = nullptr;  // what this device owns, sources in shard order
};

}  // namespace

using namespace gck;

extern "C" int gck_plan_shards(const uint64_t *sizes, const uint8_t *reset_after, uint32_t nfiles, uint32_t world,
                               uint32_t *ranges) {
    // gocask_amd/shard.py plan_shards: `world` contiguous ranges of about
    // equal bytes; a cut at i (between files i - 1 and i) only where file
    // i - 1 resets lastOffset (core/db.go:117-119); ranges may be empty.
    if (world == 0 || !ranges || (nfiles && (!sizes || !reset_after))) return GCK_EINVAL;
    std::vector<uint64_t> prefix(nfiles + 1, 0);
    for (uint32_t f = 0; f < nfiles; ++f) prefix[f + 1] = prefix[f] + sizes[f];
    std::vector<uint32_t> ok;
    for (uint32_t i = 1; i < nfiles; ++i)
        if (reset_after[i - 1]) ok.push_back(i);
    std::vector<uint32_t> bounds{0};
    uint32_t lo = 0;
    for (uint32_t k = 1; k < world; ++k) {
        const double target = (double)prefix[nfiles] * k / world;
        int64_t best = -1;
        double bd = 0;
        for (uint32_t i : ok) {
            if (i < lo) continue;
            const double d = std::abs((double)prefix[i] - target);
            if (best < 0 || d < bd) {  // ties: the smaller i (ok is increasing)
                best = i;
                bd = d;
            }
        }
        if (best < 0) {
            bounds.push_back(nfiles);
            continue;
        }
        bounds.push_back((uint32_t)best);
        lo = (uint32_t)best;
    }
    bounds.push_back(nfiles);
    for (uint32_t r = 0; r < world; ++r) {
        ranges[2 * r] = bounds[r];
        ranges[2 * r + 1] = std::max(bounds[r], bounds[r + 1]);
    }
    return GCK_OK;
}

static int replay_multi(const Src *files, uint32_t nfiles, const int32_t *devices, uint32_t ndev,
                        const gck_opts *opts, gck_result *out) {
    if ((nfiles && !files) || !devices || ndev == 0 || ndev > 64) return GCK_EINVAL;
    for (uint32_t f = 0; f < nfiles; ++f)
        if (files[f].len && !files[f].data && files[f].fd < 0) return GCK_EINVAL;
    const bool want_keys = opts && (opts->flags & GCK_OPT_KEYS);
    std::vector<int> devs(devices, devices + ndev);
    {
        std::vector<int> s = devs;
        std::sort(s.begin(), s.end());
        if (std::adjacent_find(s.begin(), s.end()) != s.end()) return GCK_EINVAL;  // one rank per device
    }
    std::vector<uint64_t> sizes(nfiles);
    std::vector<uint8_t> reset(nfiles);
    for (uint32_t f = 0; f < nfiles; ++f) {
        sizes[f] = files[f].len;
        reset[f] = files[f].reset_after ? 1 : 0;
    }
    std::vector<uint32_t> ranges(2 * ndev);
    int rc = gck_plan_shards(sizes.data(), reset.data(), nfiles, ndev, ranges.data());
    if (rc) return rc;
    std::vector<Shard> sh(ndev);
    // GCK_REPLAY_TRACE=1: the phases' wall times on stderr
    const bool trace = getenv("GCK_REPLAY_TRACE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        if (trace)
            fprintf(stderr, "gck_replay_multi %-14s %9.2f ms\n", what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    // the communicators come up on their own thread while the shards replay
    // (ncclCommInitAll takes about a second; a later call with the same
    // device list reuses them)
    std::vector<ncclComm_t> comm;
    int comm_rc = GCK_OK;
    std::thread comm_th([&]() { comm_rc = comms_for(devs, comm); });
    auto join_comm = [&]() {
        if (comm_th.joinable()) comm_th.join();
    };
    auto cleanup = [&]() {
        join_comm();
        for (uint32_t s = 0; s < ndev; ++s) {
            if (sh[s].ctx) (void)hipSetDevice(sh[s].ctx->c.device);
            for (void *p : {sh[s].d_ents, sh[s].d_keys, sh[s].r_ents, sh[s].r_keys})
                if (p) (void)hipFree(p);
            if (sh[s].ctx) gck_ctx_destroy(sh[s].ctx);
        }
    };
    // 1. every shard on its device, a host thread each (H2D + replay)
    auto replay_shard = [&](uint32_t s) {
        Shard &x = sh[s];
        x.a = ranges[2 * s];
        x.b = ranges[2 * s + 1];
        gck_opts o{};
        if (opts) o = *opts;
        o.device = devs[s];
        if ((x.rc = gck_ctx_create(&o, &x.ctx))) return;
        if ((x.rc = ctx_load_srcs(&x.ctx->c, files + x.a, x.b - x.a))) return;
        if (x.b > x.a) {
            x.rc = gck_ctx_run(x.ctx);
            if (x.rc == GCK_EUNEXPECTED_EOF) x.rc = GCK_OK;  // the run's outcome is in its stats
            if (x.rc) return;
        }
        x.rc = gck_ctx_stats(x.ctx, &x.st);
    };
    {
        std::vector<std::thread> th;
        for (uint32_t s = 1; s < ndev; ++s) th.emplace_back(replay_shard, s);
        replay_shard(0);
        for (auto &t : th) t.join();
    }
    mark("replayed");
    for (uint32_t s = 0; s < ndev; ++s)
        if (sh[s].rc) {
            rc = sh[s].rc;
            cleanup();
            return rc;
        }
    // 2. the global outcome (gocask_amd/shard.py resolve_status): shards in walk
    // order until the first startup error, which is the global status
    std::vector<bool> contrib(ndev, false);
    out->status = GCK_OK;
    uint32_t base = 0;
    bool failed = false;
    for (uint32_t s = 0; s < ndev; ++s) {
        if (failed) continue;
        contrib[s] = true;
        const gck_stats &st = sh[s].st;
        const uint32_t nf = sh[s].b - sh[s].a;
        out->n_crc_fail += nf ? st.n_crc_fail : 0;
        if (nf && st.status == GCK_EUNEXPECTED_EOF) {
            failed = true;
            out->status = GCK_EUNEXPECTED_EOF;
            out->err_file = base + st.err_file;
            out->err_off = st.err_off;
            out->files_walked = base + st.files_walked;
            out->final_last_offset = st.final_last_offset;
        } else if (nf) {
            out->final_last_offset = st.final_last_offset;  // cuts follow resetting files: the last shard's
        }
        base += nf;
    }
    if (!failed) out->files_walked = nfiles;
    out->n_groups = ndev;
    out->n_resident = ndev;
    // 3. keydir with tombstones per contributing shard, partitioned over the owners
    for (uint32_t s = 0; s < ndev && !rc; ++s) {
        Shard &x = sh[s];
        if (!contrib[s] || x.b == x.a) continue;
        uint64_t n = 0;
        if ((rc = gck_ctx_keydir(x.ctx, GCK_KD_KEEP_TOMBSTONES, &n, nullptr))) break;
        if ((rc = gck_kd_pack_sizes(x.ctx, ndev, x.counts, x.kbytes))) break;
        uint64_t ne = 0, nk = 0;
        for (uint32_t p = 0; p < ndev; ++p) {
            ne += x.counts[p];
            nk += x.kbytes[p];
        }
        if (hipSetDevice(devs[s]) != hipSuccess || hipMalloc(&x.d_ents, ne * sizeof(gck_kd_entry) + 64) != hipSuccess ||
            hipMalloc(&x.d_keys, nk + 64) != hipSuccess) {
            rc = GCK_ENOMEM;
            break;
        }
        rc = gck_kd_pack(x.ctx, s, x.a, static_cast<gck_kd_entry *>(x.d_ents), ne, static_cast<uint8_t *>(x.d_keys), nk);
    }
    mark("packed");
    // receive buffers: owner p gets partition p of every shard, in shard order
    std::vector<std::vector<uint64_t>> e_off(ndev, std::vector<uint64_t>(ndev + 1, 0)),
        k_off(ndev, std::vector<uint64_t>(ndev + 1, 0));
    for (uint32_t p = 0; p < ndev && !rc; ++p) {
        for (uint32_t s = 0; s < ndev; ++s) {
            e_off[p][s + 1] = e_off[p][s] + sh[s].counts[p];
            k_off[p][s + 1] = k_off[p][s] + sh[s].kbytes[p];
        }
        if (hipSetDevice(devs[p]) != hipSuccess ||
            hipMalloc(&sh[p].r_ents, e_off[p][ndev] * sizeof(gck_kd_entry) + 64) != hipSuccess ||
            hipMalloc(&sh[p].r_keys, k_off[p][ndev] + 64) != hipSuccess)
            rc = GCK_ENOMEM;
    }
    // 4. the exchange: RCCL send / recv of every (shard, owner) pair in one group
    join_comm();
    mark("comms");
    if (!rc) {
        rc = comm_rc;
        for (uint32_t s = 0; s < ndev && !rc; ++s) {  // packs done before the sends
            (void)hipSetDevice(devs[s]);
            if (hipStreamSynchronize((hipStream_t)gck_ctx_stream(sh[s].ctx)) != hipSuccess) rc = GCK_EDEVICE;
        }
        if (!rc) {
            const Rccl &R = rccl();
            ncclResult_t r = R.group_start();
            for (uint32_t s = 0; s < ndev && r == ncclSuccess; ++s) {
                uint64_t eo = 0, ko = 0;  // shard s's pack offsets of partition p
                for (uint32_t p = 0; p < ndev && r == ncclSuccess; ++p) {
                    const uint64_t ne = sh[s].counts[p], nk = sh[s].kbytes[p];
                    hipStream_t ss = (hipStream_t)gck_ctx_stream(sh[s].ctx), sp = (hipStream_t)gck_ctx_stream(sh[p].ctx);
                    const uint8_t *se = static_cast<const uint8_t *>(sh[s].d_ents) + eo * sizeof(gck_kd_entry);
                    const uint8_t *sk = static_cast<const uint8_t *>(sh[s].d_keys) + ko;
                    uint8_t *re = static_cast<uint8_t *>(sh[p].r_ents) + e_off[p][s] * sizeof(gck_kd_entry);
                    uint8_t *rk = static_cast<uint8_t *>(sh[p].r_keys) + k_off[p][s];
                    if (ne) {
                        r = R.send(se, ne * sizeof(gck_kd_entry), ncclUint8, (int)p, comm[s], ss);
                        if (r == ncclSuccess) r = R.recv(re, ne * sizeof(gck_kd_entry), ncclUint8, (int)s, comm[p], sp);
                    }
                    if (nk && r == ncclSuccess) {
                        r = R.send(sk, nk, ncclUint8, (int)p, comm[s], ss);
                        if (r == ncclSuccess) r = R.recv(rk, nk, ncclUint8, (int)s, comm[p], sp);
                    }
                    eo += ne;
                    ko += nk;
                }
            }
            const ncclResult_t r2 = R.group_end();
            if (r == ncclSuccess) r = r2;
            if (r != ncclSuccess) {
                set_error(R.err(r), hipErrorUnknown, __FILE__, __LINE__);
                rc = GCK_EDEVICE;
            }
        }
    }
    mark("exchanged");
    // 5. per owner, the merge; the live entries gathered in owner order
    std::vector<uint64_t> n_live(ndev, 0);
    for (uint32_t p = 0; p < ndev && !rc; ++p) {
        std::vector<uint64_t> sc(ndev), sk(ndev);
        for (uint32_t s = 0; s < ndev; ++s) {
            sc[s] = sh[s].counts[p];
            sk[s] = sh[s].kbytes[p];
        }
        rc = gck_kd_merge(sh[p].ctx, static_cast<const gck_kd_entry *>(sh[p].r_ents),
                          static_cast<const uint8_t *>(sh[p].r_keys), sc.data(), sk.data(), ndev, &n_live[p], nullptr);
    }
    uint64_t tot = 0;
    for (uint64_t v : n_live) tot += v;
    gck_rec *h = nullptr;
    if (!rc && tot) {
        h = static_cast<gck_rec *>(res_alloc(tot * sizeof(gck_rec), false));  // filled by the host below
        if (!h) rc = GCK_ENOMEM;
    }
    uint64_t at = 0;
    std::vector<uint8_t> kblob;  // GCK_OPT_KEYS: the entries' key bytes in output order
    for (uint32_t p = 0; p < ndev && !rc; ++p) {
        uint64_t n = 0, nk = 0;
        if ((rc = gck_kd_fetch_merged(sh[p].ctx, nullptr, 0, nullptr, 0, &n, &nk))) break;
        if (!n) continue;
        std::vector<gck_kd_entry> ents(n);
        std::vector<uint8_t> keys(nk + 1);
        if ((rc = gck_kd_fetch_merged(sh[p].ctx, ents.data(), n, keys.data(), nk + 1, &n, &nk))) break;
        for (uint64_t i = 0; i < n; ++i) {
            h[at + i] = ents[i].rec;
            if (want_keys) kblob.insert(kblob.end(), keys.begin() + (ptrdiff_t)ents[i].key_off,
                                        keys.begin() + (ptrdiff_t)(ents[i].key_off + ents[i].key_len));
        }
        at += n;
    }
    if (!rc && want_keys) {
        out->keys = static_cast<uint8_t *>(res_alloc(kblob.size(), false));
        if (!out->keys) rc = GCK_ENOMEM;
        else if (!kblob.empty()) memcpy(out->keys, kblob.data(), kblob.size());
        out->keys_len = kblob.size();
    }
    mark("merged+fetched");
    cleanup();
    mark("freed");
    if (rc) {
        res_free(h);
        res_free(out->keys);
        memset(out, 0, sizeof(*out));
        return rc;
    }
    out->recs = h;
    out->n = tot;
    return out->status;
}

extern "C" int gck_replay_multi(const gck_file *files, uint32_t nfiles, const int32_t *devices, uint32_t ndev,
                                const gck_opts *opts, gck_result *out) {
    if (!out) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    if (nfiles && !files) return GCK_EINVAL;
    const std::vector<Src> v = mem_srcs(files, nfiles);
    return replay_multi(v.data(), nfiles, devices, ndev, opts, out);
}

extern "C" int gck_replay_multi_paths(const gck_path *files, uint32_t nfiles, const int32_t *devices, uint32_t ndev,
                                      const gck_opts *opts, gck_result *out) {
    if (!out) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    if (nfiles && !files) return GCK_EINVAL;
    std::vector<Src> v;
    int rc = open_srcs(files, nfiles, v);
    if (rc) return rc;
    rc = replay_multi(v.data(), nfiles, devices, ndev, opts, out);
    close_srcs(v);
    return rc;
}
