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
#include <memory>
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
// (ncclCommInitAll costs far more than a replay of a small database).  A set is
// used by one call at a time: its mutex is held from ncclGroupStart until the
// exchange's streams are synchronised (NCCL forbids concurrent use of a
// communicator from several threads; two Opens would otherwise interleave).
struct CommSet {
    std::vector<int> devs;
    std::vector<ncclComm_t> comms;
    std::shared_ptr<std::mutex> mu;
};
std::mutex g_comm_mu;
std::vector<CommSet> g_comms;

int comms_for(const std::vector<int> &devs, CommSet &out) {
    const Rccl &R = rccl();
    if (!R.ok) {
        gck::set_error("dlopen librccl.so.1", hipErrorSharedObjectInitFailed, __FILE__, __LINE__);
        return GCK_EDEVICE;
    }
    std::lock_guard<std::mutex> lk(g_comm_mu);
    for (auto &e : g_comms)
        if (e.devs == devs) {
            out = e;
            return GCK_OK;
        }
    CommSet c{devs, std::vector<ncclComm_t>(devs.size(), nullptr), std::make_shared<std::mutex>()};
    const ncclResult_t r = R.init_all(c.comms.data(), (int)devs.size(), devs.data());
    if (r != ncclSuccess) {
        gck::set_error(R.err(r), hipErrorUnknown, __FILE__, __LINE__);
        return GCK_EDEVICE;
    }
    g_comms.push_back(c);
    out = c;
    return GCK_OK;
}

// One replayed file group's keydir (tombstones kept), packed over the owners:
// entries and key bytes partition-major, in its own device buffers (the
// group's ring context is reused for a later group as soon as this is done).
struct Part {
    uint32_t file0 = 0;  // global walk index of the group's first file
    uint64_t counts[64] = {}, kbytes[64] = {};
    void *d_ents = nullptr, *d_keys = nullptr;
};

// A shard's replay through gck_replay's ring (replay_groups_to): after each
// group has replayed, its keydir is built and packed on the device.
struct ShardRun : gck::GroupSink {
    uint32_t shard = 0, a = 0, b = 0, nown = 1;
    int dev = 0;
    int rc = GCK_OK;
    gck_result res{};
    std::vector<Part> parts;
    int group(uint32_t, uint32_t file0, gck_ctx *ctx) override {
        uint64_t n = 0;
        int r;
        if ((r = gck_ctx_keydir(ctx, GCK_KD_KEEP_TOMBSTONES, &n, nullptr))) return r;
        parts.emplace_back();
        Part &p = parts.back();
        p.file0 = a + file0;
        if ((r = gck_kd_pack_sizes(ctx, nown, p.counts, p.kbytes))) return r;
        uint64_t ne = 0, nk = 0;
        for (uint32_t o = 0; o < nown; ++o) {
            ne += p.counts[o];
            nk += p.kbytes[o];
        }
        if (hipSetDevice(dev) != hipSuccess || hipMalloc(&p.d_ents, ne * sizeof(gck_kd_entry) + 64) != hipSuccess ||
            hipMalloc(&p.d_keys, nk + 64) != hipSuccess) {
            (void)hipGetLastError();
            return GCK_ENOMEM;
        }
        return gck_kd_pack(ctx, shard, p.file0, static_cast<gck_kd_entry *>(p.d_ents), ne,
                           static_cast<uint8_t *>(p.d_keys), nk);
    }
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

namespace gck {

// The global outcome of a sharded replay (gocask_amd/shard.py resolve_status;
// core/db.go:110-138, internal/fs/disk.go:134-141): shards in walk order until
// the first startup error, which is the global status (its file and offset
// rebased to the whole walk); later shards contribute nothing.  CRC rejects
// sum over the contributing shards; final_last_offset is the last
// contributing shard's (cuts follow files that reset it).
void multi_resolve(const MultiOutcome *sh, uint32_t n, uint32_t nfiles, gck_result *out, uint8_t *contrib) {
    out->status = GCK_OK;
    out->err_file = 0;
    out->err_off = 0;
    out->n_crc_fail = 0;
    out->final_last_offset = 0;
    uint32_t base = 0;
    bool failed = false;
    for (uint32_t s = 0; s < n; ++s) {
        contrib[s] = !failed;
        if (failed) continue;
        const MultiOutcome &st = sh[s];
        if (st.nfiles) out->n_crc_fail += st.n_crc_fail;
        if (st.nfiles && st.status == GCK_EUNEXPECTED_EOF) {
            failed = true;
            out->status = GCK_EUNEXPECTED_EOF;
            out->err_file = base + st.err_file;
            out->err_off = st.err_off;
            out->files_walked = base + st.files_walked;
            out->final_last_offset = st.final_last_offset;
        } else if (st.nfiles) {
            out->final_last_offset = st.final_last_offset;
        }
        base += st.nfiles;
    }
    if (!failed) out->files_walked = nfiles;
}

// Receive layout of the exchange: owner p gets partition p of every source in
// source (= walk) order; off[p * (nsrc + 1) + i] = the items of sources before
// i (counts[i * nown + p] items from source i).
void multi_recv_offsets(const uint64_t *counts, uint32_t nsrc, uint32_t nown, uint64_t *off) {
    for (uint32_t p = 0; p < nown; ++p) {
        uint64_t *o = off + (uint64_t)p * (nsrc + 1);
        o[0] = 0;
        for (uint32_t i = 0; i < nsrc; ++i) o[i + 1] = o[i] + counts[(uint64_t)i * nown + p];
    }
}

// Steps 3-5 of a sharded replay, shared by gck_replay_multi and
// gck_ctx_multi_keydir: the packed sources (walk order) exchanged so that
// owner p holds partition p of every source in source order -- a device copy
// where source and owner share a device, RCCL send / receive pairs in one
// group across devices (every count is known here: no size exchange) -- then
// per owner the merge (the last writer wins, a winning tombstone drops the
// key) and the owners' live entries gathered on the host (*h, *tot; with
// want_keys their key bytes in out->keys).  h == nullptr: counted only.
// ph_ms (optional): [exchange, merge, fetch] wall milliseconds.
struct SrcRef {
    uint32_t shard;
    const Part *part;
};
static int exchange_merge(const std::vector<SrcRef> &srcs, const std::vector<int> &devs,
                          const std::vector<gck_ctx *> &mctx, bool need_rccl, bool rccl_self, CommSet &cset,
                          bool want_keys, bool trace, gck_rec **h_out, uint64_t *tot_out, gck_result *out,
                          double *ph_ms) {
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
    const uint32_t ndev = (uint32_t)devs.size();
    int rc = GCK_OK;
    const uint32_t nsrc = (uint32_t)srcs.size();
    if (nsrc > 65536) return GCK_EINVAL;
    std::vector<void *> r_ents(ndev, nullptr), r_keys(ndev, nullptr);
    auto free_recv = [&]() {
        for (uint32_t p = 0; p < ndev; ++p) {
            (void)hipSetDevice(devs[p]);
            for (void *q : {r_ents[p], r_keys[p]})
                if (q) (void)hipFree(q);
        }
    };
    std::vector<uint64_t> cnt((uint64_t)nsrc * ndev), kb((uint64_t)nsrc * ndev);
    for (uint32_t i = 0; i < nsrc; ++i)
        for (uint32_t p = 0; p < ndev; ++p) {
            cnt[(uint64_t)i * ndev + p] = srcs[i].part->counts[p];
            kb[(uint64_t)i * ndev + p] = srcs[i].part->kbytes[p];
        }
    std::vector<uint64_t> e_off((uint64_t)ndev * (nsrc + 1)), k_off((uint64_t)ndev * (nsrc + 1));
    multi_recv_offsets(cnt.data(), nsrc, ndev, e_off.data());
    multi_recv_offsets(kb.data(), nsrc, ndev, k_off.data());
    auto EO = [&](uint32_t p, uint32_t i) { return e_off[(uint64_t)p * (nsrc + 1) + i]; };
    auto KO = [&](uint32_t p, uint32_t i) { return k_off[(uint64_t)p * (nsrc + 1) + i]; };
    for (uint32_t p = 0; p < ndev && !rc; ++p) {
        if (hipSetDevice(devs[p]) != hipSuccess ||
            hipMalloc(&r_ents[p], EO(p, nsrc) * sizeof(gck_kd_entry) + 64) != hipSuccess ||
            hipMalloc(&r_keys[p], KO(p, nsrc) + 64) != hipSuccess) {
            (void)hipGetLastError();
            rc = GCK_ENOMEM;
        }
    }
    const auto t_ex = clk::now();
    if (!rc) {
        std::unique_lock<std::mutex> lk;
        if (need_rccl) lk = std::unique_lock<std::mutex>(*cset.mu);
        // RCCL only when a pair crosses devices: loading librccl registers its
        // kernels, 1.1-4.7 s of a one-device call (GCK_REPLAY_TRACE, round 4)
        static const Rccl kNone{};
        const Rccl &R = need_rccl ? rccl() : kNone;
        bool grouped = false;
        ncclResult_t r = ncclSuccess;
        for (uint32_t i = 0; i < nsrc && !rc && r == ncclSuccess; ++i) {
            const uint32_t s = srcs[i].shard;
            const Part &pt = *srcs[i].part;
            uint64_t eo = 0, ko = 0;  // the part's offsets of partition p
            for (uint32_t p = 0; p < ndev && !rc && r == ncclSuccess; ++p) {
                const uint64_t ne = pt.counts[p], nk = pt.kbytes[p];
                const uint8_t *se = static_cast<const uint8_t *>(pt.d_ents) + eo * sizeof(gck_kd_entry);
                const uint8_t *sk = static_cast<const uint8_t *>(pt.d_keys) + ko;
                uint8_t *re = static_cast<uint8_t *>(r_ents[p]) + EO(p, i) * sizeof(gck_kd_entry);
                uint8_t *rk = static_cast<uint8_t *>(r_keys[p]) + KO(p, i);
                hipStream_t sp = mctx[p]->c.stream, ss = mctx[s]->c.stream;
                eo += ne;
                ko += nk;
                if (devs[s] == devs[p] && !rccl_self) {
                    (void)hipSetDevice(devs[p]);
                    const auto tc = clk::now();
                    if ((ne && hipMemcpyAsync(re, se, ne * sizeof(gck_kd_entry), hipMemcpyDeviceToDevice, sp) != hipSuccess) ||
                        (nk && hipMemcpyAsync(rk, sk, nk, hipMemcpyDeviceToDevice, sp) != hipSuccess))
                        rc = GCK_EDEVICE;
                    if (trace)
                        fprintf(stderr, "gck_replay_multi copy src %u -> owner %u: %llu entries, %llu key bytes, %.2f ms\n", i, p,
                                (unsigned long long)ne, (unsigned long long)nk, ms_since(tc));
                    continue;
                }
                if (!grouped) {
                    r = R.group_start();
                    grouped = true;
                    if (r != ncclSuccess) break;
                }
                if (ne) {
                    r = R.send(se, ne * sizeof(gck_kd_entry), ncclUint8, (int)p, cset.comms[s], ss);
                    if (r == ncclSuccess) r = R.recv(re, ne * sizeof(gck_kd_entry), ncclUint8, (int)s, cset.comms[p], sp);
                }
                if (nk && r == ncclSuccess) {
                    r = R.send(sk, nk, ncclUint8, (int)p, cset.comms[s], ss);
                    if (r == ncclSuccess) r = R.recv(rk, nk, ncclUint8, (int)s, cset.comms[p], sp);
                }
            }
        }
        if (grouped) {
            const ncclResult_t r2 = R.group_end();
            if (r == ncclSuccess) r = r2;
        }
        if (r != ncclSuccess) {
            set_error(R.err ? R.err(r) : "rccl", hipErrorUnknown, __FILE__, __LINE__);
            rc = GCK_EDEVICE;
        }
        // the exchange is complete (and the communicators free for another
        // call) once every owner's stream is
        for (uint32_t p = 0; p < ndev; ++p) {
            (void)hipSetDevice(devs[p]);
            if (hipStreamSynchronize(mctx[p]->c.stream) != hipSuccess && !rc) rc = GCK_EDEVICE;
        }
    }
    if (ph_ms) ph_ms[0] = ms_since(t_ex);
    // per owner, the merge (sources in walk order: the last writer wins, a
    // winning tombstone drops the key); the live entries gathered in owner order
    const auto t_mg = clk::now();
    std::vector<uint64_t> n_live(ndev, 0);
    for (uint32_t p = 0; p < ndev && !rc; ++p) {
        std::vector<uint64_t> sc(nsrc ? nsrc : 1, 0), sk(nsrc ? nsrc : 1, 0);
        for (uint32_t i = 0; i < nsrc; ++i) {
            sc[i] = cnt[(uint64_t)i * ndev + p];
            sk[i] = kb[(uint64_t)i * ndev + p];
        }
        rc = gck_kd_merge(mctx[p], static_cast<const gck_kd_entry *>(r_ents[p]), static_cast<const uint8_t *>(r_keys[p]),
                          sc.data(), sk.data(), nsrc ? nsrc : 1, &n_live[p], nullptr);
    }
    if (ph_ms) ph_ms[1] = ms_since(t_mg);
    const auto t_fe = clk::now();
    uint64_t tot = 0;
    for (uint64_t v : n_live) tot += v;
    *tot_out = tot;
    // the output in owner order, each owner's part shaped on its device
    // (records, unpadded keys) and copied straight into the result arrays
    gck_rec *h = nullptr;
    std::vector<uint64_t> on(ndev, 0), okb(ndev, 0);
    uint64_t kb_tot = 0;
    for (uint32_t p = 0; p < ndev && !rc && h_out; ++p) {
        rc = merged_out_sizes(&mctx[p]->c, want_keys, &on[p], &okb[p]);
        kb_tot += okb[p];
    }
    if (!rc && tot && h_out) {
        h = static_cast<gck_rec *>(res_alloc(tot * sizeof(gck_rec), false));
        if (!h) rc = GCK_ENOMEM;
    }
    if (!rc && want_keys && h_out) {
        out->keys = static_cast<uint8_t *>(res_alloc(kb_tot, false));
        if (!out->keys) rc = GCK_ENOMEM;
        out->keys_len = kb_tot;
    }
    uint64_t at = 0, kat = 0;
    for (uint32_t p = 0; p < ndev && !rc && h_out; ++p) {
        if (at + on[p] > tot) rc = GCK_EINVAL;  // (the merge's own count: cannot differ)
        else rc = merged_out(&mctx[p]->c, h + at, want_keys ? out->keys + kat : nullptr, okb[p]);
        at += on[p];
        kat += okb[p];
    }
    if (ph_ms) ph_ms[2] = ms_since(t_fe);
    free_recv();
    if (rc) res_free(h);
    else if (h_out) *h_out = h;
    return rc;
}

// devs[s]: the device of shard s (distinct devices; loopback: several shards
// on one device, their partitions moved by device copies -- the N-owner
// orchestration without RCCL, libgocask_diag.so's test entry).
int replay_multi(const Src *files, uint32_t nfiles, const std::vector<int> &devs, const gck_opts *opts,
                 gck_result *out, bool loopback) {
    const uint32_t ndev = (uint32_t)devs.size();
    if ((nfiles && !files) || ndev == 0 || ndev > 64) return GCK_EINVAL;
    for (uint32_t f = 0; f < nfiles; ++f)
        if (files[f].len && !files[f].data && !files[f].path) return GCK_EINVAL;
    const bool want_keys = opts && (opts->flags & GCK_OPT_KEYS);
    if (!loopback) {
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
    // GCK_REPLAY_TRACE=1: the phases' wall times on stderr
    const bool trace = getenv("GCK_REPLAY_TRACE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    auto mark = [&](const char *what) {
        if (trace)
            fprintf(stderr, "gck_replay_multi %-14s %9.2f ms\n", what,
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    };
    // RCCL carries the pairs whose source and owner devices differ; a pair on
    // one device is a device copy (GCK_MULTI_RCCL_SELF=1: RCCL's self send /
    // receive instead, so a one-device box exercises the library's RCCL path).
    // The communicators come up on their own thread while the shards replay.
    const bool rccl_self = !loopback && getenv("GCK_MULTI_RCCL_SELF") != nullptr;
    const bool need_rccl = !loopback && (ndev > 1 || rccl_self);
    CommSet cset;
    int comm_rc = GCK_OK;
    std::thread comm_th;
    if (need_rccl) comm_th = std::thread([&]() { comm_rc = comms_for(devs, cset); });
    auto join_comm = [&]() {
        if (comm_th.joinable()) comm_th.join();
    };
    std::vector<ShardRun> sr(ndev);
    std::vector<gck_ctx *> mctx(ndev, nullptr);      // per owner: the merge context (pooled)
    std::vector<gck_opts> dopt(ndev);
    for (uint32_t s = 0; s < ndev; ++s) {
        if (opts) dopt[s] = *opts;
        else memset(&dopt[s], 0, sizeof(gck_opts));
        dopt[s].device = devs[s];
        dopt[s].flags &= ~GCK_OPT_KEYS;
    }
    // shards sharing a device (loopback) split its budget: each one sizing
    // its ring from the same free memory and pool would overstate it k times
    if (loopback && !(opts && opts->max_resident)) {
        for (uint32_t s = 0; s < ndev; ++s) {
            const uint64_t k = (uint64_t)std::count(devs.begin(), devs.end(), devs[s]);
            uint64_t b = 0;
            if ((rc = auto_budget(&dopt[s], &b))) return rc;
            dopt[s].max_resident = std::max<uint64_t>(1, b / k);
        }
    }
    auto cleanup = [&]() {
        join_comm();
        for (uint32_t s = 0; s < ndev; ++s) {
            (void)hipSetDevice(devs[s]);
            if (mctx[s]) (void)hipStreamSynchronize(mctx[s]->c.stream);
            for (auto &p : sr[s].parts)
                for (void *q : {p.d_ents, p.d_keys})
                    if (q) (void)hipFree(q);
            if (mctx[s]) pool_give(&dopt[s], mctx[s]);
        }
    };
    // 1. every shard on its device, a host thread each: its files stream
    // through gck_replay's ring of contexts (H2D of later groups overlapping
    // the replay of earlier ones, bounded by max_resident), and each group's
    // keydir is packed as soon as the group has replayed
    auto replay_shard = [&](uint32_t s) {
        ShardRun &x = sr[s];
        x.shard = s;
        x.a = ranges[2 * s];
        x.b = ranges[2 * s + 1];
        x.nown = ndev;
        x.dev = devs[s];
        if (x.b > x.a) {
            x.rc = replay_groups_to(files + x.a, x.b - x.a, &dopt[s], &x, &x.res);
            if (x.rc == GCK_EUNEXPECTED_EOF) x.rc = GCK_OK;  // the run's outcome is in res
        }
        if (!x.rc) x.rc = pool_take(&dopt[s], &mctx[s]);  // the owner's merge context
    };
    {
        std::vector<std::thread> th;
        for (uint32_t s = 1; s < ndev; ++s) th.emplace_back(replay_shard, s);
        replay_shard(0);
        for (auto &t : th) t.join();
    }
    mark("replayed");
    for (uint32_t s = 0; s < ndev; ++s)
        if (sr[s].rc) {
            rc = sr[s].rc;
            cleanup();
            return rc;
        }
    // 2. the global outcome
    std::vector<MultiOutcome> oc(ndev);
    for (uint32_t s = 0; s < ndev; ++s) {
        const gck_result &r = sr[s].res;
        oc[s] = MultiOutcome{r.status, sr[s].b - sr[s].a, r.err_file, r.files_walked, r.final_last_offset, r.err_off,
                             r.n_crc_fail};
    }
    std::vector<uint8_t> contrib(ndev, 0);
    multi_resolve(oc.data(), ndev, nfiles, out, contrib.data());
    uint32_t ng = 0, nr = 0;
    for (uint32_t s = 0; s < ndev; ++s) {
        ng += sr[s].res.n_groups;
        nr += sr[s].res.n_resident;
    }
    out->n_groups = ng;
    out->n_resident = nr;
    // 3.-5. the sources in walk order (every packed group of the contributing
    // shards; a failing shard's groups end with the one that failed), the
    // exchange, the per-owner merges, the live entries
    std::vector<SrcRef> srcs;
    for (uint32_t s = 0; s < ndev; ++s)
        if (contrib[s])
            for (const Part &p : sr[s].parts) srcs.push_back(SrcRef{s, &p});
    join_comm();
    mark("comms");
    if (need_rccl) rc = comm_rc;
    gck_rec *h = nullptr;
    uint64_t tot = 0;
    if (!rc) rc = exchange_merge(srcs, devs, mctx, need_rccl, rccl_self, cset, want_keys, trace, &h, &tot, out, nullptr);
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

// gck_ctx_multi_keydir: steps 1 (keydir + pack per shard, a host thread
// each), 2 (the global outcome) and 3-5 (exchange_merge) of a sharded replay
// over shards already resident and replayed in their own contexts; owner p's
// merge runs in ctxs[p].
int ctx_multi_keydir(gck_ctx *const *ctxs, uint32_t n, uint32_t flags, gck_result *out, double *ms) {
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
    std::vector<int> devs(n);
    for (uint32_t s = 0; s < n; ++s) devs[s] = ctxs[s]->c.device;
    std::vector<int> sorted = devs;
    std::sort(sorted.begin(), sorted.end());
    const bool loopback = std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end();
    const bool rccl_self = !loopback && getenv("GCK_MULTI_RCCL_SELF") != nullptr;
    const bool need_rccl = !loopback && (n > 1 || rccl_self);
    const bool trace = getenv("GCK_REPLAY_TRACE") != nullptr;
    CommSet cset;
    int comm_rc = GCK_OK;
    std::thread comm_th;
    if (need_rccl) comm_th = std::thread([&]() { comm_rc = comms_for(devs, cset); });
    std::vector<Part> parts(n);
    std::vector<int> prc(n, GCK_OK);
    std::vector<uint32_t> fbase(n + 1, 0);
    for (uint32_t s = 0; s < n; ++s) fbase[s + 1] = fbase[s] + ctxs[s]->c.nfiles;
    const auto t_loc = clk::now();
    auto local = [&](uint32_t s) {
        gck_ctx *ctx = ctxs[s];
        Part &p = parts[s];
        p.file0 = fbase[s];
        uint64_t nl = 0;
        int r = hipSetDevice(devs[s]) != hipSuccess ? GCK_EDEVICE : GCK_OK;
        if (r || (r = gck_ctx_keydir(ctx, GCK_KD_KEEP_TOMBSTONES, &nl, nullptr)) ||
            (r = gck_kd_pack_sizes(ctx, n, p.counts, p.kbytes))) {
            prc[s] = r;
            return;
        }
        uint64_t ne = 0, nk = 0;
        for (uint32_t o = 0; o < n; ++o) {
            ne += p.counts[o];
            nk += p.kbytes[o];
        }
        if (hipMalloc(&p.d_ents, ne * sizeof(gck_kd_entry) + 64) != hipSuccess ||
            hipMalloc(&p.d_keys, nk + 64) != hipSuccess) {
            (void)hipGetLastError();
            prc[s] = GCK_ENOMEM;
            return;
        }
        prc[s] = gck_kd_pack(ctx, s, p.file0, static_cast<gck_kd_entry *>(p.d_ents), ne,
                             static_cast<uint8_t *>(p.d_keys), nk);
        if (!prc[s] && hipStreamSynchronize(ctx->c.stream) != hipSuccess) prc[s] = GCK_EDEVICE;
    };
    {
        std::vector<std::thread> th;
        for (uint32_t s = 1; s < n; ++s) th.emplace_back(local, s);
        local(0);
        for (auto &t : th) t.join();
    }
    if (ms) ms[0] = ms_since(t_loc);
    int rc = GCK_OK;
    for (uint32_t s = 0; s < n && !rc; ++s) rc = prc[s];
    std::vector<MultiOutcome> oc(n);
    for (uint32_t s = 0; s < n; ++s) {
        const Ctx &c = ctxs[s]->c;
        oc[s] = MultiOutcome{c.status, c.nfiles, c.err_file, c.files_walked, c.final_last_offset, c.err_off,
                             c.n_crc_fail};
    }
    std::vector<uint8_t> contrib(n, 0);
    multi_resolve(oc.data(), n, fbase[n], out, contrib.data());
    std::vector<SrcRef> srcs;
    for (uint32_t s = 0; s < n; ++s)
        if (contrib[s]) srcs.push_back(SrcRef{s, &parts[s]});
    if (comm_th.joinable()) comm_th.join();
    if (!rc && need_rccl) rc = comm_rc;
    gck_rec *h = nullptr;
    uint64_t tot = 0;
    double ph[3] = {0, 0, 0};
    const std::vector<gck_ctx *> owners(ctxs, ctxs + n);
    if (!rc)
        rc = exchange_merge(srcs, devs, owners, need_rccl, rccl_self, cset, (flags & GCK_MULTI_KEYS) != 0, trace,
                            (flags & GCK_MULTI_FETCH) ? &h : nullptr, &tot, out, ph);
    if (ms) {
        ms[1] = ph[0];
        ms[2] = ph[1];
        ms[3] = ph[2];
    }
    for (uint32_t s = 0; s < n; ++s) {
        (void)hipSetDevice(devs[s]);
        for (void *q : {parts[s].d_ents, parts[s].d_keys})
            if (q) (void)hipFree(q);
    }
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

}  // namespace gck

extern "C" int gck_replay_multi(const gck_file *files, uint32_t nfiles, const int32_t *devices, uint32_t ndev,
                                const gck_opts *opts, gck_result *out) {
    if (!out) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    if (nfiles && !files) return GCK_EINVAL;
    if (!devices || ndev == 0 || ndev > 64) return GCK_EINVAL;
    const std::vector<Src> v = mem_srcs(files, nfiles);
    return replay_multi(v.data(), nfiles, std::vector<int>(devices, devices + ndev), opts, out, false);
}

extern "C" int gck_replay_multi_paths(const gck_path *files, uint32_t nfiles, const int32_t *devices, uint32_t ndev,
                                      const gck_opts *opts, gck_result *out) {
    if (!out) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    if (nfiles && !files) return GCK_EINVAL;
    if (!devices || ndev == 0 || ndev > 64) return GCK_EINVAL;
    std::vector<Src> v;
    int rc = open_srcs(files, nfiles, v);
    if (rc) return rc;
    rc = replay_multi(v.data(), nfiles, std::vector<int>(devices, devices + ndev), opts, out, false);
    close_srcs(v);
    return rc;
}

extern "C" int gck_ctx_multi_keydir(gck_ctx *const *ctxs, uint32_t n, uint32_t flags, gck_result *out, double *ms) {
    if (!out) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    if (!ctxs || n == 0 || n > 64) return GCK_EINVAL;
    for (uint32_t s = 0; s < n; ++s)
        if (!ctxs[s] || ctxs[s]->c.n_runs == 0) return GCK_EINVAL;  // every shard replayed first
    return gck::ctx_multi_keydir(ctxs, n, flags, out, ms);
}
