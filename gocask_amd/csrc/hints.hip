// hints.hip — hint-driven replay (the reference's roadmap
// item "merging and hint files", README.md:60).
//
// A database whose data files all have hint files (gck_ctx_compact's, format
// in include/gocask_hip.h GCK_HINT_*) gets its tuples from the hints alone:
// for each record, the gck_rec gck_ctx_run gives on the data files -- rec_off
// (the record's offset in its data file), file, key_len, value_pos
// (lastOffset + 16 + KeySize mod 2^32, core/keydir.go:25, with the lastOffset
// carried across files as core/db.go:110-140 does: reset after every file but
// the active one), value_size, crc, ts -- without reading a data-file byte, so
// without a CRC verdict (flags GCK_F_HINT, crc_calc 0).
//
// Layout: the hint files in the context's arena (gck_ctx_load).  Kernels:
//   k_hint_tails  a lane per file: its 32-byte tail (entries, entry bytes,
//                 data-file bytes, magic, version) -> the host checks the
//                 sizes, numbers the entries and blocks, carries lastOffset;
//   k_hint_parse  a lane per block of GCK_HINT_BLOCK entries: its index entry
//                 (hint and data-file offsets of the block's first entry),
//                 then the block's entries one after another (5 header words
//                 each), a tuple and a record-table row per entry; the block
//                 must end exactly where the next one starts (index) or at
//                 the file's entry bytes / data-file bytes (tail).
// The record table (d_rec_off = the entry's key - 16 in the arena, d_rec_kv =
// (KeySize, ValueSize)) is what gck_ctx_keydir and the key gather read, so the
// keydir (last entry per key across several merges' hints) and GCK_OPT_KEYS
// work on a hint replay as on a run.
#include "gck_internal.h"

#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

namespace gck {

constexpr uint64_t kHintHdrB = 20, kHintTailB = 32;

// little-endian u32 at any byte address (the arena is padded: the aligned
// dwords around it are readable)
__device__ __forceinline__ uint32_t ld4u(const uint8_t *p) {
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
    const uint32_t *a = reinterpret_cast<const uint32_t *>(p - sh);
    return __builtin_amdgcn_alignbyte(a[1], a[0], sh);
}
__device__ __forceinline__ uint64_t ld8u(const uint8_t *p) { return ld4u(p) | ((uint64_t)ld4u(p + 4) << 32); }

// Per file: tail words (entries, entry bytes, data-file bytes, magic | version
// << 32); a file shorter than a tail gets all zeros (refused by the host).
__global__ void k_hint_tails(const uint8_t *__restrict__ arena, const uint64_t *__restrict__ fbase,
                             const uint64_t *__restrict__ flen, uint32_t nf, uint64_t *__restrict__ tails) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nf) return;
    const uint64_t len = flen[f];
    uint64_t w[4] = {0, 0, 0, 0};
    if (len >= kHintTailB) {
        const uint8_t *t = arena + fbase[f] + len - kHintTailB;
#pragma unroll
        for (int k = 0; k < 4; ++k) w[k] = ld8u(t + 8 * k);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) tails[4 * f + k] = w[k];
}

// Per file, from the host: arena base, entry bytes, data-file bytes, first
// entry and first block (global numbering), entries, carried lastOffset.
struct HintFile {
    uint64_t base, ebytes, dbytes, ent0, blk0, n;
    uint32_t carry, pad;
};

__global__ __launch_bounds__(256) void k_hint_parse(const uint8_t *__restrict__ arena,
                                                    const HintFile *__restrict__ hf, uint32_t nf, uint64_t nblk,
                                                    gck_rec *__restrict__ out, uint64_t *__restrict__ rec_off,
                                                    uint2 *__restrict__ rec_kv, uint32_t *__restrict__ rec_file,
                                                    uint32_t *__restrict__ err) {
    const uint64_t b = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= nblk) return;
    // the file of block b: the last f with blk0 <= b (files without entries
    // have no blocks: blk0 of the next equals theirs)
    uint32_t lo = 0, hi = nf - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) / 2;
        if (hf[mid].blk0 <= b) lo = mid; else hi = mid - 1;
    }
    const HintFile F = hf[lo];
    const uint8_t *h = arena + F.base;
    const uint64_t lb = b - F.blk0, nb = (F.n + GCK_HINT_BLOCK - 1) / GCK_HINT_BLOCK;
    const uint8_t *ix = h + F.ebytes + 16 * lb;  // this block's index entry
    uint64_t hoff = ld8u(ix), doff = ld8u(ix + 8);
    const uint64_t end_h = lb + 1 < nb ? ld8u(ix + 16) : F.ebytes, end_d = lb + 1 < nb ? ld8u(ix + 24) : F.dbytes;
    const uint32_t cnt = (uint32_t)min<uint64_t>(GCK_HINT_BLOCK, F.n - GCK_HINT_BLOCK * lb);
    uint64_t e = F.ent0 + GCK_HINT_BLOCK * lb;
    bool bad = false;
    for (uint32_t j = 0; j < cnt; ++j, ++e) {
        if (hoff + kHintHdrB > F.ebytes) {  // (a read past the entries is never issued)
            bad = true;
            break;
        }
        const uint8_t *p = h + hoff;
        const uint32_t ts = ld4u(p), ks = ld4u(p + 4), vs = ld4u(p + 8), vpos = ld4u(p + 12), crc = ld4u(p + 16);
        // a merged file holds Puts only (KeySize >= 1); ValuePos is the value's
        // offset in the data file mod 2^32 -- the data offset the entries add up to
        if (ks == 0 || hoff + kHintHdrB + ks > F.ebytes || vpos != (uint32_t)(doff + 16 + ks)) {
            bad = true;
            break;
        }
        gck_rec r;
        r.rec_off = doff;
        r.file = lo;
        r.key_len = ks;
        r.value_pos = F.carry + vpos;
        r.value_size = vs;
        r.crc = crc;
        r.ts = ts;
        r.flags = GCK_F_HINT;
        r.crc_calc = 0;
        out[e] = r;
        rec_off[e] = F.base + hoff + (kHintHdrB - 16);  // so the key is at rec_off + 16, as for a record
        rec_kv[e] = make_uint2(ks, vs);
        rec_file[e] = lo;
        hoff += kHintHdrB + ks;
        doff += 16ull + ks + vs;
    }
    if (bad || hoff != end_h || doff != end_d) atomicOr(err, 1u);
}

// GCK_OPT_LIVE with GCK_OPT_KEYS: the record-table rows of the live entries
// (their record indices idx, walk order), for the key gather
__global__ void k_hint_live_rows(const uint32_t *__restrict__ idx, uint64_t n, const uint64_t *__restrict__ rec_off,
                                 const uint2 *__restrict__ rec_kv, uint64_t *__restrict__ ro, uint2 *__restrict__ kv) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    ro[i] = rec_off[idx[i]];
    kv[i] = rec_kv[idx[i]];
}

// gck_replay_hints on a pooled context: load, parse, then (GCK_OPT_LIVE) the
// keydir's entries as the tuples, (GCK_OPT_KEYS) their keys, and the fetch
static int replay_hints_on(gck_ctx *ctx, const gck_file *files, uint32_t nfiles, uint32_t fl, gck_result *out) {
    int rc;
    if ((rc = gck_ctx_load(ctx, files, nfiles)) || (rc = gck_ctx_replay_hints(ctx, nullptr))) return rc;
    Ctx *c = &ctx->c;
    if (fl & GCK_OPT_LIVE) {
        uint64_t nl = 0;
        if ((rc = gck_ctx_keydir(ctx, 0, &nl, nullptr))) return rc;
        GCK_HIP(hipSetDevice(c->device));
        if (nl) {  // the live entries become the tuples
            GCK_HIP(hipMemcpyAsync(c->d_out.p, c->d_kdout.p, nl * sizeof(gck_rec), hipMemcpyDeviceToDevice, c->stream));
            if (fl & GCK_OPT_KEYS) {  // their record-table rows, in their order
                if ((rc = c->d_live.ensure(nl * 16))) return rc;
                uint64_t *ro = c->d_live.as<uint64_t>();  // (scratch: the keydir's live flags are spent)
                k_hint_live_rows<<<(uint32_t)((nl + 255) / 256), 256, 0, c->stream>>>(
                    c->d_kdidx.as<uint32_t>(), nl, c->d_rec_off.as<uint64_t>(), c->d_rec_kv.as<uint2>(), ro,
                    reinterpret_cast<uint2 *>(ro + nl));
                GCK_HIP(hipMemcpyAsync(c->d_rec_off.p, ro, nl * 8, hipMemcpyDeviceToDevice, c->stream));
                GCK_HIP(hipMemcpyAsync(c->d_rec_kv.p, ro + nl, nl * 8, hipMemcpyDeviceToDevice, c->stream));
            }
        }
        c->n_recs = nl;
        c->kd_valid = false;  // the record table now holds the live entries only
        c->n_live = 0;
    }
    void *kh = nullptr;
    uint64_t kl = 0;
    if ((fl & GCK_OPT_KEYS) && (rc = ctx_gather_keys(c, &kh, &kl))) {
        if (kh) (void)hipHostFree(kh);
        return rc;
    }
    if ((rc = gck_ctx_fetch(ctx, out)) == GCK_OK && (fl & GCK_OPT_KEYS)) {
        // into a result array (gck_result_free's kind; the gather's pinned
        // buffer is the library's)
        if (hipStreamSynchronize(c->stream) != hipSuccess) rc = GCK_EDEVICE;
        else if (!(out->keys = static_cast<uint8_t *>(res_alloc(kl, false)))) rc = GCK_ENOMEM;
        else {
            par_gather(out->keys, {{kh, kl}});
            out->keys_len = kl;
        }
    }
    if (kh) (void)hipHostFree(kh);
    out->n_groups = 1;
    out->n_resident = 1;
    return rc;
}

}  // namespace gck

using namespace gck;

extern "C" {

int gck_ctx_replay_hints(gck_ctx *ctx, double *ms) {
    if (!ctx) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    const auto t0 = std::chrono::steady_clock::now();
    if (ms) *ms = 0;
    c->n_live = 0;  // the keydir (and its pack) belong to the previous tuples
    c->kd_nparts = 0;
    c->kd_valid = false;
    c->kd_hashed = false;
    c->kd_inserted = false;
    c->from_hints = true;
    c->n_recs = 0;
    const uint32_t nf = c->nfiles;
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    hipEvent_t a, b;
    GCK_HIP(hipEventCreate(&a));
    GCK_HIP(hipEventCreate(&b));
    struct EvGuard {
        hipEvent_t a, b;
        ~EvGuard() {
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
        }
    } guard{a, b};
    GCK_HIP(hipEventRecord(a, s));
    // 1. the tails: entries, blocks and carried lastOffset per file
    std::vector<uint64_t> tl(4ull * nf + 4, 0);
    int rc;
    if ((rc = c->d_cfoot.ensure((4ull * nf + 4) * 8))) return rc;  // (scratch: the compaction's footer table)
    if (nf) {
        k_hint_tails<<<(nf + 255) / 256, 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(),
                                                      c->d_flen.as<uint64_t>(), nf, c->d_cfoot.as<uint64_t>());
        GCK_HIP(hipMemcpyAsync(tl.data(), c->d_cfoot.p, 4ull * nf * 8, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipStreamSynchronize(s));
    }
    std::vector<HintFile> hf(nf);
    uint64_t ents = 0, blks = 0;
    uint32_t last = 0;  // keyDir.lastOffset at the start of each file (core/db.go:110-140)
    for (uint32_t f = 0; f < nf; ++f) {
        const uint64_t n = tl[4 * f], eb = tl[4 * f + 1], db = tl[4 * f + 2], mv = tl[4 * f + 3];
        const uint64_t nb = (n + GCK_HINT_BLOCK - 1) / GCK_HINT_BLOCK;
        // the tail must describe this file exactly (sizes checked before any
        // entry is read: every read below stays inside the file)
        if ((uint32_t)mv != GCK_HINT_MAGIC || (uint32_t)(mv >> 32) != GCK_HINT_VERSION || n > (1ull << 40) ||
            eb > c->f_len[f] || eb < (kHintHdrB + 1) * n || c->f_len[f] != eb + 16 * nb + kHintTailB)
            return GCK_EINVAL;
        hf[f] = HintFile{c->f_base[f], eb, db, ents, blks, n, last, 0};
        ents += n;
        blks += nb;
        last += (uint32_t)db;
        if (c->f_reset[f]) last = 0;  // resetOffset (core/db.go:117-119)
    }
    if (ents > 0xFFFFFFF0ull) return GCK_EINVAL;
    if ((rc = c->d_rec_off.ensure(std::max<uint64_t>(ents, 1) * 8)) ||
        (rc = c->d_rec_kv.ensure(std::max<uint64_t>(ents, 1) * 8)) ||
        (rc = c->d_rec_file.ensure(std::max<uint64_t>(ents, 1) * 4)) ||
        (rc = c->d_out.ensure(std::max<uint64_t>(ents, 1) * sizeof(gck_rec))) ||
        (rc = c->d_cpos.ensure(std::max<uint32_t>(nf, 1) * sizeof(HintFile))) || (rc = c->d_counters.ensure(64)))
        return rc;
    uint32_t *err = c->d_counters.as<uint32_t>();
    GCK_HIP(hipMemsetAsync(err, 0, 4, s));
    if (blks) {
        GCK_HIP(hipMemcpyAsync(c->d_cpos.p, hf.data(), nf * sizeof(HintFile), hipMemcpyHostToDevice, s));
        k_hint_parse<<<(uint32_t)((blks + 255) / 256), 256, 0, s>>>(
            c->arena.as<uint8_t>(), c->d_cpos.as<HintFile>(), nf, blks, c->d_out.as<gck_rec>(),
            c->d_rec_off.as<uint64_t>(), c->d_rec_kv.as<uint2>(), c->d_rec_file.as<uint32_t>(), err);
    }
    GCK_HIP(hipEventRecord(b, s));
    uint32_t e = 0;
    GCK_HIP(hipMemcpyAsync(&e, err, 4, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    GCK_HIP(hipGetLastError());
    if (e) return GCK_EINVAL;
    float t = 0;
    (void)hipEventElapsedTime(&t, a, b);
    if (ms) *ms = t;
    c->n_recs = ents;
    c->status = GCK_OK;
    c->err_file = 0;
    c->err_off = 0;
    c->files_walked = nf;
    c->final_last_offset = last;
    c->n_crc_fail = 0;
    c->n_fixups = 0;
    c->n_overflow = 0;
    c->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return GCK_OK;
}

int gck_replay_hints(const gck_file *files, uint32_t nfiles, const gck_opts *opts, gck_result *out) {
    if (!out || (nfiles && !files)) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    gck_ctx *ctx = nullptr;
    int rc = pool_take(opts, &ctx);
    if (rc) return rc;
    rc = replay_hints_on(ctx, files, nfiles, opts ? opts->flags : 0u, out);
    if (rc) gck_result_free(out);
    pool_give(opts, ctx);
    return rc;
}

}  // extern "C"
