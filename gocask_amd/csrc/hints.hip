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
//   k_hint_parse  a wavefront per segment of 64 blocks of GCK_HINT_BLOCK
//                 entries, copied into LDS; a lane per block: its index entry
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

constexpr uint64_t kHintHdrB = 20, kHintTailB = 32, kHintIdxB = 24;  // entry header, tail, index entry

typedef uint32_t u32x4h __attribute__((ext_vector_type(4), aligned(4)));

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
    uint64_t base, ebytes, dbytes, ent0, blk0, n, seg0;
    uint32_t carry, pad;
};

// One block of GCK_HINT_BLOCK entries of file lo (F), block lb: its entries
// one after another from (hoff, doff) -- the index entry -- to (end_h,
// end_d), each checked (bounds, KeySize >= 1, ValuePos = the data offset the
// entries add up to), a tuple and a record-table row each.  rd(o, k): the
// little-endian u32 at entry byte o + k (global memory, or the LDS copy of a
// segment).  False: malformed.
// The tuple and record-table row of the entry at hint offset hoff, data
// offset doff, with its five header words.
__device__ __forceinline__ void put_entry(const HintFile &F, uint32_t lo, uint64_t e, uint64_t hoff, uint64_t doff,
                                          uint32_t ts, uint32_t ks, uint32_t vs, uint32_t vpos, uint32_t crc,
                                          gck_rec *__restrict__ out, uint64_t *__restrict__ rec_off,
                                          uint2 *__restrict__ rec_kv, uint32_t *__restrict__ rec_file) {
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
}

// want: the block's integrity word from its index entry, the XOR of its
// entries' hint_entry_check (a changed key, timestamp, size or CRC byte in a
// well-formed entry fails it)
template <class Rd, class Emit>
__device__ __forceinline__ bool parse_block(const HintFile &F, uint64_t lb, uint64_t hoff, uint64_t doff,
                                            uint64_t end_h, uint64_t end_d, Rd rd, Emit emit, uint64_t want) {
    uint64_t chk = 0;
    const uint32_t cnt = (uint32_t)min<uint64_t>(GCK_HINT_BLOCK, F.n - GCK_HINT_BLOCK * lb);
    for (uint32_t j = 0; j < cnt; ++j) {
        if (hoff + kHintHdrB > F.ebytes) return false;  // (a read past the entries is never issued)
        const uint32_t ks = rd(hoff, 4), vs = rd(hoff, 8), vpos = rd(hoff, 12);
        // a merged file holds Puts only (KeySize >= 1); ValuePos is the value's
        // offset in the data file mod 2^32 -- the data offset the entries add up to
        if (ks == 0 || hoff + kHintHdrB + ks > F.ebytes || vpos != (uint32_t)(doff + 16 + ks)) return false;
        chk ^= hint_entry_check(rd(hoff, 0), ks, vs, vpos, rd(hoff, 16), [&](uint32_t q) {
            const uint32_t v = rd(hoff, (uint32_t)kHintHdrB + 4 * q), left = ks - 4 * q;
            return left >= 4 ? v : v & ((1u << (8 * left)) - 1u);
        });
        emit(j, hoff, doff, ks, vs, vpos);
        hoff += kHintHdrB + ks;
        doff += 16ull + ks + vs;
    }
    return hoff == end_h && doff == end_d && chk == want;
}

// k_hint_parse: a wavefront per segment of kHintSeg blocks of one file.  The
// segment's entry bytes are contiguous in the hint file: the wavefront copies
// them into LDS with coalesced 16-byte loads, then lane j walks block j from
// LDS -- the chain from one entry to the next (its KeySize) is an LDS round
// trip instead of a memory one.  A segment larger than the LDS copy (long
// keys) is walked from global memory as before.  (A lane per block reading
// global memory: C3's merge 0.57 ms, profiles/r5i.)
// Entries' offsets are kept in LDS by the walk, and the tuples leave in a
// second pass, a lane per entry (consecutive lanes, consecutive tuples:
// whole lines per store instead of 64 lanes writing 64 lines 640 B apart).
constexpr uint32_t kHintSeg = 64, kHintSegBytes = 40 * 1024, kHintSegEnts = kHintSeg * GCK_HINT_BLOCK;
__global__ __launch_bounds__(64) void k_hint_parse(const uint8_t *__restrict__ arena,
                                                   const HintFile *__restrict__ hf, uint32_t nf, uint64_t nseg,
                                                   gck_rec *__restrict__ out, uint64_t *__restrict__ rec_off,
                                                   uint2 *__restrict__ rec_kv, uint32_t *__restrict__ rec_file,
                                                   uint32_t *__restrict__ err) {
    __shared__ uint32_t L[kHintSegBytes / 4];
    __shared__ uint32_t Eq[kHintSegEnts];  // entry's offset in L (bytes)
    __shared__ uint64_t Ed[kHintSegEnts];  // entry's data-file offset
    const uint64_t sg = blockIdx.x;
    if (sg >= nseg) return;
    const uint32_t lane = threadIdx.x;
    // the file of segment sg: the last f with seg0 <= sg
    uint32_t lo = 0, hi = nf - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) / 2;
        if (hf[mid].seg0 <= sg) lo = mid; else hi = mid - 1;
    }
    const HintFile F = hf[lo];
    const uint8_t *h = arena + F.base;
    const uint64_t nb = (F.n + GCK_HINT_BLOCK - 1) / GCK_HINT_BLOCK;
    const uint64_t lb0 = (sg - F.seg0) * kHintSeg, nbs = min<uint64_t>(kHintSeg, nb - lb0);
    const uint64_t lb = lb0 + lane;
    const bool act = lane < nbs;
    // this block's index entry and where it must end: the next block's entry
    // (the lane above), or past the segment the next segment's first / the tail
    const uint8_t *ix = h + F.ebytes + kHintIdxB * (act ? lb : lb0);
    const uint64_t hoff = ld8u(ix), doff = ld8u(ix + 8), want = ld8u(ix + 16);
    uint64_t end_h = __shfl_down(hoff, 1), end_d = __shfl_down(doff, 1);
    if (lane == nbs - 1) {
        end_h = lb + 1 < nb ? ld8u(ix + kHintIdxB) : F.ebytes;
        end_d = lb + 1 < nb ? ld8u(ix + kHintIdxB + 8) : F.dbytes;
    }
    // the segment's entry bytes [h0, h1) (index values checked before use)
    const uint64_t h0 = __shfl(hoff, 0), h1 = __shfl(end_h, (int)(nbs - 1));
    const uint64_t a0 = h0 & ~3ull;
    bool ok = h0 <= h1 && h1 <= F.ebytes;
    if (__ballot(act && !ok)) {
        if (lane == 0) atomicOr(err, 1u);
        return;
    }
    if (h1 - a0 + 4 <= kHintSegBytes) {
        // copy [a0, h1 + 4) as dwords, 16 bytes per lane per step (the arena is
        // padded past every file; the u32 reads below need the dword after)
        const uint32_t nw = (uint32_t)((h1 + 4 - a0 + 3) / 4);
        for (uint32_t w = 4 * lane; w < nw; w += 256) {
            const u32x4h v = *reinterpret_cast<const u32x4h *>(h + a0 + 4ull * w);
            L[w] = v.x;
            if (w + 1 < kHintSegBytes / 4) L[w + 1] = v.y;
            if (w + 2 < kHintSegBytes / 4) L[w + 2] = v.z;
            if (w + 3 < kHintSegBytes / 4) L[w + 3] = v.w;
        }
        __syncthreads();
        // (a block reading past the copy is malformed -- it cannot end at its
        // index's end -- so such reads are only kept inside the array)
        auto rd = [&](uint64_t o, uint32_t k) {
            const uint32_t q = (uint32_t)(o + k - a0), sh = q & 3u, i = min(q >> 2, kHintSegBytes / 4 - 2);
            return __builtin_amdgcn_alignbyte(L[i + 1], L[i], sh);
        };
        const uint32_t eb = lane * GCK_HINT_BLOCK;  // this block's first entry in the segment
        if (act)
            ok = parse_block(F, lb, hoff, doff, end_h, end_d, rd,
                             [&](uint32_t j, uint64_t ho, uint64_t dof, uint32_t, uint32_t, uint32_t) {
                                 Eq[eb + j] = (uint32_t)(ho - a0);
                                 Ed[eb + j] = dof;
                             }, want);
        if (__ballot(act && !ok)) {
            if (lane == 0) atomicOr(err, 1u);
            return;
        }
        __syncthreads();
        const uint64_t e0 = F.ent0 + GCK_HINT_BLOCK * lb0, ne = min<uint64_t>(kHintSegEnts, F.n - GCK_HINT_BLOCK * lb0);
        for (uint32_t i = lane; i < ne; i += 64) {
            const uint32_t q = Eq[i];
            const uint64_t ho = a0 + q;
            put_entry(F, lo, e0 + i, ho, Ed[i], rd(ho, 0), rd(ho, 4), rd(ho, 8), rd(ho, 12), rd(ho, 16), out, rec_off,
                      rec_kv, rec_file);
        }
        return;
    } else {
        auto rd = [&](uint64_t o, uint32_t k) { return ld4u(h + o + k); };
        const uint64_t e0 = F.ent0 + GCK_HINT_BLOCK * lb;
        if (act)
            ok = parse_block(F, lb, hoff, doff, end_h, end_d, rd,
                             [&](uint32_t j, uint64_t ho, uint64_t dof, uint32_t ks, uint32_t vs, uint32_t vpos) {
                                 put_entry(F, lo, e0 + j, ho, dof, rd(ho, 0), ks, vs, vpos, rd(ho, 16), out, rec_off,
                                           rec_kv, rec_file);
                             }, want);
    }
    if (act && !ok) atomicOr(err, 1u);
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
    uint64_t ents = 0, blks = 0, segs = 0;
    uint32_t last = 0;  // keyDir.lastOffset at the start of each file (core/db.go:110-140)
    for (uint32_t f = 0; f < nf; ++f) {
        const uint64_t n = tl[4 * f], eb = tl[4 * f + 1], db = tl[4 * f + 2], mv = tl[4 * f + 3];
        const uint64_t nb = (n + GCK_HINT_BLOCK - 1) / GCK_HINT_BLOCK;
        // the tail must describe this file exactly (sizes checked before any
        // entry is read: every read below stays inside the file)
        // (a file without entries has no data bytes either: nothing would
        // check them, yet they would feed the carried lastOffset)
        if ((uint32_t)mv != GCK_HINT_MAGIC || (uint32_t)(mv >> 32) != GCK_HINT_VERSION || n > (1ull << 40) ||
            eb > c->f_len[f] || eb < (kHintHdrB + 1) * n || c->f_len[f] != eb + kHintIdxB * nb + kHintTailB ||
            (n == 0 && db != 0))
            return GCK_EINVAL;
        hf[f] = HintFile{c->f_base[f], eb, db, ents, blks, n, segs, last, 0};
        ents += n;
        blks += nb;
        segs += (nb + kHintSeg - 1) / kHintSeg;
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
        k_hint_parse<<<(uint32_t)segs, 64, 0, s>>>(
            c->arena.as<uint8_t>(), c->d_cpos.as<HintFile>(), nf, segs, c->d_out.as<gck_rec>(),
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
