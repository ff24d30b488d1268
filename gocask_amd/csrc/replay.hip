// replay.hip — MI355X (gfx950) cold-start replay of GoCask data files.
//
// Replaces (*DB).init / walkFile / readEntry (core/db.go:110-178) and the keydir
// offset arithmetic (core/keydir.go:22-53), and applies the lazy CRC rule of
// (*DB).get (core/db.go:311) to every record.  Pipeline:
//
//   k_spec_entry   one wavefront per 256 KiB chunk: first plausible record start
//   k_walk         one lane per chunk: speculative header chain, records staged
//   k_validate     chunk k's entry must equal chunk k-1's exit; k_fixup re-walks
//   k_scan_chunks  record slot per chunk (exclusive scan), per-file summary
//   (host)         EOF classification, lastOffset carries (core/db.go:117)
//   k_compact      record table (arena offset + header), walk order
//   k_row_index    first record touching each 4 KiB row
//   k_crc_rows     HBM-bound: every byte once, CRC partials of every value
//   k_finalize     CRC verdict, ValuePos (u32 wrap), gck_rec tuples
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>

#include "gck_internal.h"

namespace gck {

static thread_local std::string g_err;
void set_error(const char *what, hipError_t e, const char *file, int line) {
    char buf[512];
    snprintf(buf, sizeof buf, "%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
    g_err = buf;
}
const char *last_error() { return g_err.c_str(); }

enum : uint32_t { T_NONE = 0, T_SILENT = 1, T_ERR = 2 };
constexpr int kHops = 4;          // extra headers a speculative start must chain through
constexpr int kWaves = 16;        // wavefronts per k_crc_rows workgroup
#ifndef GCK_DEPTH
#define GCK_DEPTH 1
#endif
constexpr int kDepth = GCK_DEPTH;  // steps in flight per k_crc_rows wavefront
#ifndef GCK_NR
#define GCK_NR 2
#endif
constexpr int kRowsPerStep = GCK_NR;  // rows a k_crc_rows wavefront processes at once
constexpr uint32_t kNibBase = 32768;

// ---------------------------------------------------------------- helpers ---
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Raw buffer resource over [p, p + bytes) (gfx9 dword3: untyped, bounds-checked).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, (int)bytes, 0x00020000);
}

__device__ __forceinline__ uint32_t ab(uint32_t hi, uint32_t lo, uint32_t sh) {
    return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

struct Hdr {
    uint32_t crc, ts, ks, vs;
};

// 16-byte little-endian header at any byte offset (core/header.go:58-62).  The
// arena is 4 KiB aligned and padded, so the 5-dword over-read stays in bounds.
__device__ __forceinline__ Hdr ld_hdr(const uint8_t *__restrict__ arena, uint64_t o) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(arena + (o & ~3ull));
    const uint32_t sh = (uint32_t)o & 3u;
    const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3], w4 = w[4];
    Hdr h;
    h.crc = ab(w1, w0, sh);
    h.ts = ab(w2, w1, sh);
    h.ks = ab(w3, w2, sh);
    h.vs = ab(w4, w3, sh);
    return h;
}

// Follow the header chain from q for kHops+1 headers: key length in
// [1, max_key] and every record inside the file.  A chain may only end exactly
// at the file end.  (A record straddling the file end is rejected: that only
// costs a fixup for the one chunk where it is real.)
__device__ bool chain_ok(const uint8_t *__restrict__ arena, uint64_t base, uint64_t len, uint64_t q,
                         uint32_t max_key) {
    for (int h = 0; h <= kHops; ++h) {
        if (q == len) return h > 0;
        if (q + 16 > len) return false;
        const Hdr hd = ld_hdr(arena, base + q);
        const uint32_t klen = hd.ks ? hd.ks : hd.vs;
        if (klen == 0 || klen > max_key) return false;
        const uint64_t end = q + 16 + (uint64_t)hd.ks + hd.vs;
        if (end > len) return false;
        q = end;
    }
    return true;
}

// The reference's readEntry loop (core/db.go:131-178) over one chunk: decode
// headers from p while p < ce.  EOF classes follow Go's io.ReadFull /
// bufio.Reader.Discard semantics.  emit(i, p, hdr) per record.
template <class Emit>
__device__ void walk_chain(const uint8_t *__restrict__ arena, uint64_t base, uint64_t len, uint64_t ce,
                           uint64_t p, Emit emit, uint32_t &count, uint64_t &exit, uint32_t &term,
                           uint64_t &tpos) {
    uint32_t n = 0;
    term = T_NONE;
    tpos = 0;
    while (p < ce) {
        const uint64_t rem = len - p;
        if (rem < 16) { term = T_ERR; tpos = p; break; }            // ErrUnexpectedEOF
        const Hdr h = ld_hdr(arena, base + p);
        const uint32_t klen = h.ks ? h.ks : h.vs;                    // db.go:151-155
        const uint64_t rem2 = rem - 16;
        if (klen > 0 && rem2 == 0) { term = T_SILENT; tpos = p; break; }  // ReadFull io.EOF
        if (rem2 < klen) { term = T_ERR; tpos = p; break; }          // partial key
        uint64_t next;
        if (h.ks == 0) {
            next = p + 16 + klen;                                    // tombstone
        } else {
            if (rem2 - klen < h.vs) { term = T_SILENT; tpos = p; break; }  // Discard io.EOF
            next = p + 16 + (uint64_t)h.ks + h.vs;
        }
        emit(n, p, h);
        ++n;
        p = next;
    }
    count = n;
    exit = p;
}

// ------------------------------------------------------------------ kernels ---
// Bit 7 of each byte of the result is set iff that byte of w is zero (exact).
__device__ __forceinline__ uint32_t zero_bytes(uint32_t w) {
    return ~(((w & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | w | 0x7F7F7F7Fu);
}

// One wavefront per chunk finds the first byte position >= chunk start whose
// header and the next kHops headers are plausible (chunk 0 of a file starts at
// 0).  Each pass covers 4 KiB of positions, 64 per lane.  Prefilter: a header
// at p with KeySize <= 65535 (tombstones: KeySize 0) has bytes p+10 and p+11
// zero, so the lane flags positions whose bytes 10, 11 are a zero pair (about
// 2 VALU per position; in value bytes a zero pair is rare) and only flagged
// positions get the full chain test.  A hit at p is replaced by p+1 when p+1
// chains too: every true header has a plausible "shadow" one byte earlier
// (Timestamp's top byte + KeySize<<8, ValueSize<<8).  Keys longer than 65535
// bytes are never speculated here; validation finds their chunks and re-walks.
__global__ __launch_bounds__(256) void k_spec_entry(const uint8_t *__restrict__ arena,
                                                    const uint64_t *__restrict__ fbase,
                                                    const uint64_t *__restrict__ flen,
                                                    const uint32_t *__restrict__ ch_file,
                                                    const uint64_t *__restrict__ ch_start,
                                                    const uint64_t *__restrict__ ch_end,
                                                    uint64_t *__restrict__ ch_entry, uint32_t n_chunks,
                                                    uint32_t max_key) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + (threadIdx.x >> 6));  // wave-uniform
    if (c >= n_chunks) return;
    const uint32_t f = ch_file[c];
    const uint64_t cs = ch_start[c], ce = ch_end[c], base = fbase[f], len = flen[f];
    const uint32_t mk = min(max_key, 65535u);
    uint64_t found = kNone;
    if (cs == 0) {
        found = 0;
    } else {
        // The scan loop only computes candidate masks (no dependent loads in
        // it, so the next windows' loads stay in flight: windows A/B/C rotate,
        // unrolled so none is copied); a window with candidates leaves the
        // loop for the chain tests and the scan resumes after it if none holds.
        auto load = [&](uint64_t b0, u32x4 (&v)[5]) {
            // bytes [p0, p0+80): the 64 positions plus their header bytes (the
            // arena is padded 3 windows past every file).  Buffer loads: the
            // compiler keeps them where they are issued (ahead of their use).
            const __amdgpu_buffer_rsrc_t rw = make_rsrc(arena + base + b0, 4096 + 80);
#pragma unroll
            for (int k = 0; k < 5; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rw, lane * 64 + 16 * k, 0, 0);
        };
        auto cands = [&](const u32x4 (&v)[5]) -> uint64_t {  // bit t: bytes p0+t+10, p0+t+11 both zero
            uint32_t w[20];
#pragma unroll
            for (int k = 0; k < 5; ++k) {
                w[4 * k] = v[k].x;
                w[4 * k + 1] = v[k].y;
                w[4 * k + 2] = v[k].z;
                w[4 * k + 3] = v[k].w;
            }
            uint32_t zf[20];
#pragma unroll
            for (int k = 2; k < 20; ++k) zf[k] = zero_bytes(w[k]);
            uint64_t cm = 0;
#pragma unroll
            for (int k = 2; k <= 18; ++k) {
                const uint32_t pr = zf[k] & ((zf[k] >> 8) | (zf[k + 1] << 24));
                const uint32_t nib = ((pr >> 7) & 1u) | ((pr >> 14) & 2u) | ((pr >> 21) & 4u) | ((pr >> 28) & 8u);
                const int t0 = 4 * k - 10;
                cm |= t0 >= 0 ? (uint64_t)nib << t0 : (uint64_t)(nib >> -t0);
            }
            return cm;
        };
        uint64_t from = cs;
        while (found == kNone && from < ce) {
            uint64_t wb = kNone, cm = 0;
            {
                u32x4 A[5], B[5], C[5];
                load(from, A);
                load(from + 4096, B);
                for (uint64_t b0 = from;; b0 += 3 * 4096) {
                    load(b0 + 2 * 4096, C);
                    cm = cands(A);
                    if (__ballot(cm != 0)) { wb = b0; break; }
                    if (b0 + 4096 >= ce) break;
                    load(b0 + 3 * 4096, A);
                    cm = cands(B);
                    if (__ballot(cm != 0)) { wb = b0 + 4096; break; }
                    if (b0 + 2 * 4096 >= ce) break;
                    load(b0 + 4 * 4096, B);
                    cm = cands(C);
                    if (__ballot(cm != 0)) { wb = b0 + 2 * 4096; break; }
                    if (b0 + 3 * 4096 >= ce) break;
                }
            }
            if (wb == kNone) break;
            uint64_t lanes = __ballot(cm != 0);
            while (lanes && found == kNone) {
                const int l = __ffsll((long long)lanes) - 1;
                uint64_t lm = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(cm >> 32), l) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)cm, l);
                while (lm) {
                    const int t = __ffsll((long long)lm) - 1;
                    const uint64_t q = wb + 64ull * l + t;
                    if (q < ce && chain_ok(arena, base, len, q, mk)) {
                        found = q;
                        break;
                    }
                    lm &= lm - 1;
                }
                lanes &= lanes - 1;
            }
            from = wb + 4096;
        }
        if (found != kNone && found + 1 < ce && chain_ok(arena, base, len, found + 1, mk)) found += 1;
    }
    if (lane == 0) ch_entry[c] = found;
}

struct ScratchEmit {
    uint64_t *off;
    uint4 *hdr;
    uint32_t cap;
    __device__ void operator()(uint32_t i, uint64_t p, const Hdr &h) const {
        if (i < cap) {
            off[i] = p;
            hdr[i] = make_uint4(h.crc, h.ts, h.ks, h.vs);
        }
    }
};

__device__ void walk_into_chunk(const uint8_t *__restrict__ arena, const uint64_t *fbase,
                                const uint64_t *flen, uint32_t c, uint32_t f, uint64_t ce, uint64_t entry,
                                uint32_t cap, uint64_t *s_off, uint4 *s_hdr, uint32_t *ch_count,
                                uint64_t *ch_exit, uint32_t *ch_term, uint64_t *ch_tpos) {
    uint32_t count = 0, term = T_NONE;
    uint64_t exit = kNone, tpos = 0;
    if (entry != kNone) {
        ScratchEmit em{s_off + (uint64_t)c * cap, s_hdr + (uint64_t)c * cap, cap};
        walk_chain(arena, fbase[f], flen[f], ce, entry, em, count, exit, term, tpos);
    }
    ch_count[c] = count;
    ch_exit[c] = exit;
    ch_term[c] = term;
    ch_tpos[c] = tpos;
}

// One lane per chunk: latency-bound header chain from the speculative entry.
__global__ __launch_bounds__(256) void k_walk(const uint8_t *__restrict__ arena,
                                              const uint64_t *__restrict__ fbase,
                                              const uint64_t *__restrict__ flen,
                                              const uint32_t *__restrict__ ch_file,
                                              const uint64_t *__restrict__ ch_end,
                                              const uint64_t *__restrict__ ch_entry, uint32_t *ch_count,
                                              uint64_t *ch_exit, uint32_t *ch_term, uint64_t *ch_tpos,
                                              uint64_t *s_off, uint4 *s_hdr, uint32_t cap,
                                              uint32_t n_chunks) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    walk_into_chunk(arena, fbase, flen, c, ch_file[c], ch_end[c], ch_entry[c], cap, s_off, s_hdr, ch_count,
                    ch_exit, ch_term, ch_tpos);
}

// Chunk c is consistent iff its entry equals the record start that the chain
// of the nearest earlier non-empty chunk reaches (none if that chain ended).
// If every chunk is consistent, every chunk is correct (chunk 0 of each file
// is true by construction): induction over the chunk order.
__global__ __launch_bounds__(256) void k_validate(const uint32_t *__restrict__ ch_file,
                                                  const uint64_t *__restrict__ ch_start,
                                                  const uint64_t *__restrict__ ch_end,
                                                  const uint64_t *__restrict__ ch_entry,
                                                  const uint64_t *__restrict__ ch_exit,
                                                  const uint32_t *__restrict__ ch_term,
                                                  const uint32_t *__restrict__ f_first_chunk,
                                                  uint32_t *__restrict__ ch_bad, uint32_t *counter,
                                                  uint32_t c_begin, uint32_t c_end) {
    const uint32_t c = c_begin + blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= c_end) return;
    const uint32_t f = ch_file[c], fc = f_first_chunk[f];
    bool bad = false;
    if (c != fc) {
        uint32_t j = c - 1;
        while (j > fc && ch_entry[j] == kNone) --j;
        uint64_t expect = kNone;
        if (ch_entry[j] == kNone) {
            bad = true;
        } else if (ch_term[j] == T_NONE) {
            const uint64_t x = ch_exit[j];
            if (x < ch_start[c]) bad = true;
            else expect = x < ch_end[c] ? x : kNone;
        }
        if (!bad && ch_entry[c] != expect) bad = true;
    }
    ch_bad[c] = bad ? 1u : 0u;
    const uint64_t m = __ballot(bad);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(counter, (uint32_t)__popcll(m));
}

// One lane per inconsistent chunk: take the entry from the nearest earlier
// non-empty chunk and re-walk.  Chunks whose look-back crosses another
// inconsistent chunk wait for a later round (the next k_validate decides),
// so no lane reads state another lane is rewriting.
__global__ __launch_bounds__(256) void k_fixup(const uint8_t *__restrict__ arena,
                                               const uint64_t *__restrict__ fbase,
                                               const uint64_t *__restrict__ flen,
                                               const uint32_t *__restrict__ ch_file,
                                               const uint64_t *__restrict__ ch_end,
                                               const uint32_t *__restrict__ f_first_chunk,
                                               const uint32_t *__restrict__ ch_bad, uint64_t *ch_entry,
                                               uint32_t *ch_count, uint64_t *ch_exit, uint32_t *ch_term,
                                               uint64_t *ch_tpos, uint64_t *s_off, uint4 *s_hdr, uint32_t cap,
                                               uint32_t c_begin, uint32_t c_end, uint32_t *counter) {
    const uint32_t c = c_begin + blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= c_end || !ch_bad[c]) return;
    const uint32_t f = ch_file[c], fc = f_first_chunk[f];
    uint32_t j = c - 1;
    while (j > fc && ch_entry[j] == kNone && !ch_bad[j]) --j;
    if (ch_bad[j] || ch_entry[j] == kNone) return;
    uint64_t e_new = kNone;
    if (ch_term[j] == T_NONE) {
        const uint64_t x = ch_exit[j];
        if (x < ch_end[c]) e_new = x;
    }
    ch_entry[c] = e_new;
    atomicAdd(counter, 1u);
    walk_into_chunk(arena, fbase, flen, c, f, ch_end[c], e_new, cap, s_off, s_hdr, ch_count, ch_exit, ch_term,
                    ch_tpos);
}

// Exclusive scan of per-chunk record counts -> rec_base[0..n], offset by a
// device-resident base (the records of earlier file groups), without LDS (so
// the kernels can share CUs with k_crc_rows, which holds all of it):
// one wavefront per block of 4096 counts, one wavefront over the block totals,
// then an add-back.  rec_base[n] and *base_out = base + total.
constexpr uint32_t kScanBlock = 4096;

// Inclusive prefix sum over the 64 lanes (DPP row shifts + row broadcasts).
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);  // row_bcast:15
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return v;
}

__global__ __launch_bounds__(64) void k_scan_local(const uint32_t *__restrict__ ch_count,
                                                   uint64_t *__restrict__ rec_base, uint64_t *__restrict__ bsum,
                                                   uint32_t n) {
    const uint32_t lane = threadIdx.x;
    const uint32_t b0 = blockIdx.x * kScanBlock;
    uint64_t run = 0;
    for (uint32_t i0 = b0; i0 < min(b0 + kScanBlock, n); i0 += 64) {
        const uint32_t i = i0 + lane;
        const uint32_t v = i < n ? ch_count[i] : 0u;
        const uint32_t inc = wave_incl_sum(v);
        if (i < n) rec_base[i] = run + inc - v;
        run += (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);
    }
    if (lane == 0) bsum[blockIdx.x] = run;
}

__global__ __launch_bounds__(64) void k_scan_top(uint64_t *__restrict__ bsum, uint32_t nb,
                                                 const uint64_t *__restrict__ base_in, uint64_t *__restrict__ base_out,
                                                 uint64_t *__restrict__ rec_base, uint32_t n, uint64_t cap,
                                                 uint32_t *__restrict__ overflow) {
    const uint32_t lane = threadIdx.x;
    uint64_t run = *base_in;
    for (uint32_t i0 = 0; i0 < nb; i0 += 64) {
        const uint32_t i = i0 + lane;
        const uint64_t v = i < nb ? bsum[i] : 0u;
        // block totals can exceed 32 bits in sum: scan the two halves
        const uint32_t lo = wave_incl_sum((uint32_t)(v & 0xFFFFFFu));
        const uint32_t hi = wave_incl_sum((uint32_t)(v >> 24));
        const uint64_t inc = ((uint64_t)hi << 24) + lo;
        if (i < nb) bsum[i] = run + inc - v;
        run += ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 63) << 24) +
               (uint32_t)__builtin_amdgcn_readlane((int)lo, 63);
    }
    if (lane == 0) {
        // past the record-table capacity the range is clamped (later kernels
        // stay in bounds) and the run is flagged for the exact synchronous path
        if (run > cap) atomicAdd(overflow, 1u);
        rec_base[n] = min(run, cap);
        *base_out = min(run, cap);
    }
}

__global__ void k_scan_add(uint64_t *__restrict__ rec_base, const uint64_t *__restrict__ bsum, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) rec_base[i] += bsum[i / kScanBlock];
}

// Per-file summary: records of the file and its terminal condition.
__global__ void k_file_summary(const uint32_t *__restrict__ f_first_chunk,
                               const uint32_t *__restrict__ f_nchunks,
                               const uint64_t *__restrict__ rec_base, const uint64_t *__restrict__ ch_entry,
                               const uint32_t *__restrict__ ch_term, const uint64_t *__restrict__ ch_tpos,
                               uint32_t *f_term, uint64_t *f_tpos, uint64_t *f_first_rec, uint64_t *f_nrec,
                               uint32_t nfiles) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nfiles) return;
    const uint32_t fc = f_first_chunk[f], nc = f_nchunks[f];
    f_first_rec[f] = rec_base[fc];
    f_nrec[f] = rec_base[fc + nc] - rec_base[fc];
    uint32_t term = T_NONE;
    uint64_t tpos = 0;
    // the terminal chunk is the last non-empty chunk of the file
    for (int64_t k = (int64_t)fc + nc - 1; k >= (int64_t)fc; --k) {
        if (ch_entry[k] != kNone) {
            term = ch_term[k];
            tpos = ch_tpos[k];
            break;
        }
    }
    f_term[f] = term;
    f_tpos[f] = tpos;
}

struct DirectEmit {
    uint64_t *rec_off;
    uint4 *rec_hdr;
    uint32_t *rec_file;
    uint64_t rb, n_total, base;
    uint32_t f;
    __device__ void operator()(uint32_t i, uint64_t p, const Hdr &h) const {
        const uint64_t r = rb + i;
        if (r < n_total) {
            rec_off[r] = base + p;
            rec_hdr[r] = make_uint4(h.crc, h.ts, h.ks, h.vs);
            rec_file[r] = f;
        }
    }
};

// Record table in walk order: one wavefront per chunk copies its staged
// headers; chunks that overflowed the stage re-walk straight into the table.
__global__ __launch_bounds__(256) void k_compact(const uint8_t *__restrict__ arena,
                                                 const uint64_t *__restrict__ fbase,
                                                 const uint64_t *__restrict__ flen,
                                                 const uint32_t *__restrict__ ch_file,
                                                 const uint64_t *__restrict__ ch_end,
                                                 const uint64_t *__restrict__ ch_entry,
                                                 const uint32_t *__restrict__ ch_count,
                                                 const uint64_t *__restrict__ rec_base,
                                                 const uint64_t *__restrict__ s_off,
                                                 const uint4 *__restrict__ s_hdr, uint32_t cap,
                                                 uint32_t n_chunks, uint64_t n_total, uint64_t *rec_off,
                                                 uint4 *rec_hdr, uint32_t *rec_file, uint32_t *counters) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= n_chunks) return;
    const uint64_t entry = ch_entry[c];
    const uint32_t cnt = ch_count[c];
    const uint64_t rb = rec_base[c];
    if (entry == kNone || cnt == 0 || rb >= n_total) return;
    const uint32_t f = ch_file[c];
    const uint64_t base = fbase[f];
    if (cnt <= cap) {
        for (uint32_t i = lane; i < cnt; i += 64) {
            const uint64_t r = rb + i;
            if (r >= n_total) break;
            const uint64_t si = (uint64_t)c * cap + i;
            rec_off[r] = base + s_off[si];
            rec_hdr[r] = s_hdr[si];
            rec_file[r] = f;
        }
    } else if (lane == 0) {
        atomicAdd(&counters[2], 1u);
        DirectEmit em{rec_off, rec_hdr, rec_file, rb, n_total, base, f};
        uint32_t count, term;
        uint64_t exit, tpos;
        walk_chain(arena, base, flen[f], ch_end[c], entry, em, count, exit, term, tpos);
    }
}

__device__ __forceinline__ uint64_t value_end(const uint64_t *rec_off, const uint4 *rec_hdr, uint64_t r) {
    const uint4 h = rec_hdr[r];
    return rec_off[r] + 16 + (uint64_t)h.z + h.w;  // tombstone: KeySize 0, the key is the "value"
}

// Record range [rng[0], rng[1]) of one file group (device-resident: the group
// scans of the pipeline produce them without a host round trip).
//
// row_first[row] = first record whose value ends after the row's first byte,
// for the rows [r0, ...) of the group; rows past the group's last record end
// keep k_row_fill's value rng[1].  Grid-stride over the device range.
// k_row_fill writes rows (r0, r1]: row r1 (the next group's first row) gets
// rng[1] = the next group's first record, its final value, before the next
// group starts, so the row entries a group reads never change under it.  Row 0
// is 0 from the start of the run.
__global__ void k_row_fill(uint32_t *__restrict__ row_first, uint64_t r0, uint64_t r1,
                           const uint64_t *__restrict__ rng) {
    const uint32_t v = (uint32_t)rng[1];
    for (uint64_t row = r0 + 1 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; row <= r1;
         row += (uint64_t)gridDim.x * blockDim.x)
        row_first[row] = v;
}

__global__ void k_row_index(const uint64_t *__restrict__ rec_off, const uint4 *__restrict__ rec_hdr,
                            const uint64_t *__restrict__ rng, uint64_t r0, uint32_t *__restrict__ row_first) {
    const uint64_t rb = rng[0], re = rng[1];
    for (uint64_t r = rb + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < re;
         r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t ve_r = value_end(rec_off, rec_hdr, r);
        const uint64_t lo = r == rb ? r0 : (value_end(rec_off, rec_hdr, r - 1) + kRow - 1) / kRow;
        const uint64_t hi = (ve_r + kRow - 1) / kRow;
        for (uint64_t row = lo; row < hi; ++row) row_first[row] = (uint32_t)r;
    }
}

// lastOffset carried into each file of a group (core/db.go:110-123,
// core/keydir.go:22-53): after a file it is reset iff the file is not the
// active one, else advanced by the bytes the walk consumed.  One thread; the
// group's outgoing value feeds the next group.
__global__ void k_group_carry(uint32_t nf, const uint64_t *__restrict__ flen, const uint32_t *__restrict__ freset,
                              const uint32_t *__restrict__ fterm, const uint64_t *__restrict__ ftpos,
                              uint32_t *__restrict__ carry, const uint32_t *__restrict__ carry_in,
                              uint32_t *__restrict__ carry_out) {
    uint32_t last = *carry_in;
    for (uint32_t f = 0; f < nf; ++f) {
        carry[f] = last;
        last += (uint32_t)(fterm[f] != T_NONE ? ftpos[f] : flen[f]);
        if (freset[f]) last = 0;
    }
    *carry_out = last;
}

constexpr int kPlanBytes = 64;  // per row: one byte per 64 B slab (= per k_crc_rows lane)


// Per-row plan for k_crc_rows, 64 bytes, byte k for lane k (slab k):
//   bits 0..6  cut: offset (1..64) inside slab k where a record ends, 0 = none
//   bit  7     bit k of the row header H, recovered with one ballot:
//              H[0..31] = ra, the first record whose end lies past the row start
// Record ids of the cuts follow from ra and the cut ballot (mbcnt), so the
// plan carries no ids or counts.  Rows where a slab holds 2+ record ends
// (records under 64 B) are listed for k_crc_rows_big, which rewrites all of
// k_crc_rows' outputs for them.
//
// One wavefront per 64 rows (lane = row): the records ending in those rows
// are a contiguous range, read 64 at a time (coalesced); each lane ORs its
// record's cut into an LDS image of the 64 plan rows, then every lane writes
// its row (64 B, header bits added): 4 KiB contiguous per wavefront.
constexpr int kPlanWaves = 4;

__global__ __launch_bounds__(64 * kPlanWaves) void k_row_plan(const uint64_t *__restrict__ rec_off,
                                                              const uint4 *__restrict__ rec_hdr,
                                                              const uint64_t *__restrict__ rng, uint64_t r0,
                                                              uint64_t nr, const uint32_t *__restrict__ row_first,
                                                              uint4 *__restrict__ plan,
                                                              uint32_t *__restrict__ big_rows,
                                                              uint32_t *__restrict__ big_cnt, uint32_t *big_any) {
    __shared__ uint32_t cut_lds[kPlanWaves][64 * 17];  // row stride 17 words: conflict-free row reads
    __shared__ uint32_t slow_lds[kPlanWaves][64];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint64_t R0 = r0 + ((uint64_t)blockIdx.x * kPlanWaves + wv) * 64, r1 = r0 + nr;
    if (R0 >= r1) return;
    uint32_t *cw = cut_lds[wv];
    for (uint32_t i = lane; i < 64 * 17; i += 64) cw[i] = 0;
    slow_lds[wv][lane] = 0;
    const uint64_t Re = min(R0 + 64, r1);  // rows [R0, Re)
    const uint64_t R = R0 + lane;
    const bool live = R < Re;
    const uint32_t ra = live ? row_first[R] : 0u;
    const uint64_t lo = row_first[R0], hi = row_first[Re];  // records ending in rows [R0, Re)
    for (uint64_t b = lo; b < hi; b += 64) {
        const uint64_t r = b + lane;
        if (r < hi) {
            const uint64_t ve = value_end(rec_off, rec_hdr, r);
            const uint32_t rl = (uint32_t)((ve - 1) / kRow - R0);  // 0..63
            const uint32_t end = (uint32_t)(ve - (R0 + rl) * kRow), slab = (end - 1) >> 6;
            atomicOr(cw + rl * 17 + (slab >> 2), (end - slab * kSlab) << (8 * (slab & 3)));
            // the record before ends in the same slab (never for the range's
            // first record: it ends in an earlier row)
            if (r > lo && (value_end(rec_off, rec_hdr, r - 1) - 1) >> 6 == (ve - 1) >> 6) slow_lds[wv][rl] = 1;
        }
    }
    // header bits (ra) into the LDS image, then write the 64 rows out with
    // each store instruction covering 1 KiB contiguous (a lane-per-row store
    // would scatter 16 B pieces at a 64 B stride: partial-line writes)
    const uint64_t H = ra;
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // header bits live in bytes 0..31 (ra is 32 bits)
        const uint32_t nib = (uint32_t)(H >> (4 * i)) & 15u;
        cw[lane * 17 + i] |= ((nib & 1u) << 7) | ((nib & 2u) << 14) | ((nib & 4u) << 21) | ((nib & 8u) << 28);
    }
    uint4 *blk = plan + R0 * 4;  // the wavefront's rows as 16 B units
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t u = lane + 64 * k, rl = u >> 2, q = (u & 3) * 4;  // 16 B unit u: row rl, words q..q+3
        if (R0 + rl < Re)
            blk[u] = make_uint4(cw[rl * 17 + q], cw[rl * 17 + q + 1], cw[rl * 17 + q + 2], cw[rl * 17 + q + 3]);
    }
    // slow rows: compacted into this wavefront's 64 list slots, count per
    // wavefront (no atomics: a global counter here serialises at one address)
    const bool slow = live && slow_lds[wv][lane];
    const uint64_t sm = __ballot(slow);
    const uint32_t w = (uint32_t)((R0 - r0) >> 6);
    if (slow) big_rows[(uint64_t)w * 64 + __builtin_amdgcn_mbcnt_hi((uint32_t)(sm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)sm, 0u))] = (uint32_t)R;
    if (lane == 0) {
        big_cnt[w] = (uint32_t)__popcll(sm);
        if (sm) *big_any = 1u;
    }
}

// LDS image of the slicing-by-4 tables: two 64 KiB regions; in region r,
// entry b of half h, copy l31 sits at byte address r*65536 + b*256 + h*128 +
// l31*4 (tables T3, T2 in region 0, T1, T0 in region 1).  Every lane of a
// 32-lane LDS group reads its own bank, so lookups are conflict free
// (MI355X_MICROARCH.md §LDS), and the address of a lookup is ONE v_perm_b32:
// byte 0 = the lane's l31*4, byte 1 = the index byte, byte 2 = the region
// (from the lane base lb0 = l31*4 or lb1 = 65536 + l31*4); the half is the
// ds_read immediate offset.
__device__ __forceinline__ uint32_t lds_at(const uint32_t *lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(lds) + byte_addr);
}
template <int K>
__device__ __forceinline__ uint32_t tbl_addr(uint32_t c, uint32_t lb) {
    return __builtin_amdgcn_perm(c, lb, 0x0C020000u | ((4u + K) << 8));
}
// crc' = T3[b0] ^ T2[b1] ^ T1[b2] ^ T0[b3] for c = crc ^ word.
__device__ __forceinline__ uint32_t slice4(const uint32_t *lds, uint32_t lb0, uint32_t lb1, uint32_t c) {
    return lds_at(lds, tbl_addr<0>(c, lb0)) ^ lds_at(lds, tbl_addr<1>(c, lb0) + 128) ^
           lds_at(lds, tbl_addr<2>(c, lb1)) ^ lds_at(lds, tbl_addr<3>(c, lb1) + 128);
}
// One byte through T0: crc' = T0[(crc ^ b) & 0xFF] ^ crc >> 8.
__device__ __forceinline__ uint32_t byte1(const uint32_t *lds, uint32_t lb1, uint32_t crc, uint32_t b) {
    return lds_at(lds, tbl_addr<0>(crc ^ b, lb1) + 128) ^ (crc >> 8);
}


template <int CTRL, int ROWMASK>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWMASK, 0xF, false);
}

// LDS image of the CRC tables (identical in every k_crc_rows* workgroup).
__device__ __forceinline__ void fill_crc_lds(uint32_t *lds, const uint32_t *__restrict__ g_slice,
                                             const uint32_t *__restrict__ g_nib) {
    for (uint32_t i = threadIdx.x; i < 32768; i += blockDim.x)
        lds[i] = g_slice[(3 - ((i >> 13) & 2) - ((i >> 5) & 1)) * 256 + ((i >> 6) & 255)];
    for (uint32_t i = threadIdx.x; i < 8192; i += blockDim.x) {
        const uint32_t l = (i >> 12) * 32 + (i & 31), v = (i >> 5) & 15, q = (i >> 9) & 7;
        lds[kNibBase + i] = g_nib[(l * 8 + q) * 16 + v];
    }
    __syncthreads();
}

// Per-lane state of one row (see k_crc_rows).
struct RowCuts {
    int ncut = 0;
    int32_t c0 = 99, c1 = 99, c2 = 99, c3 = 99;  // record end offsets inside the slab (1..64); named
    uint32_t id0 = 0, id1 = 0, id2 = 0, id3 = 0;  // registers, never an indexed array (no scratch)
    uint32_t n_le = 0;                             // record ends at or before the slab end
    int32_t my_end = 0;                            // row-relative end of record ra + lane
    __device__ __forceinline__ void take(uint32_t end, uint32_t j, uint32_t ra, uint32_t lane, int32_t s_rel) {
        const int32_t cc = (int32_t)end - s_rel;
        if (cc > 0 && cc <= kSlab) {
            const uint32_t id = ra + j;
            c0 = ncut == 0 ? cc : c0;
            c1 = ncut == 1 ? cc : c1;
            c2 = ncut == 2 ? cc : c2;
            c3 = ncut == 3 ? cc : c3;
            id0 = ncut == 0 ? id : id0;
            id1 = ncut == 1 ? id : id1;
            id2 = ncut == 2 ? id : id2;
            id3 = ncut == 3 ? id : id3;
            ++ncut;
        }
        n_le += (int32_t)end <= s_rel + kSlab ? 1u : 0u;
        my_end = lane == j ? (int32_t)end : my_end;
    }
};

struct RowOut {
    uint32_t e[4] = {0, 0, 0, 0};  // register at each record end in the slab
    uint32_t pre_first = 0;         // run just before the first record end of the slab
    uint32_t rend = 0;              // (lane 63) run open at the row end
};

// Z_{64(63-lane)}(z) (the open register referenced to the row end, 8 nibble
// lookups in the lane's LDS table), then a segmented inclusive XOR over the
// wave: lanes whose open register belongs to the same record t form a run.
// runv = run value up to this lane, runprev = the previous lane's, tprev = its t.
__device__ __forceinline__ void wave_runs(const uint32_t *lds, uint32_t lane, uint32_t nbase, uint32_t z,
                                          uint32_t t, uint32_t &runv, uint32_t &runprev, uint32_t &tprev) {
    // Z_{64(63-lane)}(z): reference the open register to the row end
    uint32_t cz = 0;
#pragma unroll
    for (int qn = 0; qn < 8; ++qn) cz ^= lds[nbase + qn * 512 + (((z >> (4 * qn)) & 15u) << 5)];
    // inclusive prefix XOR over the wave (DPP row shifts + row broadcasts)
    uint32_t P = cz;
    P ^= dpp<0x111, 0xF>(P);  // row_shr:1
    P ^= dpp<0x112, 0xF>(P);  // row_shr:2
    P ^= dpp<0x114, 0xF>(P);  // row_shr:4
    P ^= dpp<0x118, 0xF>(P);  // row_shr:8
    P ^= dpp<0x142, 0xA>(P);  // row_bcast:15 -> rows 1, 3
    P ^= dpp<0x143, 0xC>(P);  // row_bcast:31 -> rows 2, 3
    tprev = (uint32_t)__builtin_amdgcn_update_dpp((int)kNone32, (int)t, 0x138, 0xF, 0xF, false);
    const bool start = lane == 0 || t != tprev;
    const uint64_t B = __ballot(start);
    const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
    const int rsl = 63 - __clzll((long long)(B & upto));
    const uint32_t Pp = __shfl(P, rsl > 0 ? rsl - 1 : 0);
    runv = P ^ (rsl > 0 ? Pp : 0u);
    runprev = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)runv, 0x138, 0xF, 0xF, false);
}

// The per-row work of k_crc_rows: every byte of the slab enters the CRC
// register; it is closed at each record end (exactly: the last partial word
// byte-wise), the open register at the slab end is shifted to the row end and
// a segmented XOR over the wave joins each record's lanes.
template <int MODE>
__device__ __forceinline__ RowOut crc_row(const uint32_t *lds, uint32_t lane, uint32_t lb0, uint32_t lb1, uint32_t nbase,
                                          int32_t s_rel, uint64_t rs, uint32_t (&words)[16], const RowCuts &rc,
                                          uint32_t t) {
    RowOut o;
    int q = 0;
    int32_t cc = rc.c0, n1 = rc.c1, n2 = rc.c2, n3 = rc.c3;  // pending cuts, shifted down at each cut
    int32_t cj = (cc - 1) >> 2;  // word holding the record's last byte (99 -> never)
    uint32_t crc = 0;
    if constexpr ((MODE & 8) != 0) {  // ablation: synthetic bytes instead of the loaded row
#pragma unroll
        for (int j = 0; j < 16; ++j) words[j] = (uint32_t)(rs >> 4) * 2654435761u + lane * 97u + j;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t x = words[j];
        uint32_t nc = (MODE & 2) ? __builtin_amdgcn_alignbit(crc ^ x, crc ^ x, 5) + 0x9E3779B9u
                                 : slice4(lds, lb0, lb1, crc ^ x);
        if (j == cj) {
            const int nb = cc - 4 * j;
            if (nb < 4) {
                nc = crc;
                uint32_t y = x;
                for (int b = 0; b < nb; ++b) {
                    nc = byte1(lds, lb1, nc, y);
                    y >>= 8;
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) o.e[k] = q == k ? nc : o.e[k];
            nc = 0;
            ++q;
            cc = n1;
            n1 = n2;
            n2 = n3;
            n3 = 99;
            cj = (cc - 1) >> 2;
        }
        crc = nc;
    }
    const uint32_t z = t != kNone32 ? crc : 0u;
    o.rend = crc ^ t;
    if constexpr ((MODE & 4) != 0) {  // ablation: no tail shift / segmented scan
        asm volatile("" ::"v"(crc), "v"(z));
    } else {
        uint32_t runv, runprev, tprev;
        wave_runs(lds, lane, nbase, z, t, runv, runprev, tprev);
        o.rend = t != kNone32 ? runv : 0u;
        // the first record closing in this slab continues the run of the lane before
        o.pre_first = (rc.ncut > 0 && lane > 0 && tprev == rc.id0) ? runprev : 0u;
    }
    return o;
}

struct RowOut1 {
    uint32_t e = 0;    // register at the record end in the slab
    uint32_t pre = 0;  // run of the lanes before, for the record ending in the slab
    uint32_t rend = 0; // run open at the slab end, referenced to the row end (lane 63: the row's)
};

// The per-row work of k_crc_rows for rows with at most one record end per
// slab: every byte of the slab enters the CRC register; it is closed at the
// record end cc (the last partial word byte-wise), the open register at the
// slab end is shifted to the row end and a segmented XOR over the wave joins
// each record's lanes.
template <int MODE>
__device__ __forceinline__ RowOut1 crc_row1(const uint32_t *lds, uint32_t lane, uint32_t lb0, uint32_t lb1,
                                            uint32_t nbase, uint64_t rs, uint32_t (&words)[16], int32_t cc,
                                            uint32_t my_id, uint32_t t) {
    RowOut1 o;
    const int32_t cj = cc ? (cc - 1) >> 2 : 99;  // word holding the record's last byte
    uint32_t crc = 0;
    if constexpr ((MODE & 8) != 0) {  // ablation: synthetic bytes instead of the loaded row
#pragma unroll
        for (int j = 0; j < 16; ++j) words[j] = (uint32_t)(rs >> 4) * 2654435761u + lane * 97u + j;
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t x = words[j];
        uint32_t nc = (MODE & 2) ? __builtin_amdgcn_alignbit(crc ^ x, crc ^ x, 5) + 0x9E3779B9u
                                 : slice4(lds, lb0, lb1, crc ^ x);
        if (j == cj) {
            const int nb = cc - 4 * j;
            if (nb < 4) {
                nc = crc;
                uint32_t y = x;
                for (int b = 0; b < nb; ++b) {
                    nc = byte1(lds, lb1, nc, y);
                    y >>= 8;
                }
            }
            o.e = nc;
            nc = 0;
        }
        crc = nc;
    }
    const uint32_t z = t != kNone32 ? crc : 0u;
    o.rend = crc ^ t;
    if constexpr ((MODE & 4) != 0) {  // ablation: no tail shift / segmented scan
        asm volatile("" ::"v"(crc), "v"(z));
    } else {
        uint32_t runv, runprev, tprev;
        wave_runs(lds, lane, nbase, z, t, runv, runprev, tprev);
        o.rend = t != kNone32 ? runv : 0u;
        // the record closing in this slab continues the run of the lane before
        o.pre = (cc && lane > 0 && tprev == my_id) ? runprev : 0u;
    }
    return o;
}

// NR rows of one wavefront at once (k_crc_rows): the NR CRC chains of a lane
// are independent, so their LDS lookups interleave and each wave keeps NR
// table reads in flight per step of the chain (ILP against LDS latency).  Per
// row exactly crc_row1's arithmetic.
template <int MODE, int NR>
__device__ __forceinline__ void crc_rowsN(const uint32_t *lds, uint32_t lane, uint32_t lb0, uint32_t lb1,
                                          uint32_t nbase, const uint64_t (&rs)[NR], uint32_t (&words)[NR][16],
                                          const int32_t (&cc)[NR], const uint32_t (&my_id)[NR],
                                          const uint32_t (&t)[NR], RowOut1 (&o)[NR]) {
    int32_t cj[NR];
    uint32_t crc[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        cj[i] = cc[i] ? (cc[i] - 1) >> 2 : 99;
        crc[i] = 0;
        o[i] = RowOut1{};
        if constexpr ((MODE & 8) != 0) {  // ablation: synthetic bytes instead of the loaded rows
#pragma unroll
            for (int j = 0; j < 16; ++j) words[i][j] = (uint32_t)(rs[i] >> 4) * 2654435761u + lane * 97u + j;
        }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        uint32_t nc[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i)
            nc[i] = (MODE & 2) ? __builtin_amdgcn_alignbit(crc[i] ^ words[i][j], crc[i] ^ words[i][j], 5) + 0x9E3779B9u
                               : slice4(lds, lb0, lb1, crc[i] ^ words[i][j]);
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            if (j == cj[i]) {
                const int nb = cc[i] - 4 * j;
                if (nb < 4) {
                    uint32_t x = crc[i], y = words[i][j];
                    for (int b = 0; b < nb; ++b) {
                        x = byte1(lds, lb1, x, y);
                        y >>= 8;
                    }
                    nc[i] = x;
                }
                o[i].e = nc[i];
                nc[i] = 0;
            }
            crc[i] = nc[i];
        }
    }
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const uint32_t z = t[i] != kNone32 ? crc[i] : 0u;
        o[i].rend = crc[i] ^ t[i];
        if constexpr ((MODE & 4) != 0) {  // ablation: no tail shift / segmented scan
            asm volatile("" ::"v"(crc[i]), "v"(z));
        } else {
            uint32_t runv, runprev, tprev;
            wave_runs(lds, lane, nbase, z, t[i], runv, runprev, tprev);
            o[i].rend = t[i] != kNone32 ? runv : 0u;
            o[i].pre = (cc[i] && lane > 0 && tprev == my_id[i]) ? runprev : 0u;
        }
    }
}


// The HBM-bound kernel.  A wavefront owns a 4 KiB row; lane k owns bytes
// [64k, 64k+64).  Every byte enters a CRC register, no masking: records tile
// the file, so lane k's register simply runs over whole records and is closed
// exactly at every record end and restarted at the next word.  The chain of
// record r therefore covers [align4(start_r), end_r) = header/key prefix ||
// value; k_finalize removes the prefix by linearity.  An open register at the
// slab end belongs to the record containing that position; it is referenced to
// the row end with the per-lane constant shift Z_{64(63-k)} (8 nibble lookups)
// and a segmented XOR over the wave (DPP prefix scan) joins each record's
// lanes.  Outputs: per record e (the register at its end) and pre (the run of
// the lanes before its closing slab), stored by the lane whose slab holds the
// record end (slot ra + mbcnt of the cut ballot); per row the run open at the
// row end.  A slab holds at most one record end here; rows where one holds
// more (records under 64 B) are flagged by k_row_plan and done by
// k_crc_rows_big (their stores here go to the scratch slots).
//
// Rows are local to the launch: arena, plan and out_rend point at its first
// row; n_total is the e/pre scratch slot, rend_scratch the rend one.
//
// Memory pipeline: the row data (4 x 16 B per lane) and the row plan byte are
// buffer loads (row base in a scalar resource, lane offset in a fixed VGPR)
// issued DEPTH rows ahead.  No scalar loads in the loop: an outstanding SMEM
// load would make every LDS wait (lgkmcnt(0)) wait for HBM too.  Control flow
// around the stores is uniform and their number fixed, so the compiler's vmcnt
// waits land rows after the loads they wait for.
template <int MODE, int DEPTH, int NR>
__global__ __launch_bounds__(1024) void k_crc_rows(const uint8_t *__restrict__ arena, uint64_t n_rows,
                                                   const uint8_t *__restrict__ plan, uint64_t n_total,
                                                   const uint32_t *__restrict__ g_slice,
                                                   const uint32_t *__restrict__ g_nib,
                                                   uint32_t *__restrict__ out_e, uint32_t *__restrict__ out_pre,
                                                   uint32_t *__restrict__ out_rend, uint32_t *__restrict__ rend_scratch) {
    __shared__ uint32_t lds[40960];  // 128 KiB slicing tables x32 copies + 32 KiB lane-shift tables
    fill_crc_lds(lds, g_slice, g_nib);
    const uint32_t lane = threadIdx.x & 63, l31 = lane & 31;
    const uint32_t nbase = kNibBase + (lane >> 5) * 4096 + l31;
    const uint32_t lb0 = l31 * 4, lb1 = 65536 + l31 * 4;
    const int32_t s_rel = (int32_t)lane * kSlab;
    // a step is NR consecutive rows; steps are strided over the wavefronts
    const uint64_t n_steps = (n_rows + NR - 1) / NR;
    const uint64_t stride = (uint64_t)gridDim.x * kWaves;

    uint64_t step = __builtin_amdgcn_readfirstlane((uint32_t)(blockIdx.x * kWaves + (threadIdx.x >> 6)));
    if (step >= n_steps) return;
    struct RowBuf {
        u32x4 x[4];
        uint32_t pv;
    };
    auto issue = [&](uint64_t st, RowBuf (&bs)[NR]) {
        if constexpr ((MODE & 8) != 0) return;
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            // buffer loads: the row base lives in a scalar resource, the lane
            // offset in one VGPR that never changes (no per-load VGPR address)
            const uint64_t r = min(st * NR + i, n_rows - 1);
            const __amdgpu_buffer_rsrc_t rrow = make_rsrc(arena + r * kRow, kRow);
            const __amdgpu_buffer_rsrc_t rplan = make_rsrc(plan + r * kPlanBytes, kPlanBytes);
            bs[i].x[0] = __builtin_amdgcn_raw_buffer_load_b128(rrow, (uint32_t)s_rel, 0, 0);
            bs[i].x[1] = __builtin_amdgcn_raw_buffer_load_b128(rrow, (uint32_t)s_rel + 16, 0, 0);
            bs[i].x[2] = __builtin_amdgcn_raw_buffer_load_b128(rrow, (uint32_t)s_rel + 32, 0, 0);
            bs[i].x[3] = __builtin_amdgcn_raw_buffer_load_b128(rrow, (uint32_t)s_rel + 48, 0, 0);
            bs[i].pv = __builtin_amdgcn_raw_buffer_load_b8(rplan, lane, 0, 0);
        }
    };
    auto process = [&](uint64_t st, const RowBuf (&bs)[NR]) {
        uint64_t rs[NR], row[NR];
        int32_t cc[NR];
        uint32_t ra[NR], idx[NR], my_id[NR], t[NR];
        uint32_t words[NR][16];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            row[i] = st * NR + i;
            rs[i] = row[i] * kRow;
            // row header from bit 7 of the 64 plan bytes, the cut of this slab from bits 0..6
            const uint64_t H = __ballot(bs[i].pv & 0x80u);
            ra[i] = (uint32_t)H;

            cc[i] = (MODE & 1) ? 0 : (int32_t)(bs[i].pv & 0x7Fu);
            const uint64_t C = __ballot(cc[i] != 0);
            idx[i] = __builtin_amdgcn_mbcnt_hi((uint32_t)(C >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)C, 0u));
            const uint32_t n_le = idx[i] + (cc[i] != 0);  // record ends at or before the slab end
            // the record open at the slab end: the next one after the ends
            // counted.  (Past a file's last record the slab is padding and
            // "record" t is the next file's first one or none: the padding only
            // reaches this row's rend, which no record reads, since records
            // never cross files and files start on row boundaries.)
            t[i] = ra[i] + n_le;
            my_id[i] = ra[i] + idx[i];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                words[i][4 * k] = bs[i].x[k].x;
                words[i][4 * k + 1] = bs[i].x[k].y;
                words[i][4 * k + 2] = bs[i].x[k].z;
                words[i][4 * k + 3] = bs[i].x[k].w;
            }
        }
        RowOut1 o[NR];
        crc_rowsN<MODE, NR>(lds, lane, lb0, lb1, nbase, rs, words, cc, my_id, t, o);
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            // every lane stores: the cut lanes to their record's slot, the rest
            // (and rows past the end) to the scratch slots (no branch around a
            // store).  A row where a slab holds 2+ record ends gets cuts OR'ed
            // together here; k_crc_rows_big then rewrites all its outputs.
            const bool dead = row[i] >= n_rows;
            const uint64_t slot = (cc[i] != 0 && !dead) ? (uint64_t)ra[i] + idx[i] : n_total;
            out_e[slot] = o[i].e;
            out_pre[slot] = o[i].pre;
            *(dead ? rend_scratch : out_rend + row[i]) = (uint32_t)__builtin_amdgcn_readlane((int)o[i].rend, 63);
        }
    };
    // DEPTH steps in flight while one is processed; the loop is unrolled over
    // the DEPTH+1 buffer sets so each has fixed registers (a rotating copy
    // would force a wait on loads still in flight).
    RowBuf buf[DEPTH + 1][NR] = {};
#pragma unroll
    for (int i = 0; i < DEPTH; ++i) {
        issue(step + i * stride, buf[i]);
        // the stores of a processed step, to the scratch slots: the loop is
        // entered with the same vector-memory queue shape as its back edge, so
        // the compiler's waits at the loop head are as late as in the body
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            out_e[n_total] = 0;
            out_pre[n_total] = 0;
            *rend_scratch = 0;
        }
    }
    for (;;) {
#pragma unroll
        for (int i = 0; i <= DEPTH; ++i) {
            issue(step + DEPTH * stride, buf[(i + DEPTH) % (DEPTH + 1)]);
            process(step, buf[i]);
            step += stride;
            if (step >= n_steps) return;
        }
    }
}

// Rows where a slab holds 2+ record ends (records shorter than 64 B): one
// wavefront per listed row, record ends read from the record table, direct
// stores; up to 4 ends per slab (a record is at least 16 B).
template <int MODE>
__global__ __launch_bounds__(1024) void k_crc_rows_big(const uint8_t *__restrict__ arena,
                                                       const uint32_t *__restrict__ big_rows,
                                                       const uint32_t *__restrict__ big_cnt,
                                                       const uint32_t *__restrict__ big_any, uint32_t n_lists,
                                                       const uint32_t *__restrict__ row_first,
                                                       const uint64_t *__restrict__ rng,
                                                       const uint64_t *__restrict__ rec_off,
                                                       const uint4 *__restrict__ rec_hdr,
                                                       const uint32_t *__restrict__ g_slice,
                                                       const uint32_t *__restrict__ g_nib,
                                                       uint32_t *__restrict__ out_e, uint32_t *__restrict__ out_pre,
                                                       uint32_t *__restrict__ out_rend) {
    if (*big_any == 0) return;
    const uint64_t n_total = rng[1];
    __shared__ uint32_t lds[40960];
    fill_crc_lds(lds, g_slice, g_nib);
    const uint32_t lane = threadIdx.x & 63, l31 = lane & 31;
    const uint32_t nbase = kNibBase + (lane >> 5) * 4096 + l31;
    const uint32_t lb0 = l31 * 4, lb1 = 65536 + l31 * 4;
    const int32_t s_rel = (int32_t)lane * kSlab;
    // list w holds big_cnt[w] rows at big_rows[64 w ..] (k_row_plan)
    uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + (threadIdx.x >> 6)), i = 0;
    for (;;) {
        while (w < n_lists && i >= big_cnt[w]) {
            w += gridDim.x * kWaves;
            i = 0;
        }
        if (w >= n_lists) break;
        const uint64_t row = big_rows[(uint64_t)w * 64 + i++], rs = row * kRow;
        const uint32_t ra = row_first[row], rb = row_first[row + 1], n_ends = rb - ra;

        RowCuts rc;
        for (uint32_t j0 = 0; j0 < n_ends; j0 += 64) {
            const uint32_t cnt = min(64u, n_ends - j0);
            const uint64_t r = min((uint64_t)ra + j0 + min(lane, cnt - 1), n_total - 1);
            const int32_t e_ = (int32_t)(value_end(rec_off, rec_hdr, r) - rs);
            for (uint32_t j = 0; j < cnt; ++j) rc.take((uint32_t)__builtin_amdgcn_readlane(e_, j), j0 + j, ra, lane, s_rel);
        }
        const uint32_t t = ra + rc.n_le;  // see k_crc_rows
        const uint4 *src = reinterpret_cast<const uint4 *>(arena + rs + s_rel);
        uint32_t words[16];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint4 v = src[k];
            words[4 * k] = v.x;
            words[4 * k + 1] = v.y;
            words[4 * k + 2] = v.z;
            words[4 * k + 3] = v.w;
        }
        const RowOut o = crc_row<MODE>(lds, lane, lb0, lb1, nbase, s_rel, rs, words, rc, t);
        if (rc.ncut > 0) out_e[rc.id0] = o.e[0], out_pre[rc.id0] = o.pre_first;
        if (rc.ncut > 1) out_e[rc.id1] = o.e[1], out_pre[rc.id1] = 0u;
        if (rc.ncut > 2) out_e[rc.id2] = o.e[2], out_pre[rc.id2] = 0u;
        if (rc.ncut > 3) out_e[rc.id3] = o.e[3], out_pre[rc.id3] = 0u;
        if (lane == 63) out_rend[row] = o.rend;
    }
}

// Per record (core/db.go:311 applied to every record):
//   chain = F(0, [align4(start), end)) = e ^ Z_-(row_end-end)(stitched runs),
//           runs stitched over rows by Horner with Z_4096 (LDS byte tables);
//   F(0, value) = chain ^ Z_V(F(0, prefix)), prefix = header bytes from
//           align4(start) plus the key (bytes the chain saw before the value);
//   crc = F(0, value) ^ crc32(0^V)  (table for V < 2^17).
// ValuePos = lastOffset + 16 + KeySize mod 2^32 (core/keydir.go:25), with
// lastOffset = carry + offset within the file.
__device__ __forceinline__ uint32_t z4096(const uint32_t *Tz, uint32_t a) {
    return Tz[a & 0xFF] ^ Tz[256 + ((a >> 8) & 0xFF)] ^ Tz[512 + ((a >> 16) & 0xFF)] ^ Tz[768 + (a >> 24)];
}

__global__ __launch_bounds__(256) void k_finalize(const uint8_t *__restrict__ arena,
                                                  const uint64_t *__restrict__ rec_off,
                                                  const uint4 *__restrict__ rec_hdr,
                                                  const uint32_t *__restrict__ rec_file,
                                                  const uint64_t *__restrict__ fbase,
                                                  const uint32_t *__restrict__ carry, const uint64_t *__restrict__ rng,
                                                  const uint32_t *__restrict__ e, const uint32_t *__restrict__ pre,
                                                  const uint32_t *__restrict__ rend,
                                                  const uint32_t *__restrict__ g_slice,
                                                  const uint32_t *__restrict__ xinv, const uint32_t *__restrict__ zrow,
                                                  const uint32_t *__restrict__ zl, const uint32_t *__restrict__ xa,
                                                  const uint32_t *__restrict__ xb, gck_rec *__restrict__ out,
                                                  uint32_t *counters) {
    __shared__ uint32_t Tz[1024];  // Z_4096 as 4 byte tables
    __shared__ uint32_t T[1024];   // slicing-by-4 tables T0..T3
    for (uint32_t i = threadIdx.x; i < 1024; i += blockDim.x) {
        Tz[i] = zrow[i];
        T[i] = g_slice[i];
    }
    __syncthreads();
    const uint64_t rb = rng[0], re = rng[1], G = (uint64_t)gridDim.x * blockDim.x;
    // software-pipelined over the grid-stride loop: the next record's table
    // entries are in flight while this one is finished
    struct RecIn {
        uint64_t start;
        uint4 h;
        uint32_t f, e, pre;
    };
    auto fetch = [&](uint64_t r) {
        RecIn x;
        x.start = rec_off[r];
        x.h = rec_hdr[r];
        x.f = rec_file[r];
        x.e = e[r];
        x.pre = pre[r];
        return x;
    };
    uint64_t r = rb + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t n_rej = 0;  // verdict rejects of this thread (summed per block at the end)
    RecIn cur{};
    if (r < re) cur = fetch(r);
    for (; r < re; r += G) {
        const RecIn nxt = fetch(min(r + G, re - 1));
        const uint64_t start = cur.start;
        const uint4 h = cur.h;
        const uint32_t f = cur.f;
        const uint32_t V = h.w;
        const uint64_t vs = start + 16 + h.z, ve = vs + V;
        const uint64_t w0 = (start + 3) & ~3ull;
        const uint64_t fr = w0 / kRow, lr = (ve - 1) / kRow;
        const uint64_t row_end = (lr + 1) * kRow;
        // independent loads first: the tables for the shifts, the prefix words
        const uint32_t xinv_d = xinv[row_end - ve];
        const uint32_t xv = V < 65536 ? xb[V] : multmodp(xa[V >> 16], xb[V & 0xFFFF]);
        const uint32_t zv = V < (1u << 17) ? zl[V] : 0u;
        const uint32_t L = (uint32_t)(vs - w0);
        const uint32_t *wp = reinterpret_cast<const uint32_t *>(arena + w0);
        uint32_t pw[10];
#pragma unroll
        for (int i = 0; i < 10; ++i) pw[i] = wp[i];  // header tail + keys up to 24 B (the arena is padded)
        // Horner over the rows the chain crosses; the row values are loaded 8
        // at a time so their latency overlaps
        uint32_t acc = 0;
        for (uint64_t row = fr; row < lr; row += 8) {
            uint32_t v[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) v[j] = row + j < lr ? rend[row + j] : 0u;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                if (row + j < lr) acc = z4096(Tz, acc) ^ v[j];
        }
        acc = z4096(Tz, acc) ^ cur.pre;
        const uint32_t chain = cur.e ^ (acc ? multmodp(xinv_d, acc) : 0u);
        // F(0, prefix): the bytes [w0, vs) = header tail + key as aligned words
        // (slicing-by-4), the last partial word bytewise
        uint32_t p = 0;
        for (uint32_t i = 0; i < L / 4; ++i) {
            const uint32_t x = p ^ (i < 10 ? pw[i] : wp[i]);
            p = T[768 + (x & 0xFF)] ^ T[512 + ((x >> 8) & 0xFF)] ^ T[256 + ((x >> 16) & 0xFF)] ^ T[x >> 24];
        }
        if (L & 3) {
            uint32_t y = L / 4 < 10 ? pw[L / 4] : wp[L / 4];
            for (uint32_t i = 0; i < (L & 3); ++i, y >>= 8) p = T[(p ^ y) & 0xFF] ^ (p >> 8);
        }
        const uint32_t raw0 = chain ^ (p ? multmodp(xv, p) : 0u);
        const uint32_t z = V < (1u << 17) ? zv : multmodp(multmodp(xa[V >> 16], xb[V & 0xFFFF]), 0xFFFFFFFFu) ^ 0xFFFFFFFFu;
        const uint32_t calc = raw0 ^ z;
        const uint64_t fo = start - fbase[f];
        const bool tomb = h.z == 0;
        gck_rec o;
        o.rec_off = fo;
        o.file = f;
        o.key_len = tomb ? h.w : h.z;
        o.value_pos = carry[f] + (uint32_t)fo + 16u + h.z;
        o.value_size = h.w;
        o.crc = h.x;
        o.ts = h.y;
        o.flags = (tomb ? GCK_F_TOMBSTONE : 0u) | (calc == h.x ? GCK_F_CRC_OK : 0u);
        o.crc_calc = calc;
        out[r] = o;
        n_rej += calc != h.x;
        cur = nxt;
    }
    // one global atomic per block (per-record or per-wavefront atomics on one
    // address serialise: C5 has ~100k rejects)
    __shared__ uint32_t blk_rej;
    if (threadIdx.x == 0) blk_rej = 0;
    __syncthreads();
    const uint32_t wsum = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_sum(n_rej), 63);
    if ((threadIdx.x & 63) == 0 && wsum) atomicAdd(&blk_rej, wsum);
    __syncthreads();
    if (threadIdx.x == 0 && blk_rej) atomicAdd(&counters[3], blk_rej);
}

// ------------------------------------------------------------- host side ---
static void make_tables(std::vector<uint32_t> &slice, std::vector<uint32_t> &nib, std::vector<uint32_t> &xinv,
                        std::vector<uint32_t> &xa, std::vector<uint32_t> &xb, std::vector<uint32_t> &zrow,
                        std::vector<uint32_t> &zl) {
    slice.assign(4 * 256, 0);
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ kPoly : c >> 1;
        slice[n] = c;
    }
    for (int t = 1; t < 4; ++t)
        for (uint32_t n = 0; n < 256; ++n)
            slice[t * 256 + n] = (slice[(t - 1) * 256 + n] >> 8) ^ slice[slice[(t - 1) * 256 + n] & 0xff];
    nib.assign(64 * 8 * 16, 0);
    for (int l = 0; l < 64; ++l) {
        const uint32_t K = xpow8n((uint64_t)kSlab * (63 - l));
        for (int q = 0; q < 8; ++q)
            for (uint32_t v = 1; v < 16; ++v) nib[(l * 8 + q) * 16 + v] = multmodp(K, v << (4 * q));
    }
    uint32_t xinv8 = kX0;
    for (int i = 0; i < 8; ++i) xinv8 = multmodp(xinv8, kXinv);
    xinv.assign(kRow, 0);
    xinv[0] = kX0;
    for (int d = 1; d < kRow; ++d) xinv[d] = multmodp(xinv[d - 1], xinv8);
    xa.assign(65536, 0);
    xb.assign(65536, 0);
    xa[0] = xb[0] = kX0;
    const uint32_t s16 = xpow8n(65536), s1 = kX0 >> 8;
    for (int i = 1; i < 65536; ++i) {
        xa[i] = multmodp(xa[i - 1], s16);
        xb[i] = multmodp(xb[i - 1], s1);
    }
    const uint32_t x_row = xpow8n(kRow);
    zrow.assign(1024, 0);
    for (int k = 0; k < 4; ++k)
        for (uint32_t b = 1; b < 256; ++b) zrow[k * 256 + b] = multmodp(x_row, b << (8 * k));
    zl.assign(1u << 17, 0);  // crc32 of L zero bytes
    uint32_t st = 0xFFFFFFFFu;
    for (uint32_t L = 0; L < (1u << 17); ++L) {
        zl[L] = st ^ 0xFFFFFFFFu;
        st = slice[st & 0xff] ^ (st >> 8);
    }
}

static int ctx_init(Ctx *c, const gck_opts *o) {
    gck_opts d{};
    d.device = 0;
    d.chunk_bytes = 256 << 10;
    d.max_key = 65536;
    d.chunk_cap = 256;
    if (o) {
        d.device = o->device;
        if (o->chunk_bytes) d.chunk_bytes = o->chunk_bytes;
        if (o->max_key) d.max_key = o->max_key;
        if (o->chunk_cap) d.chunk_cap = o->chunk_cap;
        d.flags = o->flags;
    }
    if (d.chunk_bytes < 4096 || (d.chunk_bytes & (d.chunk_bytes - 1))) return GCK_EINVAL;
    c->opts = d;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= d.device || d.device < 0) {
        set_error("hipGetDeviceCount", hipErrorNoDevice, __FILE__, __LINE__);
        return GCK_EDEVICE;
    }
    GCK_HIP(hipSetDevice(d.device));
    hipDeviceProp_t prop;
    GCK_HIP(hipGetDeviceProperties(&prop, d.device));
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        set_error("device is not gfx950", hipErrorInvalidDevice, __FILE__, __LINE__);
        return GCK_EDEVICE;
    }
    c->device = d.device;
    c->n_cu = prop.multiProcessorCount;
    GCK_HIP(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    // the CRC stream carries the critical path of the pipelined run
    int prio_lo = 0, prio_hi = 0;
    GCK_HIP(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    GCK_HIP(hipStreamCreateWithPriority(&c->s_crc, hipStreamNonBlocking, prio_hi));
    GCK_HIP(hipStreamCreateWithFlags(&c->s_fin, hipStreamNonBlocking));
    for (auto &e : c->ev) GCK_HIP(hipEventCreate(&e));
    GCK_HIP(hipEventCreate(&c->ev_start));
    GCK_HIP(hipEventCreate(&c->ev_end));
    if (multmodp(kXinv, kX0 >> 1) != kX0) return GCK_EINVAL;
    std::vector<uint32_t> slice, nib, xinv, xa, xb, zrow, zl;
    make_tables(slice, nib, xinv, xa, xb, zrow, zl);
    int rc;
    if ((rc = c->d_slice.ensure(slice.size() * 4)) || (rc = c->d_nib.ensure(nib.size() * 4)) ||
        (rc = c->d_xinv.ensure(xinv.size() * 4)) || (rc = c->d_xa.ensure(xa.size() * 4)) ||
        (rc = c->d_xb.ensure(xb.size() * 4)) || (rc = c->d_zrow.ensure(zrow.size() * 4)) ||
        (rc = c->d_zl.ensure(zl.size() * 4)) || (rc = c->d_counters.ensure(64)))
        return rc;
    GCK_HIP(hipMemcpy(c->d_zrow.p, zrow.data(), zrow.size() * 4, hipMemcpyHostToDevice));
    GCK_HIP(hipMemcpy(c->d_zl.p, zl.data(), zl.size() * 4, hipMemcpyHostToDevice));
    GCK_HIP(hipMemcpy(c->d_slice.p, slice.data(), slice.size() * 4, hipMemcpyHostToDevice));
    GCK_HIP(hipMemcpy(c->d_nib.p, nib.data(), nib.size() * 4, hipMemcpyHostToDevice));
    GCK_HIP(hipMemcpy(c->d_xinv.p, xinv.data(), xinv.size() * 4, hipMemcpyHostToDevice));
    GCK_HIP(hipMemcpy(c->d_xa.p, xa.data(), xa.size() * 4, hipMemcpyHostToDevice));
    GCK_HIP(hipMemcpy(c->d_xb.p, xb.data(), xb.size() * 4, hipMemcpyHostToDevice));
    return GCK_OK;
}

static void ctx_free(Ctx *c) {
    DBuf *all[] = {&c->arena, &c->d_fbase, &c->d_flen, &c->d_ffirst, &c->d_fnch, &c->d_fbad, &c->d_fterm,
                   &c->d_ftpos, &c->d_fnrec, &c->d_ffirstrec, &c->d_carry, &c->d_ch_file, &c->d_ch_start,
                   &c->d_ch_end, &c->d_ch_entry, &c->d_ch_exit, &c->d_ch_count, &c->d_ch_term, &c->d_ch_tpos, &c->d_ch_bad,
                   &c->d_rec_base, &c->d_bsum, &c->d_scratch_off, &c->d_scratch_hdr, &c->d_counters, &c->d_rec_off,
                   &c->d_rec_hdr, &c->d_rec_file, &c->d_e, &c->d_pre, &c->d_out, &c->d_row_first, &c->d_rend, &c->d_plan, &c->d_big,
                   &c->d_slice, &c->d_nib, &c->d_xinv, &c->d_xa, &c->d_xb, &c->d_zrow, &c->d_zl,
                   &c->d_freset, &c->d_gbase, &c->d_gcarry, &c->d_gcnt, &c->d_bigcnt};
    for (DBuf *b : all) b->release();
    for (auto &e : c->ev)
        if (e) (void)hipEventDestroy(e);
    for (auto *v : {&c->ev_bnd, &c->ev_crc0, &c->ev_crc1, &c->ev_fin0, &c->ev_fin1}) {
        for (auto e : *v) (void)hipEventDestroy(e);
        v->clear();
    }
    if (c->ev_start) (void)hipEventDestroy(c->ev_start);
    if (c->ev_end) (void)hipEventDestroy(c->ev_end);
    for (hipStream_t *st : {&c->stream, &c->s_crc, &c->s_fin}) {
        if (*st) (void)hipStreamDestroy(*st);
        *st = nullptr;
    }
}

// Place files (walk order) in the arena and build the chunk table.
int ctx_layout(Ctx *c, const uint64_t *lens, uint32_t nfiles, const uint8_t *reset_after) {
    GCK_HIP(hipSetDevice(c->device));
    c->nfiles = nfiles;
    c->f_base.assign(nfiles, 0);
    c->f_len.assign(lens, lens + nfiles);
    c->f_reset.assign(reset_after, reset_after + nfiles);
    c->f_first_chunk.assign(nfiles, 0);
    c->f_nchunks.assign(nfiles, 0);
    uint64_t pos = 0, data = 0;
    const uint64_t CB = c->opts.chunk_bytes;
    std::vector<uint32_t> ch_file;
    std::vector<uint64_t> ch_start, ch_end;
    for (uint32_t f = 0; f < nfiles; ++f) {
        c->f_base[f] = pos;
        pos += (lens[f] + kRow - 1) / kRow * kRow;
        data += lens[f];
        c->f_first_chunk[f] = (uint32_t)ch_file.size();
        for (uint64_t s = 0; s < lens[f]; s += CB) {
            ch_file.push_back(f);
            ch_start.push_back(s);
            ch_end.push_back(s + CB < lens[f] ? s + CB : lens[f]);
        }
        c->f_nchunks[f] = (uint32_t)ch_file.size() - c->f_first_chunk[f];
    }
    if (ch_file.size() >= 0xFFFFFFF0ull) return GCK_EINVAL;
    c->arena_len = pos;
    c->data_bytes = data;
    c->n_rows = pos / kRow;
    c->n_chunks = (uint32_t)ch_file.size();
    const uint64_t nc = c->n_chunks, nf = nfiles ? nfiles : 1;
    const uint64_t cap = c->opts.chunk_cap;
    int rc;
    // slack past the last file: k_spec_entry reads up to three 4 KiB windows
    // (+80 B) beyond a chunk end
    const bool fresh = c->arena.cap < pos + 5 * kRow;
    if ((rc = c->arena.ensure(pos + 5 * kRow))) return rc;
    if (fresh) GCK_HIP(hipMemset(c->arena.p, 0, c->arena.cap));
    if ((rc = c->d_fbase.ensure(nf * 8)) || (rc = c->d_flen.ensure(nf * 8)) || (rc = c->d_ffirst.ensure(nf * 4)) ||
        (rc = c->d_fnch.ensure(nf * 4)) || (rc = c->d_fbad.ensure(nf * 4)) || (rc = c->d_fterm.ensure(nf * 4)) ||
        (rc = c->d_ftpos.ensure(nf * 8)) || (rc = c->d_fnrec.ensure(nf * 8)) ||
        (rc = c->d_ffirstrec.ensure(nf * 8)) || (rc = c->d_carry.ensure(nf * 4)) ||
        (rc = c->d_ch_file.ensure((nc + 1) * 4)) || (rc = c->d_ch_start.ensure((nc + 1) * 8)) ||
        (rc = c->d_ch_end.ensure((nc + 1) * 8)) || (rc = c->d_ch_entry.ensure((nc + 1) * 8)) ||
        (rc = c->d_ch_exit.ensure((nc + 1) * 8)) || (rc = c->d_ch_count.ensure((nc + 1) * 4)) ||
        (rc = c->d_ch_term.ensure((nc + 1) * 4)) || (rc = c->d_ch_tpos.ensure((nc + 1) * 8)) || (rc = c->d_ch_bad.ensure((nc + 1) * 4)) ||
        (rc = c->d_rec_base.ensure((nc + 1) * 8)) || (rc = c->d_bsum.ensure((nc / kScanBlock + nf + 2) * 8)) || (rc = c->d_freset.ensure(nf * 4)) ||
        (rc = c->d_gbase.ensure(16)) || (rc = c->d_scratch_off.ensure((nc + 1) * cap * 8)) ||
        (rc = c->d_scratch_hdr.ensure((nc + 1) * cap * 16)) || (rc = c->d_row_first.ensure((c->n_rows + 1) * 4)) ||
        (rc = c->d_rend.ensure((c->n_rows + 1) * 4)) || (rc = c->d_plan.ensure((c->n_rows + 1) * 64)) || (rc = c->d_big.ensure((c->n_rows + 1) * 4)) ||
        (rc = c->d_bigcnt.ensure((c->n_rows / 64 + kMaxGroups + 2) * 4)))
        return rc;
    if (nfiles) {
        GCK_HIP(hipMemcpy(c->d_fbase.p, c->f_base.data(), nfiles * 8, hipMemcpyHostToDevice));
        GCK_HIP(hipMemcpy(c->d_flen.p, c->f_len.data(), nfiles * 8, hipMemcpyHostToDevice));
        GCK_HIP(hipMemcpy(c->d_ffirst.p, c->f_first_chunk.data(), nfiles * 4, hipMemcpyHostToDevice));
        GCK_HIP(hipMemcpy(c->d_fnch.p, c->f_nchunks.data(), nfiles * 4, hipMemcpyHostToDevice));
        std::vector<uint32_t> rs(reset_after, reset_after + nfiles);
        GCK_HIP(hipMemcpy(c->d_freset.p, rs.data(), nfiles * 4, hipMemcpyHostToDevice));
    }
    if (nc) {
        GCK_HIP(hipMemcpy(c->d_ch_file.p, ch_file.data(), nc * 4, hipMemcpyHostToDevice));
        GCK_HIP(hipMemcpy(c->d_ch_start.p, ch_start.data(), nc * 8, hipMemcpyHostToDevice));
        GCK_HIP(hipMemcpy(c->d_ch_end.p, ch_end.data(), nc * 8, hipMemcpyHostToDevice));
    }
    return GCK_OK;
}

static inline uint32_t nblk(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }

// Counter slots (d_counters, u32): 1 fixups, 2 chunks whose stage overflowed
// (re-walked by k_compact), 3 CRC rejects, 5 big rows (sync path), 6 record-
// table capacity overflow (pipelined path), 8.. validation rounds (sync path),
// 15 host validation loop.
enum : int { CNT_FIXUP = 1, CNT_STAGE = 2, CNT_REJECT = 3, CNT_BIG = 5, CNT_CAP = 6, CNT_VAL = 8, CNT_HOSTVAL = 15 };
// Per-group counter slots (d_gcnt, 8 x u32 per group).
enum : int { G_BIG = 0, G_VAL = 1 };  // G_VAL + round: validation rounds, the last one must be 0
constexpr int kRounds = 2;             // device validation/fixup rounds

// Boundary discovery for chunks [c0, c1): speculative entries, chain walks,
// kRounds validate/fixup rounds and a final validation counted at val_cnt[kRounds].
static void launch_boundary(Ctx *c, hipStream_t s, uint32_t c0, uint32_t c1, uint32_t *val_cnt) {
    const uint32_t n = c1 - c0, cap = c->opts.chunk_cap;
    if (!n) return;
    k_spec_entry<<<nblk(n, 4), 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(), c->d_flen.as<uint64_t>(),
                                            c->d_ch_file.as<uint32_t>() + c0, c->d_ch_start.as<uint64_t>() + c0,
                                            c->d_ch_end.as<uint64_t>() + c0, c->d_ch_entry.as<uint64_t>() + c0, n,
                                            c->opts.max_key);
    k_walk<<<nblk(n, 256), 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(), c->d_flen.as<uint64_t>(),
                                        c->d_ch_file.as<uint32_t>() + c0, c->d_ch_end.as<uint64_t>() + c0,
                                        c->d_ch_entry.as<uint64_t>() + c0, c->d_ch_count.as<uint32_t>() + c0,
                                        c->d_ch_exit.as<uint64_t>() + c0, c->d_ch_term.as<uint32_t>() + c0,
                                        c->d_ch_tpos.as<uint64_t>() + c0,
                                        c->d_scratch_off.as<uint64_t>() + (uint64_t)c0 * cap,
                                        c->d_scratch_hdr.as<uint4>() + (uint64_t)c0 * cap, cap, n);
    for (int r = 0; r <= kRounds; ++r) {
        k_validate<<<nblk(n, 256), 256, 0, s>>>(c->d_ch_file.as<uint32_t>(), c->d_ch_start.as<uint64_t>(),
                                                c->d_ch_end.as<uint64_t>(), c->d_ch_entry.as<uint64_t>(),
                                                c->d_ch_exit.as<uint64_t>(), c->d_ch_term.as<uint32_t>(),
                                                c->d_ffirst.as<uint32_t>(), c->d_ch_bad.as<uint32_t>(), val_cnt + r, c0,
                                                c1);
        if (r == kRounds) break;
        k_fixup<<<nblk(n, 256), 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(),
                                             c->d_flen.as<uint64_t>(), c->d_ch_file.as<uint32_t>(),
                                             c->d_ch_end.as<uint64_t>(), c->d_ffirst.as<uint32_t>(),
                                             c->d_ch_bad.as<uint32_t>(), c->d_ch_entry.as<uint64_t>(),
                                             c->d_ch_count.as<uint32_t>(), c->d_ch_exit.as<uint64_t>(),
                                             c->d_ch_term.as<uint32_t>(), c->d_ch_tpos.as<uint64_t>(),
                                             c->d_scratch_off.as<uint64_t>(), c->d_scratch_hdr.as<uint4>(), cap, c0, c1,
                                             c->d_counters.as<uint32_t>() + CNT_FIXUP);
    }
}

// Record slots of chunks [c0, c1) after the records of earlier groups
// (gbase[0] -> gbase[1]), and the summary of files [f0, f1).
static void launch_scan(Ctx *c, hipStream_t s, uint32_t c0, uint32_t c1, uint32_t f0, uint32_t f1, uint64_t *gbase,
                        uint64_t cap) {
    const uint32_t n = c1 - c0, nb = nblk(n, kScanBlock);
    uint64_t *bsum = c->d_bsum.as<uint64_t>() + c0 / kScanBlock + f0;  // disjoint per group
    if (nb) k_scan_local<<<nb, 64, 0, s>>>(c->d_ch_count.as<uint32_t>() + c0, c->d_rec_base.as<uint64_t>() + c0, bsum, n);
    k_scan_top<<<1, 64, 0, s>>>(bsum, nb, gbase, gbase + 1, c->d_rec_base.as<uint64_t>() + c0, n, cap,
                                c->d_counters.as<uint32_t>() + CNT_CAP);
    if (n) k_scan_add<<<nblk(n, 256), 256, 0, s>>>(c->d_rec_base.as<uint64_t>() + c0, bsum, n);
    if (f1 > f0)
        k_file_summary<<<nblk(f1 - f0, 64), 64, 0, s>>>(
            c->d_ffirst.as<uint32_t>() + f0, c->d_fnch.as<uint32_t>() + f0, c->d_rec_base.as<uint64_t>(),
            c->d_ch_entry.as<uint64_t>(), c->d_ch_term.as<uint32_t>(), c->d_ch_tpos.as<uint64_t>(),
            c->d_fterm.as<uint32_t>() + f0, c->d_ftpos.as<uint64_t>() + f0, c->d_ffirstrec.as<uint64_t>() + f0,
            c->d_fnrec.as<uint64_t>() + f0, f1 - f0);
}

// Record table of chunks [c0, c1), row index and row plan of rows [r0, r1).
// Slow-row lists of rows [r0, r1): list slots d_big + r0, per-64-row counts at
// d_bigcnt + (r0 / 64 + g) (disjoint per file group g), any-flag big_any.
static uint32_t *big_counts(Ctx *c, uint64_t r0, uint32_t g) { return c->d_bigcnt.as<uint32_t>() + r0 / 64 + g; }

static void launch_records(Ctx *c, hipStream_t s, uint32_t c0, uint32_t c1, uint64_t r0, uint64_t r1,
                           const uint64_t *rng, uint64_t cap, uint32_t g, uint32_t *big_any) {
    const uint32_t n = c1 - c0, ccap = c->opts.chunk_cap;
    if (n)
        k_compact<<<nblk(n, 4), 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(), c->d_flen.as<uint64_t>(),
                                             c->d_ch_file.as<uint32_t>() + c0, c->d_ch_end.as<uint64_t>() + c0,
                                             c->d_ch_entry.as<uint64_t>() + c0, c->d_ch_count.as<uint32_t>() + c0,
                                             c->d_rec_base.as<uint64_t>() + c0,
                                             c->d_scratch_off.as<uint64_t>() + (uint64_t)c0 * ccap,
                                             c->d_scratch_hdr.as<uint4>() + (uint64_t)c0 * ccap, ccap, n, cap,
                                             c->d_rec_off.as<uint64_t>(), c->d_rec_hdr.as<uint4>(),
                                             c->d_rec_file.as<uint32_t>(), c->d_counters.as<uint32_t>());
    const uint32_t grid = (uint32_t)c->n_cu * 4;
    k_row_fill<<<grid, 256, 0, s>>>(c->d_row_first.as<uint32_t>(), r0, r1, rng);
    k_row_index<<<grid, 256, 0, s>>>(c->d_rec_off.as<uint64_t>(), c->d_rec_hdr.as<uint4>(), rng, r0,
                                     c->d_row_first.as<uint32_t>());
    if (r1 > r0)
        k_row_plan<<<nblk(r1 - r0, 64 * kPlanWaves), 64 * kPlanWaves, 0, s>>>(
            c->d_rec_off.as<uint64_t>(), c->d_rec_hdr.as<uint4>(), rng, r0, r1 - r0, c->d_row_first.as<uint32_t>(),
            c->d_plan.as<uint4>(), c->d_big.as<uint32_t>() + r0, big_counts(c, r0, g), big_any);
}

// CRC partials of rows [r0, r1): k_crc_rows, then k_crc_rows_big on the rows
// k_row_plan listed.  e/pre scratch slot: cap; rend scratch: row n_rows.
static void launch_crc(Ctx *c, hipStream_t s, uint64_t r0, uint64_t r1, const uint64_t *rng, uint64_t cap,
                       uint32_t g, const uint32_t *big_any, hipEvent_t between = nullptr) {
    if (r1 <= r0) return;
    const uint64_t nr = r1 - r0, want = (nr + kWaves * kRowsPerStep - 1) / (kWaves * kRowsPerStep);
    const uint32_t grid = (uint32_t)(want < (uint64_t)c->n_cu ? want : (uint64_t)c->n_cu);
    k_crc_rows<0, kDepth, kRowsPerStep><<<grid, 1024, 0, s>>>(c->arena.as<uint8_t>() + r0 * kRow, nr,
                                                c->d_plan.as<uint8_t>() + r0 * kPlanBytes, cap,
                                                c->d_slice.as<uint32_t>(), c->d_nib.as<uint32_t>(),
                                                c->d_e.as<uint32_t>(), c->d_pre.as<uint32_t>(),
                                                c->d_rend.as<uint32_t>() + r0, c->d_rend.as<uint32_t>() + c->n_rows);
    if (between) (void)hipEventRecord(between, s);
    k_crc_rows_big<0><<<c->n_cu, 1024, 0, s>>>(c->arena.as<uint8_t>(), c->d_big.as<uint32_t>() + r0,
                                              big_counts(c, r0, g), big_any, (uint32_t)((nr + 63) / 64),
                                              c->d_row_first.as<uint32_t>(), rng, c->d_rec_off.as<uint64_t>(),
                                              c->d_rec_hdr.as<uint4>(), c->d_slice.as<uint32_t>(),
                                              c->d_nib.as<uint32_t>(), c->d_e.as<uint32_t>(), c->d_pre.as<uint32_t>(),
                                              c->d_rend.as<uint32_t>());
}

static void launch_finalize(Ctx *c, hipStream_t s, const uint64_t *rng, uint64_t max_recs) {
    if (!max_recs) return;
    const uint64_t want = nblk(max_recs, 256);
    const uint32_t grid = (uint32_t)(want < (uint64_t)c->n_cu * 8 ? want : (uint64_t)c->n_cu * 8);
    k_finalize<<<grid, 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_rec_off.as<uint64_t>(), c->d_rec_hdr.as<uint4>(),
                                    c->d_rec_file.as<uint32_t>(), c->d_fbase.as<uint64_t>(), c->d_carry.as<uint32_t>(),
                                    rng, c->d_e.as<uint32_t>(), c->d_pre.as<uint32_t>(), c->d_rend.as<uint32_t>(),
                                    c->d_slice.as<uint32_t>(), c->d_xinv.as<uint32_t>(), c->d_zrow.as<uint32_t>(),
                                    c->d_zl.as<uint32_t>(), c->d_xa.as<uint32_t>(), c->d_xb.as<uint32_t>(),
                                    c->d_out.as<gck_rec>(), c->d_counters.as<uint32_t>());
}

static int ensure_records(Ctx *c, uint64_t nr) {
    nr = nr ? nr : 1;
    int rc;
    if ((rc = c->d_rec_off.ensure(nr * 8)) || (rc = c->d_rec_hdr.ensure(nr * 16)) ||
        (rc = c->d_rec_file.ensure(nr * 4)) || (rc = c->d_e.ensure((nr + 65) * 4)) ||
        (rc = c->d_pre.ensure((nr + 65) * 4)) || (rc = c->d_out.ensure(nr * sizeof(gck_rec))))
        return rc;
    return GCK_OK;
}

// Host bookkeeping from the per-file summaries (core/db.go:110-140): status,
// files walked, final lastOffset, records in walk order; carries if asked.
static uint64_t account_files(Ctx *c, const std::vector<uint32_t> &fterm, const std::vector<uint64_t> &ftpos,
                              const std::vector<uint64_t> &ffirst, const std::vector<uint64_t> &fnrec,
                              std::vector<uint32_t> *carry) {
    const uint32_t nf = c->nfiles;
    c->status = GCK_OK;
    c->err_file = 0;
    c->err_off = 0;
    c->files_walked = nf;
    uint64_t n_total = 0;
    uint32_t last = 0;  // keyDir.lastOffset at the start of each file
    for (uint32_t f = 0; f < nf; ++f) {
        if (carry) (*carry)[f] = last;
        const uint64_t valid = fterm[f] != T_NONE ? ftpos[f] : c->f_len[f];
        n_total = ffirst[f] + fnrec[f];
        last += (uint32_t)valid;
        if (fterm[f] == T_ERR) {  // walkFile error aborts filepath.Walk (disk.go:134-141)
            c->status = GCK_EUNEXPECTED_EOF;
            c->err_file = f;
            c->err_off = ftpos[f];
            c->files_walked = f + 1;
            break;
        }
        if (c->f_reset[f]) last = 0;  // resetOffset (core/db.go:117-119)
    }
    c->final_last_offset = last;
    return n_total;
}

static int read_file_summaries(Ctx *c, hipStream_t s, std::vector<uint32_t> &fterm, std::vector<uint64_t> &ftpos,
                               std::vector<uint64_t> &ffirst, std::vector<uint64_t> &fnrec) {
    const uint32_t nf = c->nfiles;
    fterm.assign(nf, 0);
    ftpos.assign(nf, 0);
    ffirst.assign(nf, 0);
    fnrec.assign(nf, 0);
    if (nf) {
        GCK_HIP(hipMemcpyAsync(fterm.data(), c->d_fterm.p, nf * 4, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipMemcpyAsync(ftpos.data(), c->d_ftpos.p, nf * 8, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipMemcpyAsync(ffirst.data(), c->d_ffirstrec.p, nf * 8, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipMemcpyAsync(fnrec.data(), c->d_fnrec.p, nf * 8, hipMemcpyDeviceToHost, s));
    }
    return GCK_OK;
}

// The synchronous pipeline: every phase over all files, one host round trip
// after the boundary phases (exact record count, EOF verdicts, carries).
// Used for single-file corpora and as the fallback of the pipelined run.
static int ctx_run_sync(Ctx *c) {
    const auto t0 = std::chrono::steady_clock::now();
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint32_t nc = c->n_chunks, nf = c->nfiles;
    uint32_t *cnt = c->d_counters.as<uint32_t>();
    uint64_t *gbase = c->d_gbase.as<uint64_t>();
    GCK_HIP(hipMemsetAsync(cnt, 0, 64, s));
    GCK_HIP(hipMemsetAsync(gbase, 0, 16, s));
    GCK_HIP(hipMemsetAsync(c->d_row_first.p, 0, 4, s));
    GCK_HIP(hipEventRecord(c->ev[PH_BOUNDARY], s));
    launch_boundary(c, s, 0, nc, cnt + CNT_VAL);
    GCK_HIP(hipEventRecord(c->ev[PH_SCAN], s));
    const uint64_t big_cap = ~0ull >> 1;
    launch_scan(c, s, 0, nc, 0, nf, gbase, big_cap);
    GCK_HIP(hipEventRecord(c->ev[PH_HOST], s));

    std::vector<uint32_t> fterm, carry(nf);
    std::vector<uint64_t> ftpos, ffirst, fnrec;
    if (read_file_summaries(c, s, fterm, ftpos, ffirst, fnrec)) return GCK_EDEVICE;
    uint32_t hcnt[16] = {};
    GCK_HIP(hipMemcpyAsync(hcnt, cnt, 64, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    // rare: inconsistencies left after the device rounds (cascading mis-speculation)
    for (uint32_t left = hcnt[CNT_VAL + kRounds]; left;) {
        k_fixup<<<nblk(nc, 256), 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(),
                                              c->d_flen.as<uint64_t>(), c->d_ch_file.as<uint32_t>(),
                                              c->d_ch_end.as<uint64_t>(), c->d_ffirst.as<uint32_t>(),
                                              c->d_ch_bad.as<uint32_t>(), c->d_ch_entry.as<uint64_t>(),
                                              c->d_ch_count.as<uint32_t>(), c->d_ch_exit.as<uint64_t>(),
                                              c->d_ch_term.as<uint32_t>(), c->d_ch_tpos.as<uint64_t>(),
                                              c->d_scratch_off.as<uint64_t>(), c->d_scratch_hdr.as<uint4>(),
                                              c->opts.chunk_cap, 0u, nc, cnt + CNT_FIXUP);
        GCK_HIP(hipMemsetAsync(cnt + CNT_HOSTVAL, 0, 4, s));
        k_validate<<<nblk(nc, 256), 256, 0, s>>>(c->d_ch_file.as<uint32_t>(), c->d_ch_start.as<uint64_t>(),
                                                 c->d_ch_end.as<uint64_t>(), c->d_ch_entry.as<uint64_t>(),
                                                 c->d_ch_exit.as<uint64_t>(), c->d_ch_term.as<uint32_t>(),
                                                 c->d_ffirst.as<uint32_t>(), c->d_ch_bad.as<uint32_t>(),
                                                 cnt + CNT_HOSTVAL, 0u, nc);
        uint32_t v = 0;
        GCK_HIP(hipMemcpyAsync(&v, cnt + CNT_HOSTVAL, 4, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipStreamSynchronize(s));
        left = v;
        if (!left) {
            launch_scan(c, s, 0, nc, 0, nf, gbase, big_cap);
            if (read_file_summaries(c, s, fterm, ftpos, ffirst, fnrec)) return GCK_EDEVICE;
            GCK_HIP(hipMemcpyAsync(hcnt, cnt, 64, hipMemcpyDeviceToHost, s));
            GCK_HIP(hipStreamSynchronize(s));
        }
    }
    c->n_fixups = hcnt[CNT_FIXUP];
    const uint64_t n_total = account_files(c, fterm, ftpos, ffirst, fnrec, &carry);
    c->n_recs = n_total;
    if (n_total > 0xFFFFFFF0ull) return GCK_EINVAL;
    int rc;
    if ((rc = ensure_records(c, n_total))) return rc;
    c->rec_cap = n_total;
    const uint64_t rng_h[2] = {0, n_total};
    if (nf) GCK_HIP(hipMemcpyAsync(c->d_carry.p, carry.data(), nf * 4, hipMemcpyHostToDevice, s));
    GCK_HIP(hipMemcpyAsync(gbase, rng_h, 16, hipMemcpyHostToDevice, s));

    GCK_HIP(hipEventRecord(c->ev[PH_RECORDS], s));
    launch_records(c, s, 0, nc, 0, c->n_rows, gbase, n_total, 0, cnt + CNT_BIG);
    GCK_HIP(hipEventRecord(c->ev[PH_CRC], s));
    if (n_total) launch_crc(c, s, 0, c->n_rows, gbase, n_total, 0, cnt + CNT_BIG, c->ev[PH_CRCBIG]);
    else GCK_HIP(hipEventRecord(c->ev[PH_CRCBIG], s));
    GCK_HIP(hipEventRecord(c->ev[PH_FINAL], s));
    launch_finalize(c, s, gbase, n_total);
    GCK_HIP(hipEventRecord(c->ev[PH_END], s));
    GCK_HIP(hipMemcpyAsync(hcnt, cnt, 16, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    GCK_HIP(hipGetLastError());
    c->n_overflow = hcnt[CNT_STAGE];
    c->n_crc_fail = hcnt[CNT_REJECT];
    for (int p = 0; p < PH_NPHASE; ++p) c->ms_phase[p] = 0;
    for (int p = PH_BOUNDARY; p < PH_END; ++p) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, c->ev[p], c->ev[p + 1]);
        c->ms_phase[p] = ms;
    }
    float span = 0;
    (void)hipEventElapsedTime(&span, c->ev[PH_BOUNDARY], c->ev[PH_END]);
    c->ms_phase[PH_PIPE] = span;
    c->pipelined = false;
    c->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return c->status;
}

// File groups of the pipelined run: consecutive files in walk order,
// balanced by bytes, at most kMaxGroups.
static void make_groups(Ctx *c) {
    const uint32_t nf = c->nfiles;
    c->g_file.clear();
    const uint32_t G = nf < (uint32_t)kMaxGroups ? nf : (uint32_t)kMaxGroups;
    c->g_file.push_back(0);
    uint64_t acc = 0;
    for (uint32_t f = 0; f < nf; ++f) {
        acc += c->f_len[f];
        const uint32_t g = (uint32_t)c->g_file.size();  // groups closed so far + 1
        if (f + 1 < nf && g < G && acc * G >= c->data_bytes * g) c->g_file.push_back(f + 1);
    }
    c->g_file.push_back(nf);
}

// The pipelined run: file groups go through boundary discovery, record table
// and row plan on stream s (in walk order, record bases and lastOffset
// carried on the device), CRC rows on c->s_crc and finalize on c->s_fin, so
// group g's CRC overlaps group g+1's boundary work and group g-1's finalize.
// No host round trip until the end; anything unusual (validation not settled
// after kRounds, record-table capacity, a startup error) reruns synchronously.
static int ctx_run_pipe(Ctx *c) {
    const auto t0 = std::chrono::steady_clock::now();
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint32_t nf = c->nfiles, G = (uint32_t)c->g_file.size() - 1;
    uint32_t *cnt = c->d_counters.as<uint32_t>();
    uint64_t *gbase = c->d_gbase.as<uint64_t>();
    uint32_t *gcarry = c->d_gcarry.as<uint32_t>();
    uint32_t *gcnt = c->d_gcnt.as<uint32_t>();
    const uint64_t cap = c->rec_cap;
    GCK_HIP(hipMemsetAsync(cnt, 0, 64, s));
    GCK_HIP(hipMemsetAsync(gbase, 0, (G + 1) * 8, s));
    GCK_HIP(hipMemsetAsync(gcarry, 0, (G + 1) * 4, s));
    GCK_HIP(hipMemsetAsync(gcnt, 0, G * 32, s));
    GCK_HIP(hipMemsetAsync(c->d_row_first.p, 0, 4, s));
    GCK_HIP(hipEventRecord(c->ev_start, s));
    for (uint32_t g = 0; g < G; ++g) {
        const uint32_t f0 = c->g_file[g], f1 = c->g_file[g + 1];
        const uint32_t c0 = c->f_first_chunk[f0], c1 = f1 < nf ? c->f_first_chunk[f1] : c->n_chunks;
        const uint64_t r0 = c->f_base[f0] / kRow, r1 = f1 < nf ? c->f_base[f1] / kRow : c->n_rows;
        launch_boundary(c, s, c0, c1, gcnt + g * 8 + G_VAL);
        launch_scan(c, s, c0, c1, f0, f1, gbase + g, cap);
        k_group_carry<<<1, 1, 0, s>>>(f1 - f0, c->d_flen.as<uint64_t>() + f0, c->d_freset.as<uint32_t>() + f0,
                                      c->d_fterm.as<uint32_t>() + f0, c->d_ftpos.as<uint64_t>() + f0,
                                      c->d_carry.as<uint32_t>() + f0, gcarry + g, gcarry + g + 1);
        launch_records(c, s, c0, c1, r0, r1, gbase + g, cap, g, gcnt + g * 8 + G_BIG);
        GCK_HIP(hipEventRecord(c->ev_bnd[g], s));
        GCK_HIP(hipStreamWaitEvent(c->s_crc, c->ev_bnd[g], 0));
        GCK_HIP(hipEventRecord(c->ev_crc0[g], c->s_crc));
        launch_crc(c, c->s_crc, r0, r1, gbase + g, cap, g, gcnt + g * 8 + G_BIG);
        GCK_HIP(hipEventRecord(c->ev_crc1[g], c->s_crc));
        GCK_HIP(hipStreamWaitEvent(c->s_fin, c->ev_crc1[g], 0));
        GCK_HIP(hipEventRecord(c->ev_fin0[g], c->s_fin));
        launch_finalize(c, c->s_fin, gbase + g, (uint64_t)(c1 - c0) * c->opts.chunk_cap);
        GCK_HIP(hipEventRecord(c->ev_fin1[g], c->s_fin));
    }
    std::vector<uint32_t> fterm, gc(G * 8);
    std::vector<uint64_t> ftpos, ffirst, fnrec;
    if (read_file_summaries(c, c->s_fin, fterm, ftpos, ffirst, fnrec)) return GCK_EDEVICE;
    uint32_t hcnt[16] = {};
    GCK_HIP(hipMemcpyAsync(hcnt, cnt, 64, hipMemcpyDeviceToHost, c->s_fin));
    GCK_HIP(hipMemcpyAsync(gc.data(), gcnt, G * 32, hipMemcpyDeviceToHost, c->s_fin));
    GCK_HIP(hipEventRecord(c->ev_end, c->s_fin));
    GCK_HIP(hipStreamSynchronize(c->s_fin));
    GCK_HIP(hipGetLastError());
    bool settled = hcnt[CNT_CAP] == 0;
    for (uint32_t g = 0; g < G; ++g) settled &= gc[g * 8 + G_VAL + kRounds] == 0;
    const uint64_t n_total = account_files(c, fterm, ftpos, ffirst, fnrec, nullptr);
    if (!settled || c->status != GCK_OK || n_total > 0xFFFFFFF0ull) {
        ++c->n_sync_reruns;
        return ctx_run_sync(c);
    }
    c->n_recs = n_total;
    c->n_fixups = hcnt[CNT_FIXUP];
    c->n_overflow = hcnt[CNT_STAGE];
    c->n_crc_fail = hcnt[CNT_REJECT];
    for (int p = 0; p < PH_NPHASE; ++p) c->ms_phase[p] = 0;
    for (uint32_t g = 0; g < G; ++g) {
        float a = 0, b = 0;
        (void)hipEventElapsedTime(&a, c->ev_crc0[g], c->ev_crc1[g]);
        (void)hipEventElapsedTime(&b, c->ev_fin0[g], c->ev_fin1[g]);
        c->ms_phase[PH_CRC] += a;
        c->ms_phase[PH_FINAL] += b;
    }
    float span = 0;
    (void)hipEventElapsedTime(&span, c->ev_start, c->ev_end);
    c->ms_phase[PH_PIPE] = span;
    c->pipelined = true;
    c->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return GCK_OK;
}

static int ctx_run(Ctx *c) {
    const bool pipe = c->nfiles >= 2 && (c->opts.flags & GCK_OPT_PIPELINE);
    if (!pipe) return ctx_run_sync(c);
    GCK_HIP(hipSetDevice(c->device));
    make_groups(c);
    const uint32_t G = (uint32_t)c->g_file.size() - 1;
    // record-table capacity: the stage bound (chunk_cap per chunk) or the last
    // exact count, whichever is larger; beyond it the run reruns synchronously
    const uint64_t want = std::max<uint64_t>((uint64_t)c->n_chunks * c->opts.chunk_cap, c->n_recs);
    int rc;
    if ((rc = ensure_records(c, want)) || (rc = c->d_gbase.ensure((G + 1) * 8)) ||
        (rc = c->d_gcarry.ensure((G + 1) * 4)) || (rc = c->d_gcnt.ensure(G * 32)))
        return rc;
    c->rec_cap = want;
    while (c->ev_bnd.size() < G) {
        hipEvent_t e[5];
        for (auto &x : e) GCK_HIP(hipEventCreate(&x));
        c->ev_bnd.push_back(e[0]);
        c->ev_crc0.push_back(e[1]);
        c->ev_crc1.push_back(e[2]);
        c->ev_fin0.push_back(e[3]);
        c->ev_fin1.push_back(e[4]);
    }
    return ctx_run_pipe(c);
}

}  // namespace gck

using namespace gck;

extern "C" {

int gck_ctx_create(const gck_opts *opts, gck_ctx **out) {
    if (!out) return GCK_EINVAL;
    *out = nullptr;
    gck_ctx *c = new (std::nothrow) gck_ctx();
    if (!c) return GCK_ENOMEM;
    int rc = ctx_init(&c->c, opts);
    if (rc) {
        ctx_free(&c->c);
        delete c;
        return rc;
    }
    *out = c;
    return GCK_OK;
}

void gck_ctx_destroy(gck_ctx *ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->c.device);
    ctx_free(&ctx->c);
    delete ctx;
}

int gck_ctx_load(gck_ctx *ctx, const gck_file *files, uint32_t nfiles) {
    if (!ctx || (nfiles && !files)) return GCK_EINVAL;
    std::vector<uint64_t> lens(nfiles);
    std::vector<uint8_t> reset(nfiles);
    for (uint32_t f = 0; f < nfiles; ++f) {
        if (files[f].len && !files[f].data) return GCK_EINVAL;
        lens[f] = files[f].len;
        reset[f] = files[f].reset_after ? 1 : 0;
    }
    int rc = ctx_layout(&ctx->c, lens.data(), nfiles, reset.data());
    if (rc) return rc;
    for (uint32_t f = 0; f < nfiles; ++f)
        if (files[f].len)
            GCK_HIP(hipMemcpy(ctx->c.arena.as<uint8_t>() + ctx->c.f_base[f], files[f].data, files[f].len,
                              hipMemcpyHostToDevice));
    return GCK_OK;
}

int gck_ctx_run(gck_ctx *ctx) {
    if (!ctx) return GCK_EINVAL;
    return ctx_run(&ctx->c);
}

int gck_ctx_fetch(gck_ctx *ctx, gck_result *out) {
    if (!ctx || !out) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    memset(out, 0, sizeof(*out));
    out->n = c->n_recs;
    out->n_crc_fail = c->n_crc_fail;
    out->final_last_offset = c->final_last_offset;
    out->status = c->status;
    out->err_file = c->err_file;
    out->err_off = c->err_off;
    out->files_walked = c->files_walked;
    if (c->n_recs) {
        out->recs = static_cast<gck_rec *>(malloc(c->n_recs * sizeof(gck_rec)));
        if (!out->recs) return GCK_ENOMEM;
        GCK_HIP(hipSetDevice(c->device));
        GCK_HIP(hipMemcpy(out->recs, c->d_out.p, c->n_recs * sizeof(gck_rec), hipMemcpyDeviceToHost));
    }
    return GCK_OK;
}

int gck_ctx_stats(gck_ctx *ctx, gck_stats *out) {
    if (!ctx || !out) return GCK_EINVAL;
    const Ctx *c = &ctx->c;
    memset(out, 0, sizeof(*out));
    out->bytes = c->data_bytes;
    out->n_recs = c->n_recs;
    out->n_crc_fail = c->n_crc_fail;
    out->n_chunks = c->n_chunks;
    out->n_fixups = c->n_fixups;
    out->n_overflow = c->n_overflow;
    out->ms_total = c->ms_total;
    for (int p = 0; p < PH_NPHASE && p < 12; ++p) out->ms_kernel[p] = c->ms_phase[p];
    out->pipelined = c->pipelined ? 1u : 0u;
    out->n_sync_reruns = c->n_sync_reruns;
    return GCK_OK;
}

const char *gck_phase_name(int phase) {
    static const char *names[] = {"boundary", "scan",     "host_sync", "records",
                                  "crc_rows", "crc_big", "finalize",  "pipeline"};
    return phase >= 0 && phase < PH_NPHASE ? names[phase] : "";
}

int gck_ctx_device_recs(gck_ctx *ctx, const gck_rec **recs, uint64_t *n) {
    if (!ctx || !recs || !n) return GCK_EINVAL;
    *recs = ctx->c.d_out.as<gck_rec>();
    *n = ctx->c.n_recs;
    return GCK_OK;
}

void *gck_ctx_stream(gck_ctx *ctx) { return ctx ? (void *)ctx->c.stream : nullptr; }

int gck_ctx_read_file(gck_ctx *ctx, uint32_t file, uint64_t off, uint8_t *dst, uint64_t len) {
    if (!ctx || file >= ctx->c.nfiles || off + len > ctx->c.f_len[file]) return GCK_EINVAL;
    GCK_HIP(hipSetDevice(ctx->c.device));
    GCK_HIP(hipMemcpy(dst, ctx->c.arena.as<uint8_t>() + ctx->c.f_base[file] + off, len, hipMemcpyDeviceToHost));
    return GCK_OK;
}

int gck_replay(const gck_file *files, uint32_t nfiles, const gck_opts *opts, gck_result *out) {
    if (!out) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    gck_ctx *ctx = nullptr;
    int rc = gck_ctx_create(opts, &ctx);
    if (rc) return rc;
    rc = gck_ctx_load(ctx, files, nfiles);
    if (!rc) {
        rc = gck_ctx_run(ctx);
        if (rc == GCK_OK || rc == GCK_EUNEXPECTED_EOF) {
            const int frc = gck_ctx_fetch(ctx, out);
            if (frc) rc = frc;
        }
    }
    gck_ctx_destroy(ctx);
    return rc;
}

void gck_result_free(gck_result *res) {
    if (!res) return;
    free(res->recs);
    res->recs = nullptr;
    res->n = 0;
}

int gck_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *gck_version(void) { return "gocask_hip 0.1 (gfx950)"; }

const char *gck_last_error(void) { return gck::last_error(); }

// Measurement helper: time ablated variants of k_crc_rows on the state left by
// the last gck_ctx_run (outputs are clobbered; rerun before fetching).
// mode bits: 1 = no record intervals, 2 = no LDS table chain, 4 = no tail
// shift / segmented scan.
int gck_diag_crc_variant(gck_ctx *ctx, int mode, int iters, double *ms_per_iter) {
    if (!ctx || iters <= 0 || mode < 0 || mode > 15) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    if (!c->n_rows || !c->n_recs) return GCK_EINVAL;
    GCK_HIP(hipSetDevice(c->device));
    const uint64_t want = (c->n_rows + kWaves * kRowsPerStep - 1) / (kWaves * kRowsPerStep);
    const uint32_t grid = (uint32_t)(want < (uint64_t)c->n_cu ? want : (uint64_t)c->n_cu);
    hipEvent_t a, b;
    GCK_HIP(hipEventCreate(&a));
    GCK_HIP(hipEventCreate(&b));
    GCK_HIP(hipEventRecord(a, c->stream));
    for (int i = 0; i < iters; ++i) {
#define GCK_VARIANT(M)                                                                                              \
    case M:                                                                                                         \
        k_crc_rows<M, kDepth, kRowsPerStep><<<grid, 1024, 0, c->stream>>>(c->arena.as<uint8_t>(), c->n_rows, c->d_plan.as<uint8_t>(), \
                                                    c->n_recs, c->d_slice.as<uint32_t>(), c->d_nib.as<uint32_t>(),      \
                                                    c->d_e.as<uint32_t>(), c->d_pre.as<uint32_t>(),                     \
                                                    c->d_rend.as<uint32_t>(), c->d_rend.as<uint32_t>() + c->n_rows);    \
        break;
        switch (mode) {
            GCK_VARIANT(0) GCK_VARIANT(2) GCK_VARIANT(4) GCK_VARIANT(5) GCK_VARIANT(6) GCK_VARIANT(7) GCK_VARIANT(8)
            default: return GCK_EINVAL;
        }
#undef GCK_VARIANT
    }
    GCK_HIP(hipEventRecord(b, c->stream));
    GCK_HIP(hipEventSynchronize(b));
    float ms = 0;
    GCK_HIP(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    *ms_per_iter = ms / iters;
    return GCK_OK;
}

}  // extern "C"
