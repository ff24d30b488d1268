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
constexpr int kHops = 3;          // extra headers a speculative start must chain through
constexpr int kWaves = 16;        // wavefronts per k_crc_rows workgroup
constexpr uint32_t kNibBase = 32768;

// ---------------------------------------------------------------- helpers ---
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

// Follow the header chain from q: plausible sizes, records inside the file.
__device__ bool chain_ok(const uint8_t *__restrict__ arena, uint64_t base, uint64_t len, uint64_t q,
                         uint32_t max_key) {
    for (int h = 0; h <= kHops; ++h) {
        if (q == len) return true;
        if (q + 16 > len) return h > 0;
        const Hdr hd = ld_hdr(arena, base + q);
        const uint32_t klen = hd.ks ? hd.ks : hd.vs;
        if (klen == 0 || klen > max_key) return false;
        const uint64_t end = q + 16 + (uint64_t)hd.ks + hd.vs;
        if (end > len) return h > 0;
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
// One wavefront per chunk: the first byte position >= chunk start whose header
// and the next kHops headers are plausible.  Chunk 0 of a file starts at 0.
__global__ __launch_bounds__(256) void k_spec_entry(const uint8_t *__restrict__ arena,
                                                    const uint64_t *__restrict__ fbase,
                                                    const uint64_t *__restrict__ flen,
                                                    const uint32_t *__restrict__ ch_file,
                                                    const uint64_t *__restrict__ ch_start,
                                                    const uint64_t *__restrict__ ch_end,
                                                    uint64_t *__restrict__ ch_entry, uint32_t n_chunks,
                                                    uint32_t max_key) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= n_chunks) return;
    const uint32_t f = ch_file[c];
    const uint64_t cs = ch_start[c], ce = ch_end[c], base = fbase[f], len = flen[f];
    uint64_t found = kNone;
    if (cs == 0) {
        found = 0;
    } else {
        for (uint64_t p0 = cs; p0 < ce && found == kNone; p0 += 64) {
            const uint64_t p = p0 + lane;
            bool cand = false;
            if (p < ce && p + 16 <= len) {
                const uint64_t o = base + p + 8;
                const uint32_t *w = reinterpret_cast<const uint32_t *>(arena + (o & ~3ull));
                const uint32_t sh = (uint32_t)o & 3u;
                const uint32_t w0 = w[0], w1 = w[1], w2 = w[2];
                const uint32_t ks = ab(w1, w0, sh), vs = ab(w2, w1, sh);
                const uint32_t klen = ks ? ks : vs;
                cand = klen != 0 && klen <= max_key && p + 16 + (uint64_t)ks + vs <= len;
            }
            uint64_t mask = __ballot(cand);
            while (mask) {
                const int l = __ffsll((long long)mask) - 1;
                const uint64_t q = p0 + (uint64_t)l;
                if (chain_ok(arena, base, len, q, max_key)) {
                    found = q;
                    break;
                }
                mask &= mask - 1;
            }
        }
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

// Chunk c is consistent iff its entry equals the record start the nearest
// earlier non-empty chunk's chain reaches (or none if that chain ended).
__global__ __launch_bounds__(256) void k_validate(const uint32_t *__restrict__ ch_file,
                                                  const uint64_t *__restrict__ ch_start,
                                                  const uint64_t *__restrict__ ch_end,
                                                  const uint64_t *__restrict__ ch_entry,
                                                  const uint64_t *__restrict__ ch_exit,
                                                  const uint32_t *__restrict__ ch_term,
                                                  const uint32_t *__restrict__ f_first_chunk,
                                                  uint32_t *f_first_bad, uint32_t *counters,
                                                  uint32_t n_chunks) {
    const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n_chunks) return;
    const uint32_t f = ch_file[c], fc = f_first_chunk[f];
    if (c == fc) return;
    bool bad = false;
    uint32_t j = c - 1;
    int steps = 0;
    while (j > fc && ch_entry[j] == kNone && steps < 256) { --j; ++steps; }
    uint64_t expect = kNone;
    if (ch_entry[j] == kNone) {
        bad = true;
    } else if (ch_term[j] == T_NONE) {
        const uint64_t x = ch_exit[j];
        if (x < ch_start[c]) bad = true;
        else expect = x < ch_end[c] ? x : kNone;
    }
    if (!bad && ch_entry[c] != expect) bad = true;
    if (bad) {
        atomicMin(&f_first_bad[f], c - fc);
        atomicAdd(&counters[0], 1u);
    }
}

// One lane per file with an inconsistent chunk: re-derive entries sequentially
// from the last good chunk and re-walk every chunk whose entry changes.
__global__ void k_fixup(const uint8_t *__restrict__ arena, const uint64_t *__restrict__ fbase,
                        const uint64_t *__restrict__ flen, const uint32_t *__restrict__ f_first_chunk,
                        const uint32_t *__restrict__ f_nchunks, uint32_t *f_first_bad,
                        const uint64_t *__restrict__ ch_end, uint64_t *ch_entry, uint32_t *ch_count,
                        uint64_t *ch_exit, uint32_t *ch_term, uint64_t *ch_tpos, uint64_t *s_off,
                        uint4 *s_hdr, uint32_t cap, uint32_t nfiles, uint32_t *counters) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nfiles) return;
    const uint32_t fb = f_first_bad[f];
    if (fb == kNone32) return;
    const uint32_t fc = f_first_chunk[f], nc = f_nchunks[f];
    bool ended = false;
    uint64_t expect = kNone;
    int64_t j = (int64_t)fc + fb - 1;
    while (j > (int64_t)fc && ch_entry[j] == kNone) --j;
    if (ch_term[j] != T_NONE) ended = true;
    else expect = ch_exit[j];
    for (uint32_t k = fc + fb; k < fc + nc; ++k) {
        const uint64_t e_new = (!ended && expect < ch_end[k]) ? expect : kNone;
        if (e_new != ch_entry[k]) {
            ch_entry[k] = e_new;
            atomicAdd(&counters[1], 1u);
            walk_into_chunk(arena, fbase, flen, k, f, ch_end[k], e_new, cap, s_off, s_hdr, ch_count, ch_exit,
                            ch_term, ch_tpos);
        }
        if (ch_entry[k] != kNone) {
            if (ch_term[k] != T_NONE) ended = true;
            else expect = ch_exit[k];
        }
    }
    f_first_bad[f] = kNone32;
}

// Exclusive scan of per-chunk record counts (single workgroup; n <= ~1M).
__global__ __launch_bounds__(1024) void k_scan_chunks(const uint32_t *__restrict__ ch_count,
                                                      uint64_t *__restrict__ rec_base, uint32_t n) {
    __shared__ uint64_t s[1024];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (n + 1023) / 1024;
    const uint32_t b = t * per, e = min(b + per, n);
    uint64_t sum = 0;
    for (uint32_t i = b; i < e; ++i) sum += ch_count[i];
    s[t] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const uint64_t v = t >= (uint32_t)d ? s[t - d] : 0;
        __syncthreads();
        s[t] += v;
        __syncthreads();
    }
    uint64_t run = s[t] - sum;
    for (uint32_t i = b; i < e; ++i) {
        rec_base[i] = run;
        run += ch_count[i];
    }
    if (t == 1023) rec_base[n] = s[1023];
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

// row_first[row] = first record whose value ends after the row's first byte.
__global__ void k_row_index(const uint64_t *__restrict__ rec_off, const uint4 *__restrict__ rec_hdr,
                            uint64_t n_total, uint64_t n_rows, uint32_t *__restrict__ row_first) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n_total) return;
    const uint64_t ve_r = value_end(rec_off, rec_hdr, r);
    const uint64_t ve_p = r ? value_end(rec_off, rec_hdr, r - 1) : 0;
    const uint64_t lo = (ve_p + kRow - 1) / kRow, hi = (ve_r + kRow - 1) / kRow;
    for (uint64_t row = lo; row < hi; ++row) row_first[row] = (uint32_t)r;
    if (r == n_total - 1)
        for (uint64_t row = hi; row <= n_rows; ++row) row_first[row] = (uint32_t)n_total;
}

// Slicing-by-4 step through the LDS tables.  Table t, entry b, copy l31 lives
// at index t*8192 + b*32 + l31: every lane of a 32-lane LDS group reads its own
// bank, so the lookups are bank-conflict free (MI355X_MICROARCH.md §LDS).
__device__ __forceinline__ uint32_t slice4(const uint32_t *lds, uint32_t l31, uint32_t c) {
    return lds[24576 + (((c << 5) & 0x1FE0u) | l31)] ^ lds[16384 + (((c >> 3) & 0x1FE0u) | l31)] ^
           lds[8192 + (((c >> 11) & 0x1FE0u) | l31)] ^ lds[((c >> 19) & 0x1FE0u) | l31];
}

__device__ __forceinline__ uint32_t bytemask(int32_t lo, int32_t hi) {
    return (uint32_t)(((1ull << (8 * hi)) - 1) & ~((1ull << (8 * lo)) - 1));
}

// The HBM-bound kernel.  A wavefront owns a 4 KiB row; lane k owns bytes
// [64k, 64k+64).  Each lane runs the CRC register over the value bytes of its
// slab (non-value bytes masked to zero, the register cut at every value end),
// references its open tail to the row end with a per-lane constant shift
// Z_{64(63-k)} (8 nibble lookups), and a segmented XOR over lanes joins the
// pieces of each value.  Outputs per record: e (state at the value's last
// word), pre (its run just before the cut lane); per row: the run open at
// the row end.  k_finalize stitches rows (DESIGN.md §CRC algebra).
__global__ __launch_bounds__(1024) void k_crc_rows(const uint8_t *__restrict__ arena, uint64_t n_rows,
                                                   const uint32_t *__restrict__ row_first, uint64_t n_total,
                                                   const uint64_t *__restrict__ rec_off,
                                                   const uint4 *__restrict__ rec_hdr,
                                                   const uint32_t *__restrict__ g_slice,
                                                   const uint32_t *__restrict__ g_nib,
                                                   uint32_t *__restrict__ out_e, uint32_t *__restrict__ out_pre,
                                                   uint32_t *__restrict__ out_rend) {
    __shared__ uint32_t lds[40960];  // 128 KiB slicing tables x32 copies + 32 KiB lane-shift tables
    for (uint32_t i = threadIdx.x; i < 32768; i += 1024) lds[i] = g_slice[(i >> 13) * 256 + ((i >> 5) & 255)];
    for (uint32_t i = threadIdx.x; i < 8192; i += 1024) {
        const uint32_t l = (i >> 12) * 32 + (i & 31), v = (i >> 5) & 15, q = (i >> 9) & 7;
        lds[kNibBase + i] = g_nib[(l * 8 + q) * 16 + v];
    }
    __syncthreads();

    const uint32_t lane = threadIdx.x & 63, l31 = lane & 31;
    const uint32_t nbase = kNibBase + (lane >> 5) * 4096 + l31;
    const int32_t s_rel = (int32_t)lane * kSlab;
    const uint64_t n_waves = (uint64_t)gridDim.x * kWaves;
    constexpr int32_t BIG = INT_MAX / 2;

    for (uint64_t row = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6); row < n_rows; row += n_waves) {
        const uint64_t rs = row * kRow;
        const uint4 *src = reinterpret_cast<const uint4 *>(arena + rs + s_rel);
        const uint4 d0 = src[0], d1 = src[1], d2 = src[2], d3 = src[3];
        const uint32_t ra = row_first[row], rb = row_first[row + 1];

        // value intervals (row-relative, clamped) of records touching this slab
        int nint = 0;
        int32_t v0s = BIG, v0e = BIG, v1s = BIG, v1e = BIG, v2s = BIG, v2e = BIG, v3s = BIG, v3e = BIG;
        uint32_t i0 = 0, i1 = 0, i2 = 0, i3 = 0;
        if (ra < n_total) {
            const uint32_t last = rb < n_total ? rb : (uint32_t)(n_total - 1);
            for (uint32_t b0 = ra; b0 <= last; b0 += 64) {
                const uint32_t r = b0 + lane;
                int32_t my_s = 0, my_e = 0;
                if (r <= last) {
                    const uint4 h = rec_hdr[r];
                    const int64_t vs = (int64_t)(rec_off[r] + 16 + h.z) - (int64_t)rs;
                    const int64_t ve = vs + (int64_t)h.w;
                    my_s = (int32_t)max(min(vs, (int64_t)kRow + 1), (int64_t)-1);
                    my_e = (int32_t)max(min(ve, (int64_t)kRow + 1), (int64_t)-1);
                }
                const uint32_t cnt = min(64u, last - b0 + 1);
                for (uint32_t j = 0; j < cnt; ++j) {
                    const int32_t js = __builtin_amdgcn_readlane(my_s, j);
                    const int32_t je = __builtin_amdgcn_readlane(my_e, j);
                    if (je > js && js < s_rel + kSlab && je > s_rel) {
                        const uint32_t id = b0 + j;
                        if (nint == 0) { v0s = js; v0e = je; i0 = id; }
                        else if (nint == 1) { v1s = js; v1e = je; i1 = id; }
                        else if (nint == 2) { v2s = js; v2e = je; i2 = id; }
                        else if (nint == 3) { v3s = js; v3e = je; i3 = id; }
                        ++nint;
                    }
                }
            }
        }

        uint32_t crc = 0, first_cut = kNone32;
        int q = 0;
        int32_t cvs = v0s, cve = v0e;
        uint32_t cid = i0;
        const uint32_t words[16] = {d0.x, d0.y, d0.z, d0.w, d1.x, d1.y, d1.z, d1.w,
                                    d2.x, d2.y, d2.z, d2.w, d3.x, d3.y, d3.z, d3.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) {
            const int32_t o = s_rel + 4 * j;
            const int32_t lo = min(max(cvs - o, 0), 4), hi = min(max(cve - o, 0), 4);
            crc = slice4(lds, l31, crc ^ (words[j] & bytemask(lo, hi)));
            if (cve > o && cve <= o + 4) {  // this word holds the value's last byte
                out_e[cid] = crc;
                if (first_cut == kNone32) first_cut = cid;
                else out_pre[cid] = 0;     // started inside this slab: nothing before it
                crc = 0;
                ++q;
                cvs = q == 1 ? v1s : q == 2 ? v2s : q == 3 ? v3s : BIG;
                cve = q == 1 ? v1e : q == 2 ? v2e : q == 3 ? v3e : BIG;
                cid = q == 1 ? i1 : q == 2 ? i2 : i3;
            }
        }
        const bool tail = q < nint && cvs < s_rel + kSlab && cve > s_rel + kSlab;
        const uint32_t t = tail ? cid : kNone32;
        const uint32_t z = tail ? crc : 0u;
        // Z_{64(63-lane)}(z): reference the open tail to the row end
        uint32_t cz = 0;
#pragma unroll
        for (int qn = 0; qn < 8; ++qn) cz ^= lds[nbase + qn * 512 + (((z >> (4 * qn)) & 15u) << 5)];
        // segmented XOR over runs of equal t
        uint32_t P = cz;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint32_t v = __shfl_up(P, d);
            if ((int)lane >= d) P ^= v;
        }
        const uint32_t tprev = __shfl_up(t, 1);
        const bool start = lane == 0 || t != tprev;
        const uint64_t B = __ballot(start);
        const uint64_t upto = lane == 63 ? ~0ull : ((2ull << lane) - 1);
        const int rsl = 63 - __clzll((long long)(B & upto));
        const uint32_t Pp = __shfl(P, rsl > 0 ? rsl - 1 : 0);
        const uint32_t runv = P ^ (rsl > 0 ? Pp : 0u);
        const uint32_t runprev = __shfl_up(runv, 1);
        if (lane == 63) out_rend[row] = t != kNone32 ? runv : 0u;
        if (first_cut != kNone32) out_pre[first_cut] = (lane > 0 && tprev == first_cut) ? runprev : 0u;
    }
}

// Per record: stitch rows (Horner with Z_4096), undo the masked tail bytes
// (Z_-m), add the init/xorout term, compare with the header CRC
// (core/db.go:311), compute ValuePos = lastOffset + 16 + KeySize mod 2^32
// (core/keydir.go:25, lastOffset = carry + offset within the file).
__global__ __launch_bounds__(256) void k_finalize(const uint64_t *__restrict__ rec_off,
                                                  const uint4 *__restrict__ rec_hdr,
                                                  const uint32_t *__restrict__ rec_file,
                                                  const uint64_t *__restrict__ fbase,
                                                  const uint32_t *__restrict__ carry, uint64_t n_total,
                                                  const uint32_t *__restrict__ e, const uint32_t *__restrict__ pre,
                                                  const uint32_t *__restrict__ rend,
                                                  const uint32_t *__restrict__ xinv, const uint32_t *__restrict__ xa,
                                                  const uint32_t *__restrict__ xb, uint32_t x_row,
                                                  gck_rec *__restrict__ out, uint32_t *counters) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool reject = false;
    if (r < n_total) {
        const uint64_t off = rec_off[r];
        const uint4 h = rec_hdr[r];
        const uint32_t f = rec_file[r];
        const uint64_t vs = off + 16 + h.z, L = h.w, ve = vs + L;
        uint32_t raw0 = 0;
        if (L) {
            const uint64_t fr = vs / kRow, lr = (ve - 1) / kRow;
            uint32_t acc = 0;
            for (uint64_t row = fr; row < lr; ++row) acc = multmodp(x_row, acc) ^ rend[row];
            acc = multmodp(x_row, acc) ^ pre[r];
            const uint64_t row_end = (lr + 1) * kRow;
            raw0 = multmodp(xinv[(4 - (ve & 3)) & 3], e[r]) ^ multmodp(xinv[row_end - ve], acc);
        }
        const uint32_t zl = multmodp(multmodp(xa[L >> 16], xb[L & 0xFFFF]), 0xFFFFFFFFu);
        const uint32_t calc = raw0 ^ zl ^ 0xFFFFFFFFu;
        const uint64_t fo = off - fbase[f];
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
        reject = calc != h.x;
    }
    const uint64_t m = __ballot(reject);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&counters[3], (uint32_t)__popcll(m));
}

// ------------------------------------------------------------- host side ---
static void make_tables(std::vector<uint32_t> &slice, std::vector<uint32_t> &nib, std::vector<uint32_t> &xinv,
                        std::vector<uint32_t> &xa, std::vector<uint32_t> &xb, uint32_t &x_row) {
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
    x_row = xpow8n(kRow);
}

static uint32_t g_xrow = 0;

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
    for (auto &e : c->ev) GCK_HIP(hipEventCreate(&e));
    if (multmodp(kXinv, kX0 >> 1) != kX0) return GCK_EINVAL;
    std::vector<uint32_t> slice, nib, xinv, xa, xb;
    make_tables(slice, nib, xinv, xa, xb, g_xrow);
    int rc;
    if ((rc = c->d_slice.ensure(slice.size() * 4)) || (rc = c->d_nib.ensure(nib.size() * 4)) ||
        (rc = c->d_xinv.ensure(xinv.size() * 4)) || (rc = c->d_xa.ensure(xa.size() * 4)) ||
        (rc = c->d_xb.ensure(xb.size() * 4)) || (rc = c->d_counters.ensure(64)))
        return rc;
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
                   &c->d_ch_end, &c->d_ch_entry, &c->d_ch_exit, &c->d_ch_count, &c->d_ch_term, &c->d_ch_tpos,
                   &c->d_rec_base, &c->d_scratch_off, &c->d_scratch_hdr, &c->d_counters, &c->d_rec_off,
                   &c->d_rec_hdr, &c->d_rec_file, &c->d_e, &c->d_pre, &c->d_out, &c->d_row_first, &c->d_rend,
                   &c->d_slice, &c->d_nib, &c->d_xinv, &c->d_xa, &c->d_xb};
    for (DBuf *b : all) b->release();
    for (auto &e : c->ev)
        if (e) (void)hipEventDestroy(e);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    c->stream = nullptr;
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
    const bool fresh = c->arena.cap < pos + 2 * kRow;
    if ((rc = c->arena.ensure(pos + 2 * kRow))) return rc;
    if (fresh) GCK_HIP(hipMemset(c->arena.p, 0, c->arena.cap));
    if ((rc = c->d_fbase.ensure(nf * 8)) || (rc = c->d_flen.ensure(nf * 8)) || (rc = c->d_ffirst.ensure(nf * 4)) ||
        (rc = c->d_fnch.ensure(nf * 4)) || (rc = c->d_fbad.ensure(nf * 4)) || (rc = c->d_fterm.ensure(nf * 4)) ||
        (rc = c->d_ftpos.ensure(nf * 8)) || (rc = c->d_fnrec.ensure(nf * 8)) ||
        (rc = c->d_ffirstrec.ensure(nf * 8)) || (rc = c->d_carry.ensure(nf * 4)) ||
        (rc = c->d_ch_file.ensure((nc + 1) * 4)) || (rc = c->d_ch_start.ensure((nc + 1) * 8)) ||
        (rc = c->d_ch_end.ensure((nc + 1) * 8)) || (rc = c->d_ch_entry.ensure((nc + 1) * 8)) ||
        (rc = c->d_ch_exit.ensure((nc + 1) * 8)) || (rc = c->d_ch_count.ensure((nc + 1) * 4)) ||
        (rc = c->d_ch_term.ensure((nc + 1) * 4)) || (rc = c->d_ch_tpos.ensure((nc + 1) * 8)) ||
        (rc = c->d_rec_base.ensure((nc + 1) * 8)) || (rc = c->d_scratch_off.ensure((nc + 1) * cap * 8)) ||
        (rc = c->d_scratch_hdr.ensure((nc + 1) * cap * 16)) || (rc = c->d_row_first.ensure((c->n_rows + 1) * 4)) ||
        (rc = c->d_rend.ensure((c->n_rows + 1) * 4)))
        return rc;
    if (nfiles) {
        GCK_HIP(hipMemcpy(c->d_fbase.p, c->f_base.data(), nfiles * 8, hipMemcpyHostToDevice));
        GCK_HIP(hipMemcpy(c->d_flen.p, c->f_len.data(), nfiles * 8, hipMemcpyHostToDevice));
        GCK_HIP(hipMemcpy(c->d_ffirst.p, c->f_first_chunk.data(), nfiles * 4, hipMemcpyHostToDevice));
        GCK_HIP(hipMemcpy(c->d_fnch.p, c->f_nchunks.data(), nfiles * 4, hipMemcpyHostToDevice));
    }
    if (nc) {
        GCK_HIP(hipMemcpy(c->d_ch_file.p, ch_file.data(), nc * 4, hipMemcpyHostToDevice));
        GCK_HIP(hipMemcpy(c->d_ch_start.p, ch_start.data(), nc * 8, hipMemcpyHostToDevice));
        GCK_HIP(hipMemcpy(c->d_ch_end.p, ch_end.data(), nc * 8, hipMemcpyHostToDevice));
    }
    return GCK_OK;
}

static inline uint32_t nblk(uint64_t n, uint32_t per) { return (uint32_t)((n + per - 1) / per); }

static int ctx_run(Ctx *c) {
    const auto t0 = std::chrono::steady_clock::now();
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const uint32_t nc = c->n_chunks, nf = c->nfiles, cap = c->opts.chunk_cap;
    uint32_t *cnt = c->d_counters.as<uint32_t>();
    GCK_HIP(hipMemsetAsync(cnt, 0, 64, s));
    if (nf) {
        GCK_HIP(hipMemsetAsync(c->d_fbad.p, 0xFF, nf * 4, s));
    }
    GCK_HIP(hipEventRecord(c->ev[PH_SPEC], s));
    if (nc) {
        k_spec_entry<<<nblk(nc, 4), 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(),
                                                 c->d_flen.as<uint64_t>(), c->d_ch_file.as<uint32_t>(),
                                                 c->d_ch_start.as<uint64_t>(), c->d_ch_end.as<uint64_t>(),
                                                 c->d_ch_entry.as<uint64_t>(), nc, c->opts.max_key);
    }
    GCK_HIP(hipEventRecord(c->ev[PH_WALK], s));
    if (nc) {
        k_walk<<<nblk(nc, 256), 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(),
                                             c->d_flen.as<uint64_t>(), c->d_ch_file.as<uint32_t>(),
                                             c->d_ch_end.as<uint64_t>(), c->d_ch_entry.as<uint64_t>(),
                                             c->d_ch_count.as<uint32_t>(), c->d_ch_exit.as<uint64_t>(),
                                             c->d_ch_term.as<uint32_t>(), c->d_ch_tpos.as<uint64_t>(),
                                             c->d_scratch_off.as<uint64_t>(), c->d_scratch_hdr.as<uint4>(), cap, nc);
    }
    GCK_HIP(hipEventRecord(c->ev[PH_VALIDATE], s));
    if (nc) {
        k_validate<<<nblk(nc, 256), 256, 0, s>>>(c->d_ch_file.as<uint32_t>(), c->d_ch_start.as<uint64_t>(),
                                                 c->d_ch_end.as<uint64_t>(), c->d_ch_entry.as<uint64_t>(),
                                                 c->d_ch_exit.as<uint64_t>(), c->d_ch_term.as<uint32_t>(),
                                                 c->d_ffirst.as<uint32_t>(), c->d_fbad.as<uint32_t>(), cnt, nc);
        k_fixup<<<nblk(nf, 64), 64, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(),
                                            c->d_flen.as<uint64_t>(), c->d_ffirst.as<uint32_t>(),
                                            c->d_fnch.as<uint32_t>(), c->d_fbad.as<uint32_t>(),
                                            c->d_ch_end.as<uint64_t>(), c->d_ch_entry.as<uint64_t>(),
                                            c->d_ch_count.as<uint32_t>(), c->d_ch_exit.as<uint64_t>(),
                                            c->d_ch_term.as<uint32_t>(), c->d_ch_tpos.as<uint64_t>(),
                                            c->d_scratch_off.as<uint64_t>(), c->d_scratch_hdr.as<uint4>(), cap, nf,
                                            cnt);
    }
    GCK_HIP(hipEventRecord(c->ev[PH_SCAN], s));
    if (nc) {
        k_scan_chunks<<<1, 1024, 0, s>>>(c->d_ch_count.as<uint32_t>(), c->d_rec_base.as<uint64_t>(), nc);
    } else {
        GCK_HIP(hipMemsetAsync(c->d_rec_base.p, 0, 8, s));
    }
    if (nf) {
        k_file_summary<<<nblk(nf, 64), 64, 0, s>>>(c->d_ffirst.as<uint32_t>(), c->d_fnch.as<uint32_t>(),
                                                   c->d_rec_base.as<uint64_t>(), c->d_ch_entry.as<uint64_t>(),
                                                   c->d_ch_term.as<uint32_t>(), c->d_ch_tpos.as<uint64_t>(),
                                                   c->d_fterm.as<uint32_t>(), c->d_ftpos.as<uint64_t>(),
                                                   c->d_ffirstrec.as<uint64_t>(), c->d_fnrec.as<uint64_t>(), nf);
    }
    GCK_HIP(hipEventRecord(c->ev[PH_HOST], s));

    // ---- host: EOF classification + lastOffset carries (core/db.go:110-140) ----
    std::vector<uint32_t> fterm(nf), carry(nf);
    std::vector<uint64_t> ftpos(nf), ffirst(nf), fnrec(nf);
    uint32_t hc[4] = {0, 0, 0, 0};
    if (nf) {
        GCK_HIP(hipMemcpyAsync(fterm.data(), c->d_fterm.p, nf * 4, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipMemcpyAsync(ftpos.data(), c->d_ftpos.p, nf * 8, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipMemcpyAsync(ffirst.data(), c->d_ffirstrec.p, nf * 8, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipMemcpyAsync(fnrec.data(), c->d_fnrec.p, nf * 8, hipMemcpyDeviceToHost, s));
    }
    GCK_HIP(hipMemcpyAsync(hc, cnt, 16, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    c->n_fixups = hc[1];
    c->status = GCK_OK;
    c->err_file = 0;
    c->err_off = 0;
    c->files_walked = nf;
    uint64_t n_total = 0;
    uint32_t last = 0;  // keyDir.lastOffset at the start of each file
    for (uint32_t f = 0; f < nf; ++f) {
        carry[f] = last;
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
    c->n_recs = n_total;
    if (nf) GCK_HIP(hipMemcpyAsync(c->d_carry.p, carry.data(), nf * 4, hipMemcpyHostToDevice, s));
    const uint64_t nr = n_total ? n_total : 1;
    int rc;
    if ((rc = c->d_rec_off.ensure(nr * 8)) || (rc = c->d_rec_hdr.ensure(nr * 16)) ||
        (rc = c->d_rec_file.ensure(nr * 4)) || (rc = c->d_e.ensure(nr * 4)) || (rc = c->d_pre.ensure(nr * 4)) ||
        (rc = c->d_out.ensure(nr * sizeof(gck_rec))))
        return rc;
    if (n_total > 0xFFFFFFF0ull) return GCK_EINVAL;

    GCK_HIP(hipEventRecord(c->ev[PH_COMPACT], s));
    if (n_total) {
        k_compact<<<nblk(nc, 4), 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(),
                                              c->d_flen.as<uint64_t>(), c->d_ch_file.as<uint32_t>(),
                                              c->d_ch_end.as<uint64_t>(), c->d_ch_entry.as<uint64_t>(),
                                              c->d_ch_count.as<uint32_t>(), c->d_rec_base.as<uint64_t>(),
                                              c->d_scratch_off.as<uint64_t>(), c->d_scratch_hdr.as<uint4>(), cap,
                                              nc, n_total, c->d_rec_off.as<uint64_t>(), c->d_rec_hdr.as<uint4>(),
                                              c->d_rec_file.as<uint32_t>(), cnt);
    }
    GCK_HIP(hipEventRecord(c->ev[PH_ROWIDX], s));
    if (n_total) {
        k_row_index<<<nblk(n_total, 256), 256, 0, s>>>(c->d_rec_off.as<uint64_t>(), c->d_rec_hdr.as<uint4>(),
                                                      n_total, c->n_rows, c->d_row_first.as<uint32_t>());
    } else {
        GCK_HIP(hipMemsetAsync(c->d_row_first.p, 0, (c->n_rows + 1) * 4, s));
    }
    GCK_HIP(hipEventRecord(c->ev[PH_CRC], s));
    if (c->n_rows && n_total) {
        const uint64_t want = (c->n_rows + kWaves - 1) / kWaves;
        const uint32_t grid = (uint32_t)(want < (uint64_t)c->n_cu ? want : (uint64_t)c->n_cu);
        k_crc_rows<<<grid, 1024, 0, s>>>(c->arena.as<uint8_t>(), c->n_rows, c->d_row_first.as<uint32_t>(), n_total,
                                         c->d_rec_off.as<uint64_t>(), c->d_rec_hdr.as<uint4>(),
                                         c->d_slice.as<uint32_t>(), c->d_nib.as<uint32_t>(), c->d_e.as<uint32_t>(),
                                         c->d_pre.as<uint32_t>(), c->d_rend.as<uint32_t>());
    }
    GCK_HIP(hipEventRecord(c->ev[PH_FINAL], s));
    if (n_total) {
        k_finalize<<<nblk(n_total, 256), 256, 0, s>>>(
            c->d_rec_off.as<uint64_t>(), c->d_rec_hdr.as<uint4>(), c->d_rec_file.as<uint32_t>(),
            c->d_fbase.as<uint64_t>(), c->d_carry.as<uint32_t>(), n_total, c->d_e.as<uint32_t>(),
            c->d_pre.as<uint32_t>(), c->d_rend.as<uint32_t>(), c->d_xinv.as<uint32_t>(), c->d_xa.as<uint32_t>(),
            c->d_xb.as<uint32_t>(), g_xrow, c->d_out.as<gck_rec>(), cnt);
    }
    GCK_HIP(hipEventRecord(c->ev[PH_COUNT], s));
    GCK_HIP(hipMemcpyAsync(hc, cnt, 16, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    GCK_HIP(hipGetLastError());
    c->n_overflow = hc[2];
    c->n_crc_fail = hc[3];
    for (int p = 0; p < PH_COUNT; ++p) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, c->ev[p], c->ev[p + 1]);
        c->ms_phase[p] = ms;
    }
    c->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return c->status;
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
    for (int p = 0; p < PH_COUNT && p < 12; ++p) out->ms_kernel[p] = c->ms_phase[p];
    return GCK_OK;
}

const char *gck_phase_name(int phase) {
    static const char *names[] = {"spec_entry", "walk", "validate", "scan", "host_sync",
                                  "compact",    "row_index", "crc_rows", "finalize"};
    return phase >= 0 && phase < PH_COUNT ? names[phase] : "";
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

}  // extern "C"
