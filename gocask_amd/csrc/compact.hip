// compact.hip — merge (compaction) and hint files on the device (SURVEY.md
// §8f f4: "merging and hint files", the reference's roadmap item README.md:60).
//
// After gck_ctx_keydir (live Puts only), the live records, in walk order, are
// written as new data files exactly as DB.Put would write them into a fresh
// database with MaxDataFileSize M (core/db.go:185-231: an entry that does not
// fit rotates first, rotateDataFile:214-231), each record's bytes verbatim
// (header, key, value: CRCs and timestamps unchanged).  One hint file per data
// file (format invented here, include/gocask_hip.h GCK_HINT_*), little-endian:
//   entries [Timestamp u32][KeySize u32][ValueSize u32][ValuePos u32][CRC u32][key]
//   index   [hint offset u64][data-file offset u64] of every GCK_HINT_BLOCK-th entry
//   tail    [entries u64][entry bytes u64][data-file bytes u64][magic u32][version u32]
// (ValuePos = the value's offset in the merged file mod 2^32, as
// core/keydir.go:25 would set it; CRC = kdEntry.CRC), so a later start fills
// the keydir without reading values (hints.hip), in parallel over the blocks
// the index lists.
//
// Kernels: sizes and two-level exclusive scans of record and hint-entry
// sizes; the rotation points (few files: one wavefront, a 64-way search per
// file; many: each record's successor file start, then the chain from record
// 0 by pointer doubling); the
// data bytes (a wavefront per group of 64 records, 16 B output chunks, each
// from one or two chunk-aligned windows of the resident arena); the hint
// entries (a lane per record).
#include "gck_internal.h"

namespace gck {

typedef uint32_t u32x4_a4c __attribute__((ext_vector_type(4), aligned(4)));

constexpr uint32_t kCmpBlock = 1024;  // records per first-level scan block
constexpr uint64_t kHintHdr = 20;      // hint entry header bytes (GCK_HINT_*)
constexpr uint64_t kHintTail = 32, kHintIdx = 24;  // tail, index entry bytes
// index + tail bytes of a hint file of n entries
__host__ __device__ __forceinline__ uint64_t hint_footer(uint64_t n) {
    return kHintIdx * ((n + GCK_HINT_BLOCK - 1) / GCK_HINT_BLOCK) + kHintTail;
}

__device__ __forceinline__ uint64_t wave_incl_sum64(uint64_t v) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t o = __shfl_up(v, d);
        if ((threadIdx.x & 63) >= (uint32_t)d) v += o;
    }
    return v;
}

// Per record: data size 16 + KeySize + ValueSize and hint size 20 + KeySize;
// exclusive scans within blocks of kCmpBlock, block totals to bsum / hbsum.
__global__ __launch_bounds__(kCmpBlock) void k_cmp_sizes(const gck_rec *__restrict__ kd, uint64_t n,
                                                         uint64_t *__restrict__ pos, uint64_t *__restrict__ hpos,
                                                         uint64_t *__restrict__ bsum, uint64_t *__restrict__ hbsum) {
    __shared__ uint64_t wt[2][kCmpBlock / 64];
    const uint64_t i = (uint64_t)blockIdx.x * kCmpBlock + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint64_t sz = 0, hs = 0;
    if (i < n) {
        const gck_rec r = kd[i];
        sz = 16ull + r.key_len + r.value_size;
        hs = kHintHdr + r.key_len;
    }
    const uint64_t a = wave_incl_sum64(sz), b = wave_incl_sum64(hs);
    if (lane == 63) {
        wt[0][w] = a;
        wt[1][w] = b;
    }
    __syncthreads();
    uint64_t pa = 0, pb = 0;
    for (uint32_t k = 0; k < w; ++k) {
        pa += wt[0][k];
        pb += wt[1][k];
    }
    if (i < n) {
        pos[i] = pa + a - sz;
        hpos[i] = pb + b - hs;
    }
    if (threadIdx.x == kCmpBlock - 1) {
        bsum[blockIdx.x] = pa + a;
        hbsum[blockIdx.x] = pb + b;
    }
}

// One wavefront: exclusive scan of the block totals (in place), totals at [nb].
// The block totals' exclusive scan by one 1024-thread workgroup, 1024 totals
// per step (C3: 4,211 blocks; one wavefront took 43 us for it).
__global__ __launch_bounds__(1024) void k_cmp_top(uint64_t *__restrict__ bsum, uint64_t *__restrict__ hbsum, uint64_t nb) {
    __shared__ uint64_t wt[2][16], run[2];
    const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (threadIdx.x == 0) run[0] = run[1] = 0;
    __syncthreads();
    for (uint64_t i0 = 0; i0 < nb; i0 += 1024) {
        const uint64_t i = i0 + threadIdx.x;
        const uint64_t va = i < nb ? bsum[i] : 0, vb = i < nb ? hbsum[i] : 0;
        const uint64_t a = wave_incl_sum64(va), b = wave_incl_sum64(vb);
        if (lane == 63) {
            wt[0][wid] = a;
            wt[1][wid] = b;
        }
        __syncthreads();
        uint64_t pa = run[0], pb = run[1];
        for (uint32_t k = 0; k < wid; ++k) {
            pa += wt[0][k];
            pb += wt[1][k];
        }
        if (i < nb) {
            bsum[i] = pa + a - va;
            hbsum[i] = pb + b - vb;
        }
        __syncthreads();
        if (threadIdx.x == 1023) {
            run[0] = pa + a;
            run[1] = pb + b;
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        bsum[nb] = run[0];
        hbsum[nb] = run[1];
    }
}

__global__ void k_cmp_add(uint64_t *__restrict__ pos, uint64_t *__restrict__ hpos, const uint64_t *__restrict__ bsum,
                          const uint64_t *__restrict__ hbsum, uint64_t n, uint64_t nb) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        pos[i] += bsum[i / kCmpBlock];
        hpos[i] += hbsum[i / kCmpBlock];
    }
    if (i == n) {
        pos[n] = bsum[nb];
        hpos[n] = hbsum[nb];
    }
}

// Rotation points (core/db.go:214-231 applied record by record): fstart[k] is
// the first record of merged file k, fstart[nf] = n.  A file takes records
// while its size + the next entry <= M; the first file is empty when the
// first record alone exceeds M (the fresh database's active file is rotated
// away before anything is written).  One wavefront; per file a 64-way search
// of pos for the first record that does not fit.
__global__ __launch_bounds__(64) void k_cmp_breaks(const uint64_t *__restrict__ pos, uint64_t n, uint64_t M,
                                                   uint32_t *__restrict__ fstart, uint32_t cap,
                                                   uint32_t *__restrict__ n_files) {
    const uint32_t lane = threadIdx.x;
    uint32_t k = 0;
    uint64_t b = 0;
    if (n == 0) {  // nothing live: the fresh database's one (empty) file
        if (lane == 0) {
            fstart[0] = 0;
            fstart[1] = 0;
            *n_files = 1;
        }
        return;
    }
    if (pos[1] - pos[0] > M) {
        if (lane == 0) fstart[0] = 0;
        k = 1;
    }
    while (b < n && k < cap) {
        if (lane == 0) fstart[k] = (uint32_t)b;
        ++k;
        // the smallest j in (b, n) with pos[j + 1] - pos[b] > M, else n
        const uint64_t lim = pos[b] + M;
        uint64_t lo = b + 1, hi = n;  // answer in [lo, hi]
        while (lo < hi) {
            const uint64_t span = hi - lo, step = (span + 63) / 64;
            const uint64_t j = lo + (uint64_t)lane * step;
            const bool over = j < hi && pos[j + 1] > lim;
            const uint64_t m = __ballot(over);
            if (m) {  // the first probe over the limit bounds the answer
                const uint32_t f = (uint32_t)__builtin_ctzll(m);
                const uint64_t jf = lo + (uint64_t)f * step;
                hi = jf;
                lo = f ? lo + (uint64_t)(f - 1) * step + 1 : lo;
            } else {
                lo = lo + 63 * step + 1 > hi ? hi : lo + 63 * step + 1;
            }
        }
        b = lo;
    }
    if (lane == 0) {
        fstart[k < cap ? k : cap - 1] = (uint32_t)n;
        *n_files = k;
    }
}

// Rotation points for many merged files (a small max_file_size): the chain of
// file starts 0 -> next[0] -> next[next[0]] ... with next[b] = the smallest j
// in (b, n] with j == n or pos[j + 1] - pos[b] > M (a lane per record, binary
// search), marked by pointer doubling: round k marks jmp[i] for every marked
// i, then jmp[i] = jmp[jmp[i]] (= next^(2^(k+1))(i)), so after R rounds every
// start within 2^R steps of record 0 is marked.  A mark that lands during its
// own round only marks true starts earlier (images of starts are starts).
__global__ void k_cmp_next(const uint64_t *__restrict__ pos, uint64_t n, uint64_t M, uint32_t *__restrict__ jmp,
                           uint32_t *__restrict__ on) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > n) return;
    if (i == n) {
        jmp[n] = (uint32_t)n;
        return;
    }
    const uint64_t lim = pos[i] + M;
    uint64_t lo = i + 1, hi = n;  // answer in [lo, hi]
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (pos[mid + 1] > lim) hi = mid; else lo = mid + 1;
    }
    jmp[i] = (uint32_t)lo;
    on[i] = i == 0 ? 1u : 0u;
}
__global__ void k_cmp_mark(const uint32_t *__restrict__ jmp, uint32_t *on, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n && on[i]) {
        const uint32_t j = jmp[i];
        if (j < n) on[j] = 1u;
    }
}
__global__ void k_cmp_jump(const uint32_t *__restrict__ jmp, uint32_t *__restrict__ jmp2, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= n) jmp2[i] = jmp[jmp[i]];
}
// fstart from the marks: per block of kCmpBlock records the marked count
// (wave ballots), one wavefront scans the block counts, then each block
// writes its starts in order after `lead` (1 when the first file is empty).
__global__ __launch_bounds__(kCmpBlock) void k_cmp_fcount(const uint32_t *__restrict__ on, uint64_t n,
                                                          uint64_t *__restrict__ bcnt) {
    __shared__ uint32_t wc[kCmpBlock / 64];
    const uint64_t i = (uint64_t)blockIdx.x * kCmpBlock + threadIdx.x;
    const uint64_t m = __ballot(i < n && on[i]);
    if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = (uint32_t)__popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t k = 0; k < kCmpBlock / 64; ++k) t += wc[k];
        bcnt[blockIdx.x] = t;
    }
}
__global__ __launch_bounds__(64) void k_cmp_ftop(uint64_t *__restrict__ bcnt, uint64_t nb, uint32_t lead,
                                                 uint32_t *__restrict__ fstart, uint64_t n, uint32_t *__restrict__ n_files) {
    uint64_t run = 0;  // block offsets among the starts (k_cmp_fscatter adds lead)
    for (uint64_t i0 = 0; i0 < nb; i0 += 64) {
        const uint64_t i = i0 + threadIdx.x;
        const uint64_t v = i < nb ? bcnt[i] : 0;
        const uint64_t a = wave_incl_sum64(v);
        if (i < nb) bcnt[i] = run + a - v;
        run += __shfl(a, 63);
    }
    if (threadIdx.x == 0) {
        if (lead) fstart[0] = 0;  // the empty first file
        fstart[lead + run] = (uint32_t)n;
        *n_files = (uint32_t)(lead + run);
    }
}
__global__ __launch_bounds__(kCmpBlock) void k_cmp_fscatter(const uint32_t *__restrict__ on, uint64_t n,
                                                            const uint64_t *__restrict__ bcnt,
                                                            uint32_t *__restrict__ fstart) {
    __shared__ uint32_t wc[kCmpBlock / 64];
    const uint64_t i = (uint64_t)blockIdx.x * kCmpBlock + threadIdx.x;
    const bool mk = i < n && on[i];
    const uint64_t m = __ballot(mk);
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    if (lane == 0) wc[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t k = 0; k < w; ++k) before += wc[k];
    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (mk) fstart[bcnt[blockIdx.x] + before + r] = (uint32_t)i;
}

// The 16 bytes at p (any alignment): two dword-aligned loads and a byte shift.
// 16 bytes to any byte address: one dwordx4 store (gfx9 global stores need no
// alignment; as gck_crc_wave.h store16u).
__device__ __forceinline__ void st16u(uint8_t *dst, uint4 v) {
    typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
    u32x4_a1 x;
    x.x = v.x;
    x.y = v.y;
    x.z = v.z;
    x.w = v.w;
    *reinterpret_cast<u32x4_a1 *>(dst) = x;
}
__device__ __forceinline__ void st4u(uint8_t *dst, uint32_t v) {
    typedef uint32_t u32_a1 __attribute__((aligned(1)));
    *reinterpret_cast<u32_a1 *>(dst) = v;
}
__device__ __forceinline__ uint4 ld16u(const uint8_t *p) {
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
    const uint8_t *a = p - sh;
    const u32x4_a4c x = *reinterpret_cast<const u32x4_a4c *>(a);
    const uint32_t y = *reinterpret_cast<const uint32_t *>(a + (sh ? 16 : 12));  // (as encode.hip load16u)
    return make_uint4(__builtin_amdgcn_alignbyte(x.y, x.x, sh), __builtin_amdgcn_alignbyte(x.z, x.y, sh),
                      __builtin_amdgcn_alignbyte(x.w, x.z, sh), __builtin_amdgcn_alignbyte(y, x.w, sh));
}

// Data bytes: a wavefront per group of 64 consecutive live records; output
// rows of 1 KiB, lane l the 16 B chunk at 16 l.  A chunk holds bytes of at
// most two records (a live record is >= 17 bytes: the key is not empty);
// each record's part comes from the arena window aligned to the chunk (chunk
// byte i = record byte X + i - P), so a chunk is one or two unaligned 16 B
// loads and a byte select.  Bytes outside the group's range are another
// group's: those chunks are stored byte by byte.  A row inside one record
// takes a uniform path (fields by readlane, one load, one store per lane).
__global__ __launch_bounds__(256) void k_cmp_copy(const uint8_t *__restrict__ arena,
                                                  const uint64_t *__restrict__ fbase,
                                                  const gck_rec *__restrict__ kd, const uint64_t *__restrict__ pos,
                                                  uint64_t n, uint8_t *__restrict__ out, uint32_t *__restrict__ queue) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t groups = (n + 63) / 64, waves = (uint64_t)gridDim.x * (blockDim.x / 64);
    // groups: the first per wavefront static, the rest from an atomic queue
    for (uint64_t g = (uint64_t)blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6); g < groups;) {
        const uint64_t g0 = g * 64, mine = g0 + lane;
        const uint32_t cnt = (uint32_t)min<uint64_t>(64, n - g0);
        const bool have = lane < cnt;
        uint64_t src = 0, len = 0, P = 0;
        if (have) {
            const gck_rec r = kd[mine];
            src = fbase[r.file] + r.rec_off;
            len = 16ull + r.key_len + r.value_size;
            P = pos[mine];
        }
        const uint64_t O0 = __shfl(P, 0), O1 = pos[g0 + cnt];
        auto rl64 = [](uint64_t v, uint32_t k) {
            return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(v >> 32), (int)k) << 32) |
                   (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)k);
        };
        uint32_t rr = 0;
        for (uint64_t R = O0 & ~15ull; R < O1; R += 1024) {
            const uint64_t X = R + 16ull * lane;
            uint32_t r = rr;
            for (uint32_t k = rr + 1; k < cnt; ++k) {
                const uint64_t pk = rl64(P, k);
                if (pk >= R + 1024) break;
                if (X >= pk) r = k;
            }
            rr = (uint32_t)__builtin_amdgcn_readlane((int)r, 63);
            if ((uint32_t)__builtin_amdgcn_readlane((int)r, 0) == rr) {
                const uint64_t p0 = rl64(P, rr), l0 = rl64(len, rr);
                if (R >= p0 && R + 1024 <= p0 + l0) {  // (uniform) the row inside one record
                    const uint64_t s0 = rl64(src, rr);
                    *reinterpret_cast<uint4 *>(out + X) = ld16u(arena + s0 + (X - p0));
                    continue;
                }
            }
            // (no early exit for lanes past O1: the permutes below read the
            // record fields from other lanes, and ds_bpermute returns 0 from
            // lanes that are not active; their chunks get an empty mask)
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            uint32_t mask = 0;
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const uint32_t sidx = min<uint32_t>(r + j, cnt - 1);
                const uint64_t ps = __shfl(P, (int)sidx), ls = __shfl(len, (int)sidx), ss = __shfl(src, (int)sidx);
                const uint64_t b0 = max(max(X, ps), O0), b1 = min(min(X + 16, ps + ls), O1);
                if (r + j >= cnt || b0 >= b1) continue;
                uint4 v;
                if ((int64_t)(ss + X) - (int64_t)ps >= 0) {
                    v = ld16u(arena + ss + X - ps);
                } else {  // a window starting before the arena: bytes one by one
                    uint32_t by[16];
#pragma unroll
                    for (int i = 0; i < 16; ++i) by[i] = X + i >= ps && X + i < ps + ls ? arena[ss + (X + i - ps)] : 0u;
                    v = make_uint4(by[0] | by[1] << 8 | by[2] << 16 | by[3] << 24, by[4] | by[5] << 8 | by[6] << 16 | by[7] << 24,
                                   by[8] | by[9] << 8 | by[10] << 16 | by[11] << 24,
                                   by[12] | by[13] << 8 | by[14] << 16 | by[15] << 24);
                }
                const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
                const uint32_t m = ((1u << (uint32_t)(b1 - X)) - 1u) & ~((1u << (uint32_t)(b0 - X)) - 1u);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t bm = (m >> (4 * q)) & 15u;
                    const uint32_t km = (bm & 1u ? 0xFFu : 0u) | (bm & 2u ? 0xFF00u : 0u) | (bm & 4u ? 0xFF0000u : 0u) |
                                        (bm & 8u ? 0xFF000000u : 0u);
                    w[q] = (w[q] & ~km) | (vv[q] & km);
                }
                mask |= m;
            }
            if (mask == 0xFFFFu) {
                *reinterpret_cast<uint4 *>(out + X) = make_uint4(w[0], w[1], w[2], w[3]);
            } else if (mask) {  // the group's first or last chunk: its bytes only
                for (uint32_t i = 0; i < 16; ++i)
                    if ((mask >> i) & 1) out[X + i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
            }
        }
        uint32_t t = 0;
        if (lane == 0) t = atomicAdd(queue, 1u);
        g = waves + (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
    }
}

// Hint entries: a lane per record (20 + KeySize bytes each), at hpos[i] plus
// the index and tail bytes of the files before its own (foot[f]); the lane of
// every GCK_HINT_BLOCK-th record of a file writes its index entry.
// The integrity word of hint entry t (record kd[t], at data offset qo in its
// merged file): hint_entry_check over its header words and key.
__device__ __forceinline__ unsigned long long cmp_entry_check(const uint8_t *__restrict__ arena,
                                                              const uint64_t *__restrict__ fbase, const gck_rec &q,
                                                              uint64_t qo) {
    const uint8_t *kp = arena + fbase[q.file] + q.rec_off + 16;
    const uint32_t ql = q.key_len;
    auto kw = [&](uint32_t w) {  // key word w, zero past the key (the arena is padded)
        const uint8_t *p = kp + 4 * w;
        const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
        const uint32_t *a = reinterpret_cast<const uint32_t *>(p - sh);
        const uint32_t v = __builtin_amdgcn_alignbyte(a[1], a[0], sh), left = ql - 4 * w;
        return left >= 4 ? v : v & ((1u << (8 * left)) - 1u);
    };
    return hint_entry_check(q.ts, ql, q.value_size, (uint32_t)(qo + 16 + ql), q.crc, kw);
}

__global__ __launch_bounds__(256) void k_cmp_hints(const uint8_t *__restrict__ arena, const uint64_t *__restrict__ fbase,
                            const gck_rec *__restrict__ kd, const uint64_t *__restrict__ pos,
                            const uint64_t *__restrict__ hpos, const uint32_t *__restrict__ fstart,
                            const uint64_t *__restrict__ foot, uint32_t nf, uint64_t n, uint8_t *__restrict__ hints) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t w0 = i - lane;  // the wavefront's first record
    // (every lane stays to the wave-wide prefix below; lanes past n carry 0)
    unsigned long long c = 0;
    gck_rec r{};
    uint32_t lo = 0;
    uint64_t i0 = 0, fo = 0;
    if (i < n) {
        r = kd[i];
        // the merged file of record i: the last k with fstart[k] <= i
        uint32_t hi = nf - 1;
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) / 2;
            if (fstart[mid] <= i) lo = mid; else hi = mid - 1;
        }
        i0 = fstart[lo];
        fo = pos[i] - pos[i0];  // the record's offset in its merged file
        uint8_t *d = hints + hpos[i] + foot[lo];
        const uint8_t *key = arena + fbase[r.file] + r.rec_off + 16;
        // 16 B pieces at any alignment: the key's last 16 bytes first (a key
        // under 16 B reaches back into the entry's header, from the record's
        // header in the arena: written over below), then its whole pieces, then
        // the header -- one thread's stores land in program order.  (Byte stores:
        // 370 us for C3's 138 MB of hints, pieces 215 us, profiles/r4zzf.)
        const uint32_t kl = r.key_len;
        if (kl & 15) st16u(d + kHintHdr + kl - 16, ld16u(key + kl - 16));
        for (uint32_t k = 0; k + 16 <= kl; k += 16) st16u(d + kHintHdr + k, ld16u(key + k));
        st16u(d, make_uint4(r.ts, r.key_len, r.value_size, (uint32_t)(fo + 16 + r.key_len)));
        st4u(d + 16, r.crc);
        c = cmp_entry_check(arena, fbase, r, fo);
    }
    // inclusive prefix XOR of the entries' words over the wavefront: a block
    // [i, i1) inside the wave is P[i1 - 1] ^ P[i - 1] (files in between cancel)
    unsigned long long P = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned long long y = __shfl_up(P, d);
        if (lane >= (uint32_t)d) P ^= y;
    }
    const uint64_t j = i - i0;
    const bool idx = i < n && j % GCK_HINT_BLOCK == 0;
    const uint64_t i1 = idx ? min<uint64_t>(i + GCK_HINT_BLOCK, (uint64_t)fstart[lo + 1]) : i + 1;
    const uint32_t last = (uint32_t)(min<uint64_t>(i1, w0 + 64) - 1 - w0);  // the block's last lane in this wave
    const unsigned long long P_last = __shfl(P, (int)last), P_before = __shfl(P, (int)(lane ? lane - 1 : 0));
    if (idx) {
        // the block's index entry, after the file's entries: its first entry's
        // hint and data offsets, and the XOR of its entries' integrity words
        unsigned long long chk = P_last ^ (lane ? P_before : 0ull);
        for (uint64_t t = w0 + 64; t < i1; ++t) chk ^= cmp_entry_check(arena, fbase, kd[t], pos[t] - pos[i0]);  // (past the wave)
        const uint64_t h0 = hpos[i0] + foot[lo];  // the hint file's first byte
        const uint64_t ebytes = hpos[fstart[lo + 1]] - hpos[i0];
        uint8_t *x = hints + h0 + ebytes + kHintIdx * (j / GCK_HINT_BLOCK);
        st16u(x, make_uint4((uint32_t)(hpos[i] - hpos[i0]), (uint32_t)((hpos[i] - hpos[i0]) >> 32), (uint32_t)fo,
                            (uint32_t)(fo >> 32)));
        st4u(x + 16, (uint32_t)chk);
        st4u(x + 20, (uint32_t)(chk >> 32));
    }
}

// Every hint file's tail (a lane per file; a file may have no entries).
__global__ void k_cmp_hint_tails(const uint64_t *__restrict__ pos, const uint64_t *__restrict__ hpos,
                                 const uint32_t *__restrict__ fstart, const uint64_t *__restrict__ foot, uint32_t nf,
                                 uint8_t *__restrict__ hints) {
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= nf) return;
    const uint64_t a = fstart[f], b = fstart[f + 1], ne = b - a, eb = hpos[b] - hpos[a], db = pos[b] - pos[a];
    uint8_t *t = hints + hpos[a] + foot[f] + eb + hint_footer(ne) - kHintTail;
    st16u(t, make_uint4((uint32_t)ne, (uint32_t)(ne >> 32), (uint32_t)eb, (uint32_t)(eb >> 32)));
    st16u(t + 16, make_uint4((uint32_t)db, (uint32_t)(db >> 32), GCK_HINT_MAGIC, GCK_HINT_VERSION));
}

}  // namespace gck

using namespace gck;

namespace {
// hipEvents destroyed on every return path
struct EvPair {
    hipEvent_t a = nullptr, b = nullptr;
    ~EvPair() {
        if (a) (void)hipEventDestroy(a);
        if (b) (void)hipEventDestroy(b);
    }
};
constexpr uint64_t kSerialBreakFiles = 256;  // up to this many merged files: the one-wavefront search
}  // namespace

extern "C" int gck_ctx_compact(gck_ctx *ctx, uint64_t max_file_size, uint32_t *n_files, uint64_t *data_bytes,
                               uint64_t *hint_bytes, double *ms) {
    if (!ctx || !n_files || !data_bytes || !hint_bytes || max_file_size == 0) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    // the keydir must describe the last run (gck_ctx_run invalidates it), and
    // that run must have opened: the reference refuses a database whose replay
    // hit a startup error (core/db.go:134-138), so there is nothing to merge
    if (!c->kd_valid || c->status != GCK_OK || c->from_hints) return GCK_EINVAL;  // (a hint replay holds no records)
    if (c->kd_flags & GCK_KD_KEEP_TOMBSTONES) return GCK_EINVAL;  // a merge keeps Puts only
    GCK_HIP(hipSetDevice(c->device));
    const uint64_t n = c->n_live;
    if (n > 0xFFFFFFF0ull) return GCK_EINVAL;
    const uint64_t nb = (n + kCmpBlock - 1) / kCmpBlock;
    const uint32_t cap = (uint32_t)n + 2;  // files: at most one per record, plus an empty first one
    int rc;
    if ((rc = c->d_cpos.ensure((n + 1) * 8)) || (rc = c->d_chpos.ensure((n + 1) * 8)) ||
        (rc = c->d_cbsum.ensure((nb + 1) * 16)) || (rc = c->d_cfstart.ensure((uint64_t)(cap + 1) * 4)) ||
        (rc = c->d_cnf.ensure(16)))
        return rc;
    hipStream_t s = c->stream;
    EvPair ev;
    GCK_HIP(hipEventCreate(&ev.a));
    GCK_HIP(hipEventCreate(&ev.b));
    GCK_HIP(hipEventRecord(ev.a, s));
    uint64_t *pos = c->d_cpos.as<uint64_t>(), *hpos = c->d_chpos.as<uint64_t>();
    uint64_t *bsum = c->d_cbsum.as<uint64_t>(), *hbsum = bsum + nb + 1;
    if (nb) k_cmp_sizes<<<(uint32_t)nb, kCmpBlock, 0, s>>>(c->d_kdout.as<gck_rec>(), n, pos, hpos, bsum, hbsum);
    k_cmp_top<<<1, 1024, 0, s>>>(bsum, hbsum, nb);
    k_cmp_add<<<(uint32_t)((n + 1 + 255) / 256), 256, 0, s>>>(pos, hpos, bsum, hbsum, n, nb);
    uint64_t tot[3] = {0, 0, 0};  // data bytes, hint bytes, pos[1]
    uint32_t nf = 0;
    GCK_HIP(hipMemcpyAsync(&tot[0], pos + n, 8, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipMemcpyAsync(&tot[1], hpos + n, 8, hipMemcpyDeviceToHost, s));
    if (n) GCK_HIP(hipMemcpyAsync(&tot[2], pos + 1, 8, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    // consecutive merged files hold more than M together (a file closes when
    // the next entry does not fit), so there are at most 2 bytes / M + 2
    const uint64_t est = std::min<uint64_t>(2 * (tot[0] / max_file_size) + 2, (uint64_t)cap);
    if (n == 0 || est <= kSerialBreakFiles) {
        k_cmp_breaks<<<1, 64, 0, s>>>(pos, n, max_file_size, c->d_cfstart.as<uint32_t>(), cap + 1, c->d_cnf.as<uint32_t>());
    } else {
        if ((rc = c->d_cjmp.ensure((n + 1) * 8 + (n + 1) * 4)) || (rc = c->d_con.ensure(n * 4 + 16))) return rc;
        uint32_t *jmp = c->d_cjmp.as<uint32_t>(), *jmp2 = jmp + (n + 1), *on = c->d_con.as<uint32_t>();
        const uint32_t g1 = (uint32_t)((n + 1 + 255) / 256);
        k_cmp_next<<<g1, 256, 0, s>>>(pos, n, max_file_size, jmp, on);
        for (uint64_t reach = 1; reach < est; reach <<= 1) {  // starts within `reach` steps of record 0 are marked
            k_cmp_mark<<<g1, 256, 0, s>>>(jmp, on, n);
            if (reach * 2 < est) {
                k_cmp_jump<<<g1, 256, 0, s>>>(jmp, jmp2, n);
                std::swap(jmp, jmp2);
            }
        }
        k_cmp_fcount<<<(uint32_t)nb, kCmpBlock, 0, s>>>(on, n, bsum);
        const uint32_t lead = tot[2] > max_file_size ? 1u : 0u;  // pos[1] - pos[0] (= 0) > M: an empty first file
        k_cmp_ftop<<<1, 64, 0, s>>>(bsum, nb, lead, c->d_cfstart.as<uint32_t>(), n, c->d_cnf.as<uint32_t>());
        k_cmp_fscatter<<<(uint32_t)nb, kCmpBlock, 0, s>>>(on, n, bsum, c->d_cfstart.as<uint32_t>() + lead);
    }
    GCK_HIP(hipMemcpyAsync(&nf, c->d_cnf.p, 4, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    // each hint file's index and tail follow its entries: foot[f] = the index
    // and tail bytes of the files before f (from the files' record counts)
    std::vector<uint32_t> fs(nf + 1);
    GCK_HIP(hipMemcpy(fs.data(), c->d_cfstart.p, (nf + 1) * 4ull, hipMemcpyDeviceToHost));
    std::vector<uint64_t> foot(nf + 1, 0);
    for (uint32_t k = 0; k < nf; ++k) {
        if (fs[k] > fs[k + 1] || fs[k + 1] > n) return GCK_EDEVICE;  // file starts in order (never trusted blindly)
        foot[k + 1] = foot[k] + hint_footer(fs[k + 1] - fs[k]);
    }
    tot[1] += foot[nf];
    if ((rc = c->d_cdata.ensure(tot[0] + 16)) || (rc = c->d_chint.ensure(tot[1] + 16)) ||
        (rc = c->d_cfoot.ensure((nf + 1) * 8ull)))
        return rc;
    GCK_HIP(hipMemcpyAsync(c->d_cfoot.p, foot.data(), (nf + 1) * 8ull, hipMemcpyHostToDevice, s));
    if (n) {
        const uint64_t groups = (n + 63) / 64;
        // 16 wavefronts per CU, groups from an atomic queue: 6.41-6.43 ms on
        // C3 against 6.88-6.94 with a static stride (which itself had been
        // 7.22-7.26 at 32 wavefronts); 32 or 8 with the queue slower
        // (profiles/r4zzg, r4zzh, r4zzi)
        const uint32_t grid = (uint32_t)std::min<uint64_t>((groups + 3) / 4, (uint64_t)c->n_cu * 4);
        uint32_t *queue = c->d_queue.as<uint32_t>() + kQueueCompact;
        GCK_HIP(hipMemsetAsync(queue, 0, 4, s));
        k_cmp_copy<<<grid, 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(), c->d_kdout.as<gck_rec>(), pos, n,
                                        c->d_cdata.as<uint8_t>(), queue);
        k_cmp_hints<<<(uint32_t)((n + 255) / 256), 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_fbase.as<uint64_t>(),
                                                               c->d_kdout.as<gck_rec>(), pos, hpos,
                                                               c->d_cfstart.as<uint32_t>(), c->d_cfoot.as<uint64_t>(),
                                                               nf, n, c->d_chint.as<uint8_t>());
    }
    if (nf)
        k_cmp_hint_tails<<<(nf + 255) / 256, 256, 0, s>>>(pos, hpos, c->d_cfstart.as<uint32_t>(), c->d_cfoot.as<uint64_t>(),
                                                         nf, c->d_chint.as<uint8_t>());
    GCK_HIP(hipGetLastError());
    GCK_HIP(hipEventRecord(ev.b, s));
    GCK_HIP(hipEventSynchronize(ev.b));
    float t = 0;
    GCK_HIP(hipEventElapsedTime(&t, ev.a, ev.b));
    if (ms) *ms = t;
    c->cmp_files = nf;
    c->cmp_data = tot[0];
    c->cmp_hint = tot[1];
    *n_files = nf;
    *data_bytes = tot[0];
    *hint_bytes = tot[1];
    return GCK_OK;
}

extern "C" int gck_ctx_fetch_compact(gck_ctx *ctx, uint8_t *data, uint64_t *file_sizes, uint8_t *hints,
                                     uint64_t *hint_sizes) {
    if (!ctx) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    GCK_HIP(hipSetDevice(c->device));
    const uint32_t nf = c->cmp_files;
    const uint64_t n = c->n_live;
    std::vector<uint32_t> fs(nf + 1);
    if (nf) GCK_HIP(hipMemcpy(fs.data(), c->d_cfstart.p, (nf + 1) * 4, hipMemcpyDeviceToHost));
    for (uint32_t k = 0; k < nf; ++k)  // file starts are record indices in order (never trust them blindly)
        if (fs[k] > fs[k + 1] || fs[k + 1] > n) return GCK_EDEVICE;
    std::vector<uint64_t> pos(n + 1), hpos(n + 1);
    if (file_sizes || hint_sizes) {
        GCK_HIP(hipMemcpy(pos.data(), c->d_cpos.p, (n + 1) * 8, hipMemcpyDeviceToHost));
        GCK_HIP(hipMemcpy(hpos.data(), c->d_chpos.p, (n + 1) * 8, hipMemcpyDeviceToHost));
        for (uint32_t k = 0; k < nf; ++k) {
            if (file_sizes) file_sizes[k] = pos[fs[k + 1]] - pos[fs[k]];
            if (hint_sizes) hint_sizes[k] = hpos[fs[k + 1]] - hpos[fs[k]] + hint_footer(fs[k + 1] - fs[k]);
        }
    }
    if (data && c->cmp_data) GCK_HIP(hipMemcpy(data, c->d_cdata.p, c->cmp_data, hipMemcpyDeviceToHost));
    if (hints && c->cmp_hint) GCK_HIP(hipMemcpy(hints, c->d_chint.p, c->cmp_hint, hipMemcpyDeviceToHost));
    return GCK_OK;
}
