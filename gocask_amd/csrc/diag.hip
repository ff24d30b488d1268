// diag.hip — measurement helpers (not on the replay path), built as the
// separate libgocask_diag.so (gck_diag.h), linked against libgocask_hip.so.
//
// gck_diag_stream_read: a plain streaming read of the resident arena (16 B per
// lane, grid-stride, non-temporal loads — the faster of the two policies, as
// k_crc_rows uses — XOR-reduced so nothing is dead-code eliminated).  It is
// the practical HBM read ceiling that k_crc_rows is compared against in
// bench.py / DESIGN.md (SURVEY.md §8d asks for the fraction of a measured
// streaming-read kernel besides the spec peak).
#include <cstring>

#include "gck_internal.h"
#include "gck_diag.h"

namespace gck {

template <bool NT = false>
__device__ __forceinline__ uint4 ld16(const uint4 *p) {
    if constexpr (NT) {
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(p));
        return make_uint4(v.x, v.y, v.z, v.w);
    } else
        return *p;
}
template <bool NT = false>
__global__ __launch_bounds__(256) void k_stream_read(const uint4 *__restrict__ p, uint64_t n16, uint32_t *sink) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 4;
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x * 4 + threadIdx.x; i < n16; i += stride) {
        uint4 a = ld16<NT>(p + i);
        uint4 b = i + 256 < n16 ? ld16<NT>(p + i + 256) : make_uint4(0, 0, 0, 0);
        uint4 c = i + 512 < n16 ? ld16<NT>(p + i + 512) : make_uint4(0, 0, 0, 0);
        uint4 d = i + 768 < n16 ? ld16<NT>(p + i + 768) : make_uint4(0, 0, 0, 0);
        acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.y ^ c.z ^ c.w ^ d.x ^ d.y ^ d.z ^ d.w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;  // practically never: keeps the loads live
}

// Row-streaming probes with k_crc_rows' geometry (1024-thread workgroups, one
// per CU, a wavefront per 4 KiB row, two rows in flight): SLAB = lane l reads
// its 64 contiguous bytes as 4 x 16 B (lane stride 64 B, the k_crc_rows
// layout); otherwise lane l reads 16 B at 16 l + 1024 j (each instruction
// reads 1 KiB contiguous).
template <bool SLAB>
__global__ __launch_bounds__(1024) void k_stream_rows(const uint8_t *__restrict__ arena, uint64_t n_rows,
                                                      uint32_t *sink) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t stride = (uint64_t)gridDim.x * 16;
    uint32_t acc = 0;
    for (uint64_t row = blockIdx.x * 16 + (threadIdx.x >> 6); row < n_rows; row += 2 * stride) {
        const uint64_t row2 = min(row + stride, n_rows - 1);
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t off = SLAB ? lane * 64 + 16 * j : lane * 16 + 1024 * j;
            v[j] = *reinterpret_cast<const uint4 *>(arena + row * 4096 + off);
            v[4 + j] = *reinterpret_cast<const uint4 *>(arena + row2 * 4096 + off);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// The same with non-temporal loads in k_crc_rows' current geometry (lane
// p + 16 b at 1024 j + 64 p + 16 b, one row per step, the next row issued
// before the current one is consumed): BLOCKS = each wavefront streams whole
// 64-row blocks (256 KiB, block index strided over the wavefronts), as
// k_crc_rows' work items; otherwise rows are strided over the wavefronts
// (neighbouring wavefronts read neighbouring rows).
template <bool BLOCKS>
__global__ __launch_bounds__(1024) void k_stream_rows_nt(const uint8_t *__restrict__ arena, uint64_t n_rows,
                                                         uint32_t *sink) {
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const uint32_t lane = threadIdx.x & 63, off = 64 * (lane & 15) + 16 * (lane >> 4);
    const uint64_t wv = (uint64_t)blockIdx.x * 16 + (threadIdx.x >> 6), nw = (uint64_t)gridDim.x * 16;
    auto row_of = [&](uint64_t k) -> uint64_t {  // the wave's k-th row
        return BLOCKS ? ((k / 64) * nw + wv) * 64 + (k % 64) : k * nw + wv;
    };
    auto ld = [&](uint64_t row, v4u (&v)[4]) {
        const uint64_t r = min(row, n_rows - 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(arena + r * 4096 + off + 1024 * j));
    };
    uint32_t acc = 0;
    v4u A[4], B[4];
    uint64_t k = 0;
    if (row_of(0) >= n_rows) return;
    ld(row_of(0), A);
    for (;;) {
        ld(row_of(k + 1), B);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc ^= A[j].x ^ A[j].y ^ A[j].z ^ A[j].w;
        if (row_of(k + 1) >= n_rows) break;
        ld(row_of(k + 2), A);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc ^= B[j].x ^ B[j].y ^ B[j].z ^ B[j].w;
        if (row_of(k + 2) >= n_rows) break;
        k += 2;
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// The XCD-balanced stream ceiling: k_crc_rows' geometry and work assignment
// with its compute removed -- 1024-thread workgroups, one per CU (the 160 KiB
// of LDS declared, as k_crc_rows' tables, so occupancy matches), 64-row blocks,
// the first static_eighths / 8 of the full rounds static (wavefront w of W
// takes blocks k W + w), the rest claimed from an atomic queue two blocks at a
// time, one row's four 16 B non-temporal buffer loads (whole KiB per
// instruction) issued before the previous row is consumed.  A static grid
// stride (k_stream_read) leaves XCDs that finish early idle while others still
// read (in-kernel stamps); the queue keeps every XCD busy to
// the end, as in k_crc_rows.  STAMP: each wavefront stamps (shader clock,
// 100 MHz real time) at start and end plus its XCC id into g_dclk.
constexpr uint32_t kDclkWaves = 16384;
__device__ uint64_t g_dclk[4 * kDclkWaves];
__device__ uint32_t g_dxcc[kDclkWaves];

template <bool STAMP>
__global__ __launch_bounds__(1024) void k_stream_blocks(const uint8_t *__restrict__ arena, uint64_t n_rows,
                                                        uint32_t *__restrict__ queue, uint32_t *sink,
                                                        uint32_t static_eighths) {
    __shared__ uint32_t lds[40960];
    uint64_t t0 = 0, r0 = 0;
    if constexpr (STAMP) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    constexpr uint32_t kRowsPerBlock = 64, kClaimBlocks = 2;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t s_rel = 64 * (lane & 15) + 16 * (lane >> 4);
    const uint64_t n_blocks = (n_rows + kRowsPerBlock - 1) / kRowsPerBlock;
    const uint32_t W = gridDim.x * 16;
    const uint32_t w = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * 16 + (threadIdx.x >> 6)));
    const uint32_t n_static = (uint32_t)(n_blocks / W) * static_eighths / 8;
    uint32_t st_k = 0, last = kClaimBlocks - 1;
    auto grab = [&]() -> uint64_t {
        if (st_k < n_static) return (uint64_t)(st_k++) * W + w;
        if (last % kClaimBlocks == kClaimBlocks - 1) {
            uint32_t v = 0;
            if (lane == 0) v = atomicAdd(queue, 1u);
            last = n_static * W + kClaimBlocks * (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
        } else {
            ++last;
        }
        return last;
    };
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    auto issue = [&](uint64_t row, v4u (&v)[4]) {
        const uint32_t r = min((uint32_t)row, (uint32_t)(n_rows - 1));
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(arena + (uint64_t)r * 4096), 0, 4096, 0x00020000);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, s_rel + 1024 * k, 0, 2);
    };
    uint32_t acc = 0;
    uint64_t q = grab();
    if (q < n_blocks) {
        v4u A[4], B[4];
        issue(q * kRowsPerBlock, A);
        for (;;) {
            const uint64_t qn = grab();
            const uint64_t rb = q * kRowsPerBlock;
            for (uint32_t j = 0; j < kRowsPerBlock; j += 2) {
                issue(rb + j + 1, B);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 4; ++k) acc ^= A[k].x ^ A[k].y ^ A[k].z ^ A[k].w;
                issue(j + 2 < kRowsPerBlock ? rb + j + 2 : qn * kRowsPerBlock, A);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 4; ++k) acc ^= B[k].x ^ B[k].y ^ B[k].z ^ B[k].w;
            }
            if (qn >= n_blocks) break;
            q = qn;
        }
    }
    if (acc == 0x9E3779B9u) {
        lds[threadIdx.x] = acc;
        sink[0] = lds[(threadIdx.x + 1) & 1023];
    }
    if constexpr (STAMP) {
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        const uint32_t wi = blockIdx.x * 16 + (threadIdx.x >> 6);
        if (lane == 0 && wi < kDclkWaves) {
            g_dclk[4 * wi] = t0;
            g_dclk[4 * wi + 1] = r0;
            g_dclk[4 * wi + 2] = t1;
            g_dclk[4 * wi + 3] = r1;
            g_dxcc[wi] = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;  // HW_REG_XCC_ID[3:0]
        }
    }
}

// Stream probes for the bytes-in-flight question (round 6): k_crc_rows' row
// loads (lane p + 16 b reads the 16 B at 1024 k + 64 p + 16 b, non-temporal
// buffer loads) with PF rows in flight per wavefront, no compute.  MODE 0:
// rows strided over the wavefronts (row k W + w); otherwise whole 64-row
// blocks: 1 static (block k W + w), 2 all from an atomic queue (each claimed
// as the block before starts), 3 k_crc_rows' split (the first half of the
// full rounds static, the rest from the queue), 4 static with the
// wavefronts of a round scattered over its blocks (block k W + (w * odd mod
// W), W a power of two: a CU's wavefronts no longer read neighbouring
// blocks), 5 static with a dummy queue claim per block (the atomics of
// mode 2 without their order); 6 / 7: modes 3 / 2 with one queue per XCD
// (queue j hands out the queued blocks j, j + 8, ...; a wavefront claims from
// its XCD's queue and moves to the next queue when that one runs dry), the
// eight counters 256 B apart.  Occupancy is set by the
// workgroup size and the dynamic LDS the launch asks for.
template <int PF, int MODE>
__global__ void k_stream_xp(const uint8_t *__restrict__ arena, uint64_t n_rows, uint32_t *sink, int stamp,
                            uint32_t *queue) {
    extern __shared__ uint32_t dyn_lds[];
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const uint32_t lane = threadIdx.x & 63, s_rel = 64 * (lane & 15) + 16 * (lane >> 4);
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x / 64);
    const uint64_t w = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)));
    const uint64_t n_blocks = (n_rows + 63) / 64;
    const uint64_t n_static = MODE == 1 || MODE == 4 || MODE == 5 ? ~0ull : MODE == 3 || MODE == 6 ? n_blocks / W / 2 : 0;
    uint32_t qj = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u, q_tries = 0;  // (HW_REG_XCC_ID)
    uint64_t st_k = 0;
    const uint64_t ws = MODE == 4 ? (w * 0x9E3779B1ull) & (W - 1) : w;
    auto grab = [&]() -> uint64_t {  // the wavefront's next block
        if (st_k < n_static) {
            if (MODE == 5) {
                uint32_t v = 0;
                if (lane == 0) v = atomicAdd(queue, 1u);
                if (__builtin_amdgcn_readfirstlane((int)v) == -1) return n_blocks;  // (never: keeps the atomic)
            }
            return (st_k++) * W + ws;
        }
        if (MODE == 6 || MODE == 7) {
            for (;;) {
                uint32_t v = 0;
                if (lane == 0) v = atomicAdd(queue + 64 * qj, 1u);
                const uint64_t b = n_static * W + 8ull * (uint32_t)__builtin_amdgcn_readfirstlane((int)v) + qj;
                if (b < n_blocks || q_tries == 7) return b < n_blocks ? b : n_blocks;
                ++q_tries;
                qj = (qj + 1) & 7u;
            }
        }
        uint32_t v = 0;
        if (lane == 0) v = atomicAdd(queue, 1u);
        return n_static * W + (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
    };
    uint64_t bq[2] = {0, 0};  // the blocks of sequence positions 64 j (j even, odd)
    if (MODE != 0) {
        bq[0] = grab();
        bq[1] = grab();
    }
    auto row_of = [&](uint64_t k) -> uint64_t {  // the wavefront's k-th row
        if (MODE == 0) return k * W + w;
        const uint64_t b = bq[(k / 64) & 1];
        return b < n_blocks ? b * 64 + (k % 64) : n_rows;
    };
    auto issue = [&](uint64_t row, v4u (&v)[4]) {
        const uint32_t r = (uint32_t)min(row, n_rows - 1);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t *>(arena + (uint64_t)r * 4096), 0, 4096, 0x00020000);
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, s_rel + 1024 * k, 0, 2);
    };
    uint32_t acc = 0;
    if (row_of(0) < n_rows) {
        v4u B[PF + 1][4];
#pragma unroll
        for (int d = 0; d < PF; ++d) issue(row_of(d), B[d]);
        for (uint64_t k = 0;; k += PF + 1) {
#pragma unroll
            for (int u = 0; u <= PF; ++u) {
                issue(row_of(k + u + PF), B[(u + PF) % (PF + 1)]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int j = 0; j < 4; ++j) acc ^= B[u][j].x ^ B[u][j].y ^ B[u][j].z ^ B[u][j].w;
                // a block starts: claim the one after it (its rows are issued
                // PF rows before they are read)
                if (MODE != 0 && (k + u + 1) % 64 == 0) bq[((k + u + 1) / 64 + 1) & 1] = grab();
                if (row_of(k + u + 1) >= n_rows) goto done;
            }
        }
    }
done:
    if (acc == 0x9E3779B9u) {
        dyn_lds[threadIdx.x] = acc;
        sink[0] = dyn_lds[(threadIdx.x + 1) % blockDim.x];
    }
    if (stamp) {  // (as k_stream_blocks<true>: gck_diag_clock_read)
        const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0 && w < kDclkWaves) {
            g_dclk[4 * w] = t0;
            g_dclk[4 * w + 1] = r0;
            g_dclk[4 * w + 2] = t1;
            g_dclk[4 * w + 3] = r1;
            g_dxcc[w] = (uint32_t)__builtin_amdgcn_s_getreg((3 << 11) | 20) & 15u;  // HW_REG_XCC_ID[3:0]
        }
    }
}

// Random-access probes with k_walk's access shape (a 16 B load per hop):
// DEP = each lane's next address depends on the bytes it just loaded (a chain
// walk); otherwise the lane's hops are independent (8 loads in flight).
template <bool DEP>
__global__ __launch_bounds__(256) void k_chase(const uint8_t *__restrict__ arena, uint64_t len, uint32_t lanes,
                                               uint32_t hops, uint32_t *sink) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x;
    if (t >= lanes) return;
    const uint64_t n16 = (len >> 4) - 4;
    uint64_t x = 0x9E3779B97F4A7C15ull * (t + 1);
    auto pick = [&](uint64_t v) {
        v = (v ^ (v >> 31)) * 0xBF58476D1CE4E5B9ull;
        v ^= v >> 29;
        return (((v & 0xFFFFFFFFull) * n16) >> 32) << 4;
    };
    uint32_t acc = 0;
    if (DEP) {
        uint64_t o = pick(x);
        for (uint32_t h = 0; h < hops; ++h) {
            const uint4 a = *reinterpret_cast<const uint4 *>(arena + o);
            acc += a.x ^ a.y ^ a.z ^ a.w;
            o = pick(x + acc + h);
        }
    } else {
        for (uint32_t h = 0; h < hops; h += 8) {
            uint4 a[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) a[j] = *reinterpret_cast<const uint4 *>(arena + pick(x + h + j));
#pragma unroll
            for (int j = 0; j < 8; ++j) acc += a[j].x ^ a[j].y ^ a[j].z ^ a[j].w;
        }
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

// Window probe for a walk that reads W = 16 LPC bytes per round trip: 65,536
// dependent chains (k_walk's concurrency), LPC lanes per chain each loading
// 16 B of the chain's window; the next address depends on the whole window
// (an XOR over the chain's lanes).  hops = round trips per chain.
template <int LPC>
__global__ __launch_bounds__(256) void k_chase_win(const uint8_t *__restrict__ arena, uint64_t len, uint32_t hops,
                                                   uint32_t *sink) {
    const uint32_t t = blockIdx.x * 256 + threadIdx.x, chain = t / LPC, sub = t % LPC;
    const uint64_t n16 = (len >> 4) - 64;
    auto pick = [&](uint64_t v) {
        v = (v ^ (v >> 31)) * 0xBF58476D1CE4E5B9ull;
        v ^= v >> 29;
        return (((v & 0xFFFFFFFFull) * n16) >> 32) << 4;
    };
    const uint64_t x = 0x9E3779B97F4A7C15ull * (chain + 1);
    uint32_t acc = 0;
    uint64_t o = pick(x);
    for (uint32_t h = 0; h < hops; ++h) {
        const uint4 a = *reinterpret_cast<const uint4 *>(arena + o + 16 * sub);
        uint32_t v = a.x ^ a.y ^ a.z ^ a.w;
#pragma unroll
        for (int m = 1; m < LPC; m <<= 1) v ^= (uint32_t)__shfl_xor((int)v, m);
        acc += v;
        o = pick(x + acc + h);
    }
    if (acc == 0x9E3779B9u) sink[0] = acc;
}

}  // namespace gck

using namespace gck;

// Window probes: k_chase_win<lpc> with `hops` round trips per chain.
extern "C" int gck_diag_chase_win(gck_ctx *ctx, int lpc, uint32_t hops, int iters, double *ms_per_iter) {
    if (!ctx || iters <= 0 || !(lpc == 1 || lpc == 4 || lpc == 8 || lpc == 16 || lpc == 32)) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    GCK_HIP(hipSetDevice(c->device));
    if (!c->n_rows) return GCK_EINVAL;
    uint32_t *sink = c->d_counters.as<uint32_t>() + 14;
    const uint32_t threads = 65536u * (uint32_t)lpc, grid = threads / 256;
    auto launch = [&]() {
        uint8_t *a = c->arena.as<uint8_t>();
        const uint64_t n = c->arena_len;
        if (lpc == 1) k_chase_win<1><<<grid, 256, 0, c->stream>>>(a, n, hops, sink);
        else if (lpc == 4) k_chase_win<4><<<grid, 256, 0, c->stream>>>(a, n, hops, sink);
        else if (lpc == 8) k_chase_win<8><<<grid, 256, 0, c->stream>>>(a, n, hops, sink);
        else if (lpc == 16) k_chase_win<16><<<grid, 256, 0, c->stream>>>(a, n, hops, sink);
        else k_chase_win<32><<<grid, 256, 0, c->stream>>>(a, n, hops, sink);
    };
    hipEvent_t e0, e1;
    GCK_HIP(hipEventCreate(&e0));
    GCK_HIP(hipEventCreate(&e1));
    launch();
    GCK_HIP(hipEventRecord(e0, c->stream));
    for (int i = 0; i < iters; ++i) launch();
    GCK_HIP(hipEventRecord(e1, c->stream));
    GCK_HIP(hipEventSynchronize(e1));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    *ms_per_iter = ms / iters;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return GCK_OK;
}

// pattern 0: k_stream_read; 15: the same with non-temporal loads; 1: k_stream_rows<SLAB>; 2: k_stream_rows<coalesced>;
// 16: k_stream_rows_nt, rows strided over the wavefronts; 17: the same in 64-row blocks;
// 3..8: k_chase<dependent> with 8 Ki << (pattern-3) lanes; 9..14: the same
// lane counts, independent loads.  The chase patterns make 10,240,000 hops in
// all (C3's record count); *gbs reports hops per ns (G hops/s) for them.
extern "C" int gck_diag_stream_pattern(gck_ctx *ctx, int pattern, int iters, double *ms_per_iter, double *gbs) {
    if (!ctx || iters <= 0 || pattern < 0 || pattern > 17) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    GCK_HIP(hipSetDevice(c->device));
    if (!c->n_rows) return GCK_EINVAL;
    uint32_t *sink = c->d_counters.as<uint32_t>() + 14;
    const uint32_t lanes = pattern >= 3 && pattern <= 14 ? 8192u << ((pattern - 3) % 6) : 0u;
    const uint32_t hops = lanes ? ((10240000u / lanes + 7) & ~7u) : 0u;
    auto launch = [&]() {
        if (pattern == 16)
            k_stream_rows_nt<false><<<c->n_cu, 1024, 0, c->stream>>>(c->arena.as<uint8_t>(), c->n_rows, sink);
        else if (pattern == 17)
            k_stream_rows_nt<true><<<c->n_cu, 1024, 0, c->stream>>>(c->arena.as<uint8_t>(), c->n_rows, sink);
        else if (pattern == 15)
            k_stream_read<true><<<(uint32_t)c->n_cu * 8, 256, 0, c->stream>>>(c->arena.as<uint4>(), c->arena_len / 16, sink);
        else if (pattern >= 9)
            k_chase<false><<<(lanes + 255) / 256, 256, 0, c->stream>>>(c->arena.as<uint8_t>(), c->arena_len, lanes, hops,
                                                                      sink);
        else if (pattern >= 3)
            k_chase<true><<<(lanes + 255) / 256, 256, 0, c->stream>>>(c->arena.as<uint8_t>(), c->arena_len, lanes, hops,
                                                                     sink);
        else if (pattern == 0)
            k_stream_read<false><<<(uint32_t)c->n_cu * 8, 256, 0, c->stream>>>(c->arena.as<uint4>(), c->arena_len / 16, sink);
        else if (pattern == 1)
            k_stream_rows<true><<<c->n_cu, 1024, 0, c->stream>>>(c->arena.as<uint8_t>(), c->n_rows, sink);
        else
            k_stream_rows<false><<<c->n_cu, 1024, 0, c->stream>>>(c->arena.as<uint8_t>(), c->n_rows, sink);
    };
    hipEvent_t a, b;
    GCK_HIP(hipEventCreate(&a));
    GCK_HIP(hipEventCreate(&b));
    launch();  // warm-up
    GCK_HIP(hipEventRecord(a, c->stream));
    for (int i = 0; i < iters; ++i) launch();
    GCK_HIP(hipEventRecord(b, c->stream));
    GCK_HIP(hipEventSynchronize(b));
    float ms = 0;
    GCK_HIP(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    const double per = ms / iters;
    if (ms_per_iter) *ms_per_iter = per;
    if (gbs) *gbs = lanes ? (double)lanes * hops / (per * 1e-3) / 1e9 : (double)c->arena_len / (per * 1e-3) / 1e9;
    return GCK_OK;
}

extern "C" int gck_diag_stream_read(gck_ctx *ctx, int iters, double *ms_per_iter, double *gbs) {
    if (!ctx || iters <= 0) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    GCK_HIP(hipSetDevice(c->device));
    const uint64_t n16 = c->arena_len / 16;
    if (!n16) return GCK_EINVAL;
    const uint32_t grid = (uint32_t)c->n_cu * 8;
    uint32_t *sink = c->d_counters.as<uint32_t>() + 14;
    hipEvent_t a, b;
    GCK_HIP(hipEventCreate(&a));
    GCK_HIP(hipEventCreate(&b));
    k_stream_read<true><<<grid, 256, 0, c->stream>>>(c->arena.as<uint4>(), n16, sink);  // warm-up
    GCK_HIP(hipEventRecord(a, c->stream));
    for (int i = 0; i < iters; ++i) k_stream_read<true><<<grid, 256, 0, c->stream>>>(c->arena.as<uint4>(), n16, sink);
    GCK_HIP(hipEventRecord(b, c->stream));
    GCK_HIP(hipEventSynchronize(b));
    float ms = 0;
    GCK_HIP(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    const double per = ms / iters;
    if (ms_per_iter) *ms_per_iter = per;
    if (gbs) *gbs = (double)c->arena_len / (per * 1e-3) / 1e9;
    return GCK_OK;
}

extern "C" int gck_diag_stream_blocks(gck_ctx *ctx, int iters, uint32_t static_eighths, int stamp,
                                      double *ms_per_iter, double *gbs) {
    if (!ctx || iters <= 0 || static_eighths > 8) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    GCK_HIP(hipSetDevice(c->device));
    if (!c->n_rows) return GCK_EINVAL;
    if (int rc = c->d_queue.ensure(kQueueSlots * 4 + 64)) return rc;
    uint32_t *queue = c->d_queue.as<uint32_t>() + kQueueSlots;  // a slot of its own past the product's queues
    uint32_t *sink = c->d_counters.as<uint32_t>() + 14;
    auto launch = [&](bool st) {
        (void)hipMemsetAsync(queue, 0, 4, c->stream);
        if (st)
            k_stream_blocks<true><<<c->n_cu, 1024, 0, c->stream>>>(c->arena.as<uint8_t>(), c->n_rows, queue, sink,
                                                                   static_eighths);
        else
            k_stream_blocks<false><<<c->n_cu, 1024, 0, c->stream>>>(c->arena.as<uint8_t>(), c->n_rows, queue, sink,
                                                                    static_eighths);
    };
    hipEvent_t a, b;
    GCK_HIP(hipEventCreate(&a));
    GCK_HIP(hipEventCreate(&b));
    launch(false);  // warm-up
    GCK_HIP(hipEventRecord(a, c->stream));
    for (int i = 0; i < iters; ++i) launch(stamp && i == iters - 1);
    GCK_HIP(hipEventRecord(b, c->stream));
    GCK_HIP(hipEventSynchronize(b));
    float ms = 0;
    GCK_HIP(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    const double per = ms / iters;
    if (ms_per_iter) *ms_per_iter = per;
    if (gbs) *gbs = (double)c->arena_len / (per * 1e-3) / 1e9;
    return GCK_OK;
}

// k_stream_xp<pf, blocks> with workgroups of `threads` (64..1024) and
// lds_kib of dynamic LDS each, `wg_per_cu` workgroups per CU in the grid.
extern "C" int gck_diag_stream_xp(gck_ctx *ctx, int pf, int blocks, int threads, int lds_kib, int wg_per_cu,
                                  int iters, int stamp, double *ms_per_iter, double *gbs) {
    if (!ctx || iters <= 0 || pf < 1 || pf > 3 || blocks < 0 || blocks > 7 || threads < 64 || threads > 1024 || threads % 64 || lds_kib < 0 ||
        lds_kib > 160 || wg_per_cu < 1)
        return GCK_EINVAL;
    Ctx *c = &ctx->c;
    GCK_HIP(hipSetDevice(c->device));
    if (!c->n_rows) return GCK_EINVAL;
    uint32_t *sink = c->d_counters.as<uint32_t>() + 14;
    const size_t lds = std::max<size_t>((size_t)lds_kib << 10, threads * 4);
    const uint32_t grid = (uint32_t)(c->n_cu * wg_per_cu);
    int st = 0;  // the last timed launch stamps its wavefronts
    static uint32_t *queue = nullptr;  // 8 counters 256 B apart (zeroed before every launch)
    if (!queue) GCK_HIP(hipMalloc(&queue, 4096));
    auto launch = [&]() {
        (void)hipMemsetAsync(queue, 0, 4096, c->stream);
#define GCK_XP_L(P, M) k_stream_xp<P, M><<<grid, threads, lds, c->stream>>>(c->arena.as<uint8_t>(), c->n_rows, sink, st, queue)
#define GCK_XP_M(M) if (pf == 1) GCK_XP_L(1, M); else if (pf == 2) GCK_XP_L(2, M); else GCK_XP_L(3, M)
        if (blocks == 0) { GCK_XP_M(0); } else if (blocks == 1) { GCK_XP_M(1); } else if (blocks == 2) { GCK_XP_M(2); } else if (blocks == 3) { GCK_XP_M(3); } else if (blocks == 4) { GCK_XP_M(4); } else if (blocks == 5) { GCK_XP_M(5); } else if (blocks == 6) { GCK_XP_M(6); } else { GCK_XP_M(7); }
#undef GCK_XP_M
#undef GCK_XP_L
    };
    // (dynamic LDS above 64 KiB needs the attribute)
#define GCK_XP_A(P, M) GCK_HIP(hipFuncSetAttribute(reinterpret_cast<const void *>(k_stream_xp<P, M>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 << 10))
    GCK_XP_A(1, 0); GCK_XP_A(2, 0); GCK_XP_A(3, 0);
    GCK_XP_A(1, 1); GCK_XP_A(2, 1); GCK_XP_A(3, 1);
    GCK_XP_A(1, 2); GCK_XP_A(2, 2); GCK_XP_A(3, 2);
    GCK_XP_A(1, 3); GCK_XP_A(2, 3); GCK_XP_A(3, 3);
    GCK_XP_A(1, 4); GCK_XP_A(2, 4); GCK_XP_A(3, 4);
    GCK_XP_A(1, 5); GCK_XP_A(2, 5); GCK_XP_A(3, 5);
    GCK_XP_A(1, 6); GCK_XP_A(2, 6); GCK_XP_A(3, 6);
    GCK_XP_A(1, 7); GCK_XP_A(2, 7); GCK_XP_A(3, 7);
#undef GCK_XP_A
    hipEvent_t a, b;
    GCK_HIP(hipEventCreate(&a));
    GCK_HIP(hipEventCreate(&b));
    launch();  // warm-up
    GCK_HIP(hipEventRecord(a, c->stream));
    for (int i = 0; i < iters; ++i) {
        st = stamp && i == iters - 1;
        launch();
    }
    GCK_HIP(hipEventRecord(b, c->stream));
    GCK_HIP(hipEventSynchronize(b));
    float ms = 0;
    GCK_HIP(hipEventElapsedTime(&ms, a, b));
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    const double per = ms / iters;
    if (ms_per_iter) *ms_per_iter = per;
    if (gbs) *gbs = (double)c->n_rows * 4096 / (per * 1e-3) / 1e9;
    return GCK_OK;
}

// The stamps of the last stamped k_stream_blocks / k_stream_xp launch: 4 u64 per wavefront
// (clock, real time at start; clock, real time at end) and its XCC id.
extern "C" int gck_diag_clock_read(uint64_t *stamps, uint32_t *xcc, uint32_t cap_waves) {
    if (!stamps || !xcc || cap_waves < kDclkWaves) return GCK_EINVAL;
    GCK_HIP(hipMemcpyFromSymbol(stamps, HIP_SYMBOL(g_dclk), sizeof(uint64_t) * 4 * kDclkWaves, 0,
                                hipMemcpyDeviceToHost));
    GCK_HIP(hipMemcpyFromSymbol(xcc, HIP_SYMBOL(g_dxcc), sizeof(uint32_t) * kDclkWaves, 0, hipMemcpyDeviceToHost));
    return GCK_OK;
}

// Per-chunk state of the last run: the chain length k_walk followed (records
// staged) and the final entry of every chunk (UINT64_MAX: none), for the
// boundary-phase measurements (tools/chunks.py).
extern "C" int gck_diag_chunks(gck_ctx *ctx, uint32_t *count, uint64_t *entry, uint64_t cap, uint64_t *n) {
    if (!ctx || !n) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    *n = c->n_chunks;
    if (!count || !entry) return GCK_OK;
    if (cap < c->n_chunks) return GCK_EINVAL;
    GCK_HIP(hipSetDevice(c->device));
    GCK_HIP(hipStreamSynchronize(c->stream));
    if (c->n_chunks) {
        GCK_HIP(hipMemcpy(count, c->d_ch_count.p, (uint64_t)c->n_chunks * 4, hipMemcpyDeviceToHost));
        GCK_HIP(hipMemcpy(entry, c->d_ch_entry.p, (uint64_t)c->n_chunks * 8, hipMemcpyDeviceToHost));
    }
    return GCK_OK;
}

static_assert(sizeof(gck_diag_outcome) == sizeof(gck::MultiOutcome), "gck_diag_outcome mirrors gck::MultiOutcome");

extern "C" int gck_diag_multi_resolve(const gck_diag_outcome *sh, uint32_t n, uint32_t nfiles, gck_result *out,
                                      uint8_t *contrib) {
    if ((n && (!sh || !contrib)) || !out) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    gck::multi_resolve(reinterpret_cast<const gck::MultiOutcome *>(sh), n, nfiles, out, contrib);
    return GCK_OK;
}

extern "C" int gck_diag_multi_recv_offsets(const uint64_t *counts, uint32_t nsrc, uint32_t nown, uint64_t *off) {
    if (!off || nown == 0 || (nsrc && !counts)) return GCK_EINVAL;
    gck::multi_recv_offsets(counts, nsrc, nown, off);
    return GCK_OK;
}

extern "C" int gck_diag_replay_multi_loopback(const gck_file *files, uint32_t nfiles, uint32_t nshards,
                                              int32_t device, const gck_opts *opts, gck_result *out) {
    if (!out) return GCK_EINVAL;
    memset(out, 0, sizeof(*out));
    if ((nfiles && !files) || nshards == 0 || nshards > 64) return GCK_EINVAL;
    const std::vector<gck::Src> v = gck::mem_srcs(files, nfiles);
    return gck::replay_multi(v.data(), nfiles, std::vector<int>(nshards, device), opts, out, true);
}
