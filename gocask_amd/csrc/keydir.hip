// keydir.hip — device-side keydir of a replay.
//
// The reference builds map[string]kdEntry by applying every record in walk
// order: set on a Put (core/keydir.go:22-34), delete on a tombstone
// (core/keydir.go:45-49, core/db.go:166-170).  The resulting map holds, for
// every key, its LAST record in walk order if that record is a Put, and no
// entry if it is a tombstone.  This file computes exactly that set on the
// device from the last gck_ctx_run, so only live entries cross PCIe and enter
// the Go map (gck_ctx_fetch_keydir).
#include "gck_internal.h"

namespace gck {

constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr int kKdTile = 1024;  // records per compaction tile (one workgroup)

// Key of a record: KeySize bytes after the header, or ValueSize bytes for a
// tombstone (KeySize 0; core/db.go:151-155).
__device__ __forceinline__ uint32_t key_len(const uint4 &h) { return h.z ? h.z : h.w; }

__device__ __forceinline__ uint64_t mix64d(uint64_t x) {
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Word i (4 key bytes, little-endian) of a key at arena offset o, read as
// aligned dwords and funnel-shifted; bytes past the key are masked to zero
// (the arena is padded, so the word after the key is always readable).
struct KeyWords {
    const uint32_t *w;
    uint32_t sh, len;
    __device__ KeyWords(const uint8_t *arena, uint64_t o, uint32_t n)
        : w(reinterpret_cast<const uint32_t *>(arena + (o & ~3ull))), sh((uint32_t)(o & 3)), len(n) {}
    __device__ __forceinline__ uint32_t operator[](uint32_t i) const {
        const uint32_t v = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
        const uint32_t left = len - 4 * i;
        return left >= 4 ? v : v & ((1u << (8 * left)) - 1u);
    }
};

// k_key_hash: one lane per record, a 64-bit hash of its key bytes.
__global__ __launch_bounds__(256) void k_key_hash(const uint8_t *__restrict__ arena,
                                                  const uint64_t *__restrict__ rec_off,
                                                  const uint4 *__restrict__ rec_hdr, uint64_t n,
                                                  uint64_t *__restrict__ khash) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t len = key_len(rec_hdr[r]);
        const KeyWords k(arena, rec_off[r] + 16, len);
        uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)len << 32);
        for (uint32_t i = 0; 4 * i < len; ++i) h = mix64d(h ^ k[i]) + i;
        khash[r] = mix64d(h);
    }
}

__device__ bool same_key(const uint8_t *__restrict__ arena, const uint64_t *__restrict__ rec_off, uint64_t a,
                         uint64_t b, uint32_t len) {
    const KeyWords ka(arena, rec_off[a] + 16, len), kb(arena, rec_off[b] + 16, len);
    for (uint32_t i = 0; 4 * i < len; ++i)
        if (ka[i] != kb[i]) return false;
    return true;
}

// k_kd_insert: one lane per record into an open-addressing table of record
// indices.  A slot is claimed by CAS; records of the same key (hash, length
// and bytes equal) keep the largest index with atomicMax, so the last writer
// in walk order wins whatever order the lanes run in.  Keys are never removed,
// so a probe sequence never skips a key's slot.
__global__ __launch_bounds__(256) void k_kd_insert(const uint8_t *__restrict__ arena,
                                                   const uint64_t *__restrict__ rec_off,
                                                   const uint4 *__restrict__ rec_hdr,
                                                   const uint64_t *__restrict__ khash, uint64_t n,
                                                   uint32_t *__restrict__ table, uint64_t mask) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t h = khash[r];
        const uint32_t len = key_len(rec_hdr[r]);
        for (uint64_t s = h & mask;; s = (s + 1) & mask) {
            uint32_t cur = __hip_atomic_load(table + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == kEmpty) {
                const uint32_t prev = atomicCAS(table + s, kEmpty, (uint32_t)r);
                if (prev == kEmpty) break;  // claimed
                cur = prev;
            }
            if (khash[cur] == h && key_len(rec_hdr[cur]) == len && same_key(arena, rec_off, cur, r, len)) {
                atomicMax(table + s, (uint32_t)r);  // same key: the later record wins
                break;
            }
        }
    }
}

// k_kd_mark: one lane per slot; the key's winning record is live if it is a
// Put (or, for a merge across shards, always: tombstones then stay as delete
// markers).
__global__ __launch_bounds__(256) void k_kd_mark(const uint32_t *__restrict__ table, uint64_t slots,
                                                 const uint4 *__restrict__ rec_hdr, uint32_t keep_tombstones,
                                                 uint32_t *__restrict__ live) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < slots; s += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t r = table[s];
        if (r != kEmpty && (keep_tombstones || rec_hdr[r].z != 0)) live[r] = 1;
    }
}

// Exclusive rank of v inside a workgroup of kKdTile lanes; the total is out.
__device__ uint32_t block_excl(uint32_t v, uint32_t *wsum, uint32_t &total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(x, d);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (uint32_t i = 0; i < blockDim.x / 64; ++i) {
        base += i < w ? wsum[i] : 0u;
        tot += wsum[i];
    }
    __syncthreads();
    total = tot;
    return base + x - v;
}

// Compaction of the live records in walk order: per-tile counts, one
// workgroup scanning the tile counts, per-tile ranks and the gather.
__global__ __launch_bounds__(kKdTile) void k_kd_tiles(const uint32_t *__restrict__ live, uint64_t n,
                                                      uint32_t *__restrict__ tile_cnt) {
    __shared__ uint32_t wsum[kKdTile / 64];
    const uint64_t r = (uint64_t)blockIdx.x * kKdTile + threadIdx.x;
    uint32_t total;
    (void)block_excl(r < n ? live[r] : 0u, wsum, total);
    if (threadIdx.x == 0) tile_cnt[blockIdx.x] = total;
}

__global__ __launch_bounds__(kKdTile) void k_kd_tile_scan(uint32_t *__restrict__ tile_cnt, uint32_t nt) {
    __shared__ uint32_t wsum[kKdTile / 64];
    uint32_t run = 0;
    for (uint32_t i0 = 0; i0 < nt; i0 += kKdTile) {
        const uint32_t i = i0 + threadIdx.x;
        const uint32_t v = i < nt ? tile_cnt[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_excl(v, wsum, total);
        if (i < nt) tile_cnt[i] = run + ex;
        run += total;
    }
    if (threadIdx.x == 0) tile_cnt[nt] = run;  // the live count
}

__global__ __launch_bounds__(kKdTile) void k_kd_scatter(const uint32_t *__restrict__ live, uint64_t n,
                                                        const uint32_t *__restrict__ tile_base,
                                                        const gck_rec *__restrict__ recs, gck_rec *__restrict__ out) {
    __shared__ uint32_t wsum[kKdTile / 64];
    const uint64_t r = (uint64_t)blockIdx.x * kKdTile + threadIdx.x;
    const uint32_t v = r < n ? live[r] : 0u;
    uint32_t total;
    const uint32_t ex = block_excl(v, wsum, total);
    if (v) out[tile_base[blockIdx.x] + ex] = recs[r];
}

}  // namespace gck

using namespace gck;

extern "C" {

int gck_ctx_keydir(gck_ctx *ctx, uint32_t flags, uint64_t *n_live, double *ms) {
    if (!ctx || !n_live) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    *n_live = 0;
    c->n_live = 0;
    const uint64_t n = c->n_recs;
    if (!n) return GCK_OK;
    if (n >= kEmpty) return GCK_EINVAL;
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    uint64_t slots = 1024;
    while (slots < 2 * n) slots <<= 1;  // load factor <= 1/2
    const uint64_t nt = (n + kKdTile - 1) / kKdTile;
    int rc;
    if ((rc = c->d_khash.ensure(n * 8)) || (rc = c->d_ktab.ensure(slots * 4)) || (rc = c->d_live.ensure(n * 4)) ||
        (rc = c->d_ktile.ensure((nt + 1) * 4)) || (rc = c->d_kdout.ensure(n * sizeof(gck_rec))))
        return rc;
    hipEvent_t a, b;
    GCK_HIP(hipEventCreate(&a));
    GCK_HIP(hipEventCreate(&b));
    GCK_HIP(hipEventRecord(a, s));
    GCK_HIP(hipMemsetAsync(c->d_ktab.p, 0xFF, slots * 4, s));
    GCK_HIP(hipMemsetAsync(c->d_live.p, 0, n * 4, s));
    const uint32_t grid = (uint32_t)c->n_cu * 8;
    k_key_hash<<<grid, 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_rec_off.as<uint64_t>(), c->d_rec_hdr.as<uint4>(), n,
                                    c->d_khash.as<uint64_t>());
    k_kd_insert<<<grid, 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_rec_off.as<uint64_t>(), c->d_rec_hdr.as<uint4>(),
                                     c->d_khash.as<uint64_t>(), n, c->d_ktab.as<uint32_t>(), slots - 1);
    k_kd_mark<<<grid, 256, 0, s>>>(c->d_ktab.as<uint32_t>(), slots, c->d_rec_hdr.as<uint4>(),
                                   (flags & GCK_KD_KEEP_TOMBSTONES) ? 1u : 0u, c->d_live.as<uint32_t>());
    k_kd_tiles<<<(uint32_t)nt, kKdTile, 0, s>>>(c->d_live.as<uint32_t>(), n, c->d_ktile.as<uint32_t>());
    k_kd_tile_scan<<<1, kKdTile, 0, s>>>(c->d_ktile.as<uint32_t>(), (uint32_t)nt);
    k_kd_scatter<<<(uint32_t)nt, kKdTile, 0, s>>>(c->d_live.as<uint32_t>(), n, c->d_ktile.as<uint32_t>(),
                                                  c->d_out.as<gck_rec>(), c->d_kdout.as<gck_rec>());
    GCK_HIP(hipEventRecord(b, s));
    uint32_t live = 0;
    GCK_HIP(hipMemcpyAsync(&live, c->d_ktile.as<uint32_t>() + nt, 4, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    GCK_HIP(hipGetLastError());
    float t = 0;
    (void)hipEventElapsedTime(&t, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (ms) *ms = t;
    c->n_live = live;
    *n_live = live;
    return GCK_OK;
}

int gck_ctx_fetch_keydir(gck_ctx *ctx, gck_rec *dst, uint64_t cap, uint64_t *n) {
    if (!ctx || !n || (cap && !dst)) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    *n = c->n_live;
    if (c->n_live > cap) return GCK_EINVAL;
    if (c->n_live) {
        GCK_HIP(hipSetDevice(c->device));
        GCK_HIP(hipMemcpy(dst, c->d_kdout.p, c->n_live * sizeof(gck_rec), hipMemcpyDeviceToHost));
    }
    return GCK_OK;
}

}  // extern "C"
