// keydir.hip — device-side keydir of a replay.
//
// The reference builds map[string]kdEntry by applying every record in walk
// order: set on a Put (core/keydir.go:22-34), delete on a tombstone
// (core/keydir.go:45-49, core/db.go:166-170).  The resulting map holds, for
// every key, its LAST record in walk order if that record is a Put, and no
// entry if it is a tombstone.  This file computes exactly that set on the
// device from the last gck_ctx_run, so only live entries cross PCIe and enter
// the Go map (gck_ctx_fetch_keydir).
#include "kd_common.h"

namespace gck {

// k_kd_insert: one lane per record: the 64-bit hash of its key (kept in
// khash for the merge), then its insert (kd_common.h kd_insert_rec).  Lanes take the
// records from the last one back: a key's later record then mostly claims its
// slot first and the earlier ones skip the atomicMax (C3: 1.85 -> 1.78 ms).
// A second keydir of the same run (hashed) reads the hashes kept in khash
// instead of the key bytes (1.78 -> 1.53 ms, profiles/r5g).
__global__ __launch_bounds__(256) void k_kd_insert(const uint8_t *__restrict__ arena,
                                                   const uint64_t *__restrict__ rec_off,
                                                   const uint2 *__restrict__ rec_kv, uint64_t n,
                                                   uint64_t *__restrict__ khash,
                                                   unsigned long long *__restrict__ table, uint64_t mask,
                                                   int hashed, uint32_t *__restrict__ kstat, uint64_t bound) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t r = n - 1 - i;
        const uint2 kv = rec_kv[r];
        const uint32_t len = key_len(kv);
        const KeyRegs k(arena, rec_off[r] + 16, len);
        const uint64_t h = hashed ? khash[r] : key_hash(k.m, len);
        if (!hashed) khash[r] = h;
        if (!kd_insert_rec(arena, rec_off, rec_kv, table, mask, h, r, kv.x == 0, k, len, bound, kstat + 2))
            atomicOr(kstat, 1u);
    }
}

// k_kd_mark: one lane per slot; the key's winning record is live if it is a
// Put (or, for a merge across shards, always: tombstones then stay as delete
// markers).  The keys (claimed slots) are counted into
// kstat[1]: the next table of this context is sized by them.
__global__ __launch_bounds__(256) void k_kd_mark(const unsigned long long *__restrict__ table, uint64_t slots,
                                                 uint32_t keep_tombstones, uint32_t *__restrict__ live,
                                                 uint32_t *__restrict__ kstat) {
    uint32_t keys = 0;
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < slots; s += (uint64_t)gridDim.x * blockDim.x) {
        const unsigned long long v = table[kSlotWords * s];
        if (v == kEmptySlot) continue;
        ++keys;
        if (keep_tombstones || !(v & 1)) live[slot_rec(v)] = 1;
    }
    for (int o = 32; o > 0; o >>= 1) keys += __shfl_down(keys, o);
    if ((threadIdx.x & 63) == 0 && keys) atomicAdd(kstat + 1, keys);
}

// Exclusive rank of v inside a workgroup of kKdTile lanes; the total is out.
template <class T>
__device__ T block_excl(T v, T *wsum, T &total) {
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    T x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const T y = __shfl_up(x, d);
        if (lane >= (uint32_t)d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    T base = 0, tot = 0;
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
                                                        const gck_rec *__restrict__ recs, gck_rec *__restrict__ out,
                                                        uint32_t *__restrict__ out_idx) {
    __shared__ uint32_t wsum[kKdTile / 64];
    const uint64_t r = (uint64_t)blockIdx.x * kKdTile + threadIdx.x;
    const uint32_t v = r < n ? live[r] : 0u;
    uint32_t total;
    const uint32_t ex = block_excl(v, wsum, total);
    if (v) {
        out[tile_base[blockIdx.x] + ex] = recs[r];
        out_idx[tile_base[blockIdx.x] + ex] = (uint32_t)r;
    }
}

// ---- merge across shards (gck_kd_pack / gck_kd_merge) -----------------------

static_assert(sizeof(gck_kd_entry) == 64, "gck_kd_entry is 64 bytes");

__device__ __forceinline__ uint32_t kd_part(uint64_t h, uint32_t nparts) { return (uint32_t)(h >> 40) % nparts; }
__device__ __forceinline__ uint64_t pad8(uint64_t n) { return (n + 7) & ~7ull; }

// Entry sources of the partition / compaction kernels below.  sel: the entry
// takes part; put: write its gck_kd_entry and its zero-padded key.
struct LocalSrc {  // the keydir of the last run (gck_ctx_keydir)
    const uint8_t *arena;
    const uint64_t *rec_off, *khash;
    const gck_rec *recs;  // live entries, walk order
    const uint32_t *idx;  // their record indices
    uint32_t shard, file_base;
    __device__ bool sel(uint64_t) const { return true; }
    __device__ uint64_t hash(uint64_t i) const { return khash[idx[i]]; }
    __device__ uint32_t klen(uint64_t i) const { return recs[i].key_len; }
    // (the 64-byte entry as four 16-byte stores and the key as 8-byte ones:
    // field by field, a lane's stores each wrote a piece of its line)
    __device__ void put(uint64_t i, gck_kd_entry *e, uint64_t key_rel, uint32_t *kdst) const {
        const uint32_t r = idx[i];
        const uint2 *rp = reinterpret_cast<const uint2 *>(recs + i);  // gck_rec: 5 x 8 bytes
        const uint2 r0 = rp[0], r1 = rp[1], r2 = rp[2], r3 = rp[3], r4 = rp[4];
        const uint32_t len = r1.y;  // key_len
        const KeyWords k(arena, rec_off[r] + 16, len);
        uint2 *kd = reinterpret_cast<uint2 *>(kdst);
        for (uint32_t w = 0; 8ull * w < pad8(len); ++w)
            kd[w] = make_uint2(8 * w < len ? k[2 * w] : 0u, 8 * w + 4 < len ? k[2 * w + 1] : 0u);
        const uint64_t h = khash[r];
        uint4 *ep = reinterpret_cast<uint4 *>(e);
        ep[0] = make_uint4((uint32_t)h, (uint32_t)(h >> 32), (uint32_t)key_rel, (uint32_t)(key_rel >> 32));
        ep[1] = make_uint4(len, shard, r0.x, r0.y);          // key_len, shard, rec.rec_off
        ep[2] = make_uint4(r1.x + file_base, r1.y, r2.x, r2.y);  // rec.file, key_len, value_pos, value_size
        ep[3] = make_uint4(r3.x, r3.y, r4.x, r4.y);          // rec.crc, ts, flags, crc_calc
    }
};
static_assert(offsetof(gck_kd_entry, rec) == 24 && sizeof(gck_rec) == 40, "gck_kd_entry layout");

struct MergedSrc {  // received entries that won the merge
    const gck_kd_entry *E;
    const uint8_t *K;
    const uint64_t *koff;  // key offset of each entry in K
    const uint32_t *live;
    __device__ bool sel(uint64_t i) const { return live[i] != 0; }
    __device__ uint64_t hash(uint64_t i) const { return E[i].hash; }
    __device__ uint32_t klen(uint64_t i) const { return E[i].key_len; }
    __device__ void put(uint64_t i, gck_kd_entry *e, uint64_t key_rel, uint32_t *kdst) const {
        const uint4 *sp = reinterpret_cast<const uint4 *>(E + i);
        const uint4 a = sp[0], b = sp[1], c = sp[2], d = sp[3];
        const uint2 *src = reinterpret_cast<const uint2 *>(K + koff[i]);
        uint2 *kd = reinterpret_cast<uint2 *>(kdst);
        for (uint32_t w = 0; 8ull * w < pad8(b.x); ++w) kd[w] = src[w];  // b.x: key_len
        uint4 *ep = reinterpret_cast<uint4 *>(e);
        ep[0] = make_uint4(a.x, a.y, (uint32_t)key_rel, (uint32_t)(key_rel >> 32));
        ep[1] = b;
        ep[2] = c;
        ep[3] = d;
    }
};

// k_pk_tiles: per tile of kKdTile entries, the partition of each selected
// entry, its rank among the tile's entries of that partition (count and key
// bytes) and the tile's per-partition sums: tsum rows 0..nparts-1 count,
// rows nparts..2*nparts-1 key bytes, one column per tile.
template <class Src>
__global__ __launch_bounds__(kKdTile) void k_pk_tiles(Src src, uint64_t n, uint32_t nparts,
                                                      uint32_t *__restrict__ part, uint32_t *__restrict__ crank,
                                                      uint64_t *__restrict__ brank, uint64_t *__restrict__ tsum,
                                                      uint64_t nt) {
    __shared__ uint64_t wsum[kKdTile / 64];
    const uint64_t i = (uint64_t)blockIdx.x * kKdTile + threadIdx.x;
    const bool in = i < n && src.sel(i);
    uint32_t p = 0;
    uint64_t bytes = 0;
    if (in) {
        p = nparts > 1 ? kd_part(src.hash(i), nparts) : 0u;
        bytes = pad8(src.klen(i));
    }
    uint64_t cr = 0, br = 0;
    for (uint32_t q = 0; q < nparts; ++q) {
        const bool mine = in && p == q;
        uint64_t tc, tb;
        const uint64_t c = block_excl<uint64_t>(mine ? 1u : 0u, wsum, tc);
        const uint64_t b = block_excl<uint64_t>(mine ? bytes : 0u, wsum, tb);
        if (mine) {
            cr = c;
            br = b;
        }
        if (threadIdx.x == 0) {
            tsum[(uint64_t)q * nt + blockIdx.x] = tc;
            tsum[(uint64_t)(nparts + q) * nt + blockIdx.x] = tb;
        }
    }
    if (i < n) {
        part[i] = in ? p : kEmpty;
        crank[i] = (uint32_t)cr;
        brank[i] = br;
    }
}

// k_pk_scan: one workgroup per tsum row, exclusive in place; the row total
// goes to tot[row].
__global__ __launch_bounds__(kKdTile) void k_pk_scan(uint64_t *__restrict__ tsum, uint64_t nt,
                                                     uint64_t *__restrict__ tot) {
    __shared__ uint64_t wsum[kKdTile / 64];
    uint64_t *row = tsum + (uint64_t)blockIdx.x * nt;
    uint64_t run = 0;
    for (uint64_t i0 = 0; i0 < nt; i0 += kKdTile) {
        const uint64_t i = i0 + threadIdx.x;
        const uint64_t v = i < nt ? row[i] : 0u;
        uint64_t total;
        const uint64_t ex = block_excl<uint64_t>(v, wsum, total);
        if (i < nt) row[i] = run + ex;
        run += total;
    }
    if (threadIdx.x == 0) tot[blockIdx.x] = run;
}

// k_pk_scatter: each selected entry to its partition, partitions laid out
// one after another (entries and keys alike), tile order then rank within.
template <class Src>
__global__ __launch_bounds__(256) void k_pk_scatter(Src src, uint64_t n, uint32_t nparts,
                                                    const uint32_t *__restrict__ part,
                                                    const uint32_t *__restrict__ crank,
                                                    const uint64_t *__restrict__ brank,
                                                    const uint64_t *__restrict__ tsum, uint64_t nt,
                                                    const uint64_t *__restrict__ tot, gck_kd_entry *__restrict__ out,
                                                    uint8_t *__restrict__ keys) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t p = part[i];
        if (p == kEmpty) continue;
        const uint64_t t = i / kKdTile;
        uint64_t ebase = 0, kbase = 0;
        for (uint32_t q = 0; q < p; ++q) {
            ebase += tot[q];
            kbase += tot[nparts + q];
        }
        const uint64_t e = ebase + tsum[(uint64_t)p * nt + t] + crank[i];
        const uint64_t kr = tsum[(uint64_t)(nparts + p) * nt + t] + brank[i];
        src.put(i, out + e, kr, reinterpret_cast<uint32_t *>(keys + kbase + kr));
    }
}

// k_mg_koff: offset of each received entry's key in the concatenated blobs;
// pre = entry prefix over sources [nsrc+1], blob prefix [nsrc+1], error word.
__global__ __launch_bounds__(256) void k_mg_koff(const gck_kd_entry *__restrict__ E, uint64_t n,
                                                 uint64_t *__restrict__ pre, uint32_t nsrc,
                                                 uint64_t *__restrict__ koff) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t s = 0;
        while (s + 1 < nsrc && i >= pre[s + 1]) ++s;
        const uint64_t ko = E[i].key_off, blob = pre[nsrc + 2 + s] - pre[nsrc + 1 + s];
        if ((ko & 7) || ko + pad8(E[i].key_len) > blob) {  // not a packed entry: refuse the merge
            atomicOr(reinterpret_cast<unsigned long long *>(pre + 2 * (nsrc + 1)), 1ull);
            koff[i] = pre[nsrc + 1 + s];
        } else {
            koff[i] = pre[nsrc + 1 + s] + ko;
        }
    }
}

__device__ bool blob_same(const uint8_t *__restrict__ K, uint64_t a, uint64_t b, uint32_t len) {
    const uint32_t *x = reinterpret_cast<const uint32_t *>(K + a), *y = reinterpret_cast<const uint32_t *>(K + b);
    for (uint32_t w = 0; 4ull * w < len; ++w)  // padding bytes are zero on both sides
        if (x[w] != y[w]) return false;
    return true;
}

// k_mg_insert: as k_kd_insert over received entries; the entry index orders
// shards (sources are concatenated in shard order), so atomicMax keeps the
// highest shard's entry of every key.
__global__ __launch_bounds__(256) void k_mg_insert(const gck_kd_entry *__restrict__ E, const uint8_t *__restrict__ K,
                                                   const uint64_t *__restrict__ koff, uint64_t n,
                                                   uint32_t *__restrict__ table, uint64_t mask) {
    for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n; r += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t h = E[r].hash;
        const uint32_t len = E[r].key_len;
        // slot = entry index << 1 | 1 for a delete: the max still orders by
        // index, and k_mg_mark reads the winner's kind from the slot
        const uint32_t mine = ((uint32_t)r << 1) | ((E[r].rec.flags & GCK_F_TOMBSTONE) ? 1u : 0u);
        for (uint64_t s = h & mask;; s = (s + 1) & mask) {
            uint32_t cur = __hip_atomic_load(table + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cur == kEmpty) {
                const uint32_t prev = atomicCAS(table + s, kEmpty, mine);
                if (prev == kEmpty) break;
                cur = prev;
            }
            const uint32_t ci = cur >> 1;
            if (E[ci].hash == h && E[ci].key_len == len && blob_same(K, koff[ci], koff[r], len)) {
                atomicMax(table + s, mine);
                break;
            }
        }
    }
}

// k_mg_mark: a key's winning entry stays unless it is a delete.
__global__ __launch_bounds__(256) void k_mg_mark(const uint32_t *__restrict__ table, uint64_t slots,
                                                 uint32_t *__restrict__ live) {
    for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < slots; s += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t v = table[s];
        if (v != kEmpty && !(v & 1u)) live[v >> 1] = 1;
    }
}

}  // namespace gck

using namespace gck;

extern "C" {

int gck_ctx_keydir(gck_ctx *ctx, uint32_t flags, uint64_t *n_live, double *ms) {
    if (!ctx || !n_live) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    *n_live = 0;
    c->n_live = 0;
    c->kd_flags = flags;
    c->cmp_files = 0;
    c->kd_valid = false;
    const uint64_t n = c->n_recs;
    if (!n) {
        c->kd_valid = true;
        c->kd_slots = 0;
        return GCK_OK;
    }
    if (n >= kKdMaxRecs) return GCK_EINVAL;
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    // the run's finalize may have filled the table already (gck_ctx_keydir_hash):
    // then only the marking and the compaction are left, for every keydir of
    // that run (they do not change the table)
    bool filled = c->kd_inserted;
    uint64_t slots = filled ? c->kd_tab_slots : kd_table_slots(kd_keys_expected(c->kd_keys_hint, n));
    const uint64_t nt = (n + kKdTile - 1) / kKdTile;
    int rc;
    if ((rc = c->d_khash.ensure(n * 8)) || (rc = c->d_live.ensure(n * 4)) || (rc = c->d_kdstat.ensure(12)) ||
        (rc = c->d_ktile.ensure((nt + 1) * 4)) || (rc = c->d_kdout.ensure(n * sizeof(gck_rec))) ||
        (rc = c->d_kdidx.ensure(n * 4)))
        return rc;
    uint32_t *kstat = c->d_kdstat.as<uint32_t>();
    struct Ev {
        hipEvent_t a = nullptr, b = nullptr;
        ~Ev() {
            if (a) (void)hipEventDestroy(a);
            if (b) (void)hipEventDestroy(b);
        }
    } ev;
    GCK_HIP(hipEventCreate(&ev.a));
    GCK_HIP(hipEventCreate(&ev.b));
    GCK_HIP(hipEventRecord(ev.a, s));
    uint32_t live = 0, hst[3] = {0, 0, 0};
    constexpr int kLastAttempt = 2;  // sized for every record distinct, probes unbounded
    for (int attempt = 0;; ++attempt) {
        if ((rc = c->d_ktab.ensure(slots * 8 * kSlotWords))) return rc;
        if (filled) {
            GCK_HIP(hipMemsetAsync(kstat + 1, 0, 8, s));  // (word 0: the finalize's overflow)
        } else {
            GCK_HIP(hipMemsetAsync(c->d_ktab.p, 0xFF, slots * 8 * kSlotWords, s));
            GCK_HIP(hipMemsetAsync(kstat, 0, 12, s));
        }
        GCK_HIP(hipMemsetAsync(c->d_live.p, 0, n * 4, s));
        const uint32_t grid = (uint32_t)c->n_cu * 8;
        if (!filled)
            k_kd_insert<<<grid, 256, 0, s>>>(c->arena.as<uint8_t>(), c->d_rec_off.as<uint64_t>(),
                                             c->d_rec_kv.as<uint2>(), n, c->d_khash.as<uint64_t>(),
                                             c->d_ktab.as<unsigned long long>(), slots - 1, c->kd_hashed ? 1 : 0,
                                             kstat, attempt == kLastAttempt ? slots : (uint64_t)kMaxProbe);
        c->kd_hashed = true;
        k_kd_mark<<<grid, 256, 0, s>>>(c->d_ktab.as<unsigned long long>(), slots,
                                       (flags & GCK_KD_KEEP_TOMBSTONES) ? 1u : 0u, c->d_live.as<uint32_t>(), kstat);
        k_kd_tiles<<<(uint32_t)nt, kKdTile, 0, s>>>(c->d_live.as<uint32_t>(), n, c->d_ktile.as<uint32_t>());
        k_kd_tile_scan<<<1, kKdTile, 0, s>>>(c->d_ktile.as<uint32_t>(), (uint32_t)nt);
        k_kd_scatter<<<(uint32_t)nt, kKdTile, 0, s>>>(c->d_live.as<uint32_t>(), n, c->d_ktile.as<uint32_t>(),
                                                      c->d_out.as<gck_rec>(), c->d_kdout.as<gck_rec>(),
                                                      c->d_kdidx.as<uint32_t>());
        GCK_HIP(hipEventRecord(ev.b, s));
        GCK_HIP(hipMemcpyAsync(&live, c->d_ktile.as<uint32_t>() + nt, 4, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipMemcpyAsync(hst, kstat, 12, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipStreamSynchronize(s));
        GCK_HIP(hipGetLastError());
        if (!hst[0]) break;
        // a key found no slot within kMaxProbe probes (more keys than the
        // table was sized for, or hashes that cluster): again, sized for every
        // record distinct, the last time without a probe bound (that build
        // cannot overflow: its load is <= 0.8)
        if (attempt == kLastAttempt) return GCK_EDEVICE;
        filled = false;
        const uint64_t all = kd_table_slots(n);
        slots = attempt + 1 == kLastAttempt ? std::max(all, slots) : (slots < all ? all : 2 * slots);
    }
    c->kd_probe_bound = std::max<uint64_t>(kMaxProbe, hst[2]);
    float t = 0;
    (void)hipEventElapsedTime(&t, ev.a, ev.b);
    if (ms) *ms = t;
    c->kd_inserted = true;  // the table holds this run's records: a rebuild only marks and compacts
    c->kd_tab_slots = slots;
    c->kd_keys_hint = hst[1];
    c->n_live = live;
    c->kd_valid = true;
    c->kd_slots = slots;
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

int gck_kd_pack_sizes(gck_ctx *ctx, uint32_t nparts, uint64_t *counts, uint64_t *key_bytes) {
    if (!ctx || !counts || !key_bytes || nparts == 0 || nparts > 64) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    c->kd_nparts = 0;
    const uint64_t n = c->n_live;
    const uint64_t nt = n ? (n + kKdTile - 1) / kKdTile : 1;
    int rc;
    if ((rc = c->d_kpart.ensure(n * 4)) || (rc = c->d_kcrank.ensure(n * 4)) || (rc = c->d_kbrank.ensure(n * 8)) ||
        (rc = c->d_kpsum.ensure(2 * nparts * nt * 8)) || (rc = c->d_kptot.ensure(2 * 64 * 8)))
        return rc;
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    uint64_t tot[128] = {};
    if (n) {
        const LocalSrc src{c->arena.as<uint8_t>(), c->d_rec_off.as<uint64_t>(), c->d_khash.as<uint64_t>(),
                           c->d_kdout.as<gck_rec>(), c->d_kdidx.as<uint32_t>(), 0u, 0u};
        k_pk_tiles<LocalSrc><<<(uint32_t)nt, kKdTile, 0, s>>>(src, n, nparts, c->d_kpart.as<uint32_t>(),
                                                              c->d_kcrank.as<uint32_t>(), c->d_kbrank.as<uint64_t>(),
                                                              c->d_kpsum.as<uint64_t>(), nt);
        k_pk_scan<<<2 * nparts, kKdTile, 0, s>>>(c->d_kpsum.as<uint64_t>(), nt, c->d_kptot.as<uint64_t>());
        GCK_HIP(hipMemcpyAsync(tot, c->d_kptot.p, 2 * nparts * 8, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipStreamSynchronize(s));
        GCK_HIP(hipGetLastError());
    }
    for (uint32_t p = 0; p < nparts; ++p) {
        counts[p] = tot[p];
        key_bytes[p] = tot[nparts + p];
        c->kd_tot[p] = tot[p];
        c->kd_tot[nparts + p] = tot[nparts + p];
    }
    c->kd_nparts = nparts;
    c->kd_packed = n;
    return GCK_OK;
}

int gck_kd_pack(gck_ctx *ctx, uint32_t shard, uint32_t file_base, gck_kd_entry *d_entries, uint64_t entries_cap,
                uint8_t *d_keys, uint64_t keys_cap) {
    if (!ctx) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    const uint32_t np = c->kd_nparts;
    if (!np || c->kd_packed != c->n_live) return GCK_EINVAL;  // gck_kd_pack_sizes first
    uint64_t ne = 0, nk = 0;
    for (uint32_t p = 0; p < np; ++p) {
        ne += c->kd_tot[p];
        nk += c->kd_tot[np + p];
    }
    if (ne > entries_cap || nk > keys_cap || (ne && (!d_entries || !d_keys))) return GCK_EINVAL;
    if (!ne) return GCK_OK;
    const uint64_t n = c->n_live, nt = (n + kKdTile - 1) / kKdTile;
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    const LocalSrc src{c->arena.as<uint8_t>(), c->d_rec_off.as<uint64_t>(), c->d_khash.as<uint64_t>(),
                       c->d_kdout.as<gck_rec>(), c->d_kdidx.as<uint32_t>(), shard, file_base};
    k_pk_scatter<LocalSrc><<<(uint32_t)c->n_cu * 4, 256, 0, s>>>(
        src, n, np, c->d_kpart.as<uint32_t>(), c->d_kcrank.as<uint32_t>(), c->d_kbrank.as<uint64_t>(),
        c->d_kpsum.as<uint64_t>(), nt, c->d_kptot.as<uint64_t>(), d_entries, d_keys);
    GCK_HIP(hipStreamSynchronize(s));
    GCK_HIP(hipGetLastError());
    return GCK_OK;
}

int gck_kd_merge(gck_ctx *ctx, const gck_kd_entry *d_entries, const uint8_t *d_keys, const uint64_t *src_counts,
                 const uint64_t *src_key_bytes, uint32_t nsrc, uint64_t *n_live, double *ms) {
    if (!ctx || !n_live || !src_counts || !src_key_bytes || nsrc == 0 || nsrc > 65536) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    *n_live = 0;
    c->n_merged = 0;
    c->merged_key_bytes = 0;
    c->kd_nparts = 0;  // the pack state shares buffers with the merge
    std::vector<uint64_t> pre(2 * (nsrc + 1) + 1, 0);
    for (uint32_t i = 0; i < nsrc; ++i) {
        pre[i + 1] = pre[i] + src_counts[i];
        pre[nsrc + 2 + i] = pre[nsrc + 1 + i] + src_key_bytes[i];
    }
    const uint64_t n = pre[nsrc];
    if (ms) *ms = 0;
    if (!n) return GCK_OK;
    if (n >= 0x7FFFFFFFull || !d_entries || !d_keys) return GCK_EINVAL;  // (slots: index << 1 | delete)
    uint64_t slots = 1024;
    while (slots < 2 * n) slots <<= 1;
    const uint64_t nt = (n + kKdTile - 1) / kKdTile;
    int rc;
    if ((rc = c->d_msrc.ensure(pre.size() * 8)) || (rc = c->d_mkoff.ensure(n * 8)) ||
        (rc = c->d_mtab.ensure(slots * 4)) || (rc = c->d_mlive.ensure(n * 4)) || (rc = c->d_kpart.ensure(n * 4)) ||
        (rc = c->d_kcrank.ensure(n * 4)) || (rc = c->d_kbrank.ensure(n * 8)) || (rc = c->d_kpsum.ensure(2 * nt * 8)) ||
        (rc = c->d_kptot.ensure(2 * 64 * 8)))
        return rc;
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    hipEvent_t a, b;
    GCK_HIP(hipEventCreate(&a));
    GCK_HIP(hipEventCreate(&b));
    GCK_HIP(hipEventRecord(a, s));
    GCK_HIP(hipMemcpyAsync(c->d_msrc.p, pre.data(), pre.size() * 8, hipMemcpyHostToDevice, s));
    GCK_HIP(hipMemsetAsync(c->d_mtab.p, 0xFF, slots * 4, s));
    GCK_HIP(hipMemsetAsync(c->d_mlive.p, 0, n * 4, s));
    const uint32_t grid = (uint32_t)c->n_cu * 8;
    k_mg_koff<<<grid, 256, 0, s>>>(d_entries, n, c->d_msrc.as<uint64_t>(), nsrc, c->d_mkoff.as<uint64_t>());
    k_mg_insert<<<grid, 256, 0, s>>>(d_entries, d_keys, c->d_mkoff.as<uint64_t>(), n, c->d_mtab.as<uint32_t>(),
                                     slots - 1);
    k_mg_mark<<<grid, 256, 0, s>>>(c->d_mtab.as<uint32_t>(), slots, c->d_mlive.as<uint32_t>());
    const MergedSrc src{d_entries, d_keys, c->d_mkoff.as<uint64_t>(), c->d_mlive.as<uint32_t>()};
    k_pk_tiles<MergedSrc><<<(uint32_t)nt, kKdTile, 0, s>>>(src, n, 1u, c->d_kpart.as<uint32_t>(),
                                                           c->d_kcrank.as<uint32_t>(), c->d_kbrank.as<uint64_t>(),
                                                           c->d_kpsum.as<uint64_t>(), nt);
    k_pk_scan<<<2, kKdTile, 0, s>>>(c->d_kpsum.as<uint64_t>(), nt, c->d_kptot.as<uint64_t>());
    uint64_t tot[2] = {}, err = 0;
    GCK_HIP(hipMemcpyAsync(tot, c->d_kptot.p, 16, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipMemcpyAsync(&err, c->d_msrc.as<uint64_t>() + 2 * (nsrc + 1), 8, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    GCK_HIP(hipGetLastError());
    if (err) {
        (void)hipEventDestroy(a);
        (void)hipEventDestroy(b);
        return GCK_EINVAL;
    }
    if ((rc = c->d_mhdr.ensure(tot[0] * sizeof(gck_kd_entry))) || (rc = c->d_mkeys.ensure(tot[1]))) return rc;
    k_pk_scatter<MergedSrc><<<grid, 256, 0, s>>>(src, n, 1u, c->d_kpart.as<uint32_t>(), c->d_kcrank.as<uint32_t>(),
                                                 c->d_kbrank.as<uint64_t>(), c->d_kpsum.as<uint64_t>(), nt,
                                                 c->d_kptot.as<uint64_t>(), c->d_mhdr.as<gck_kd_entry>(),
                                                 c->d_mkeys.as<uint8_t>());
    GCK_HIP(hipEventRecord(b, s));
    GCK_HIP(hipStreamSynchronize(s));
    GCK_HIP(hipGetLastError());
    float t = 0;
    (void)hipEventElapsedTime(&t, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (ms) *ms = t;
    c->n_merged = tot[0];
    c->merged_key_bytes = tot[1];
    *n_live = tot[0];
    return GCK_OK;
}

int gck_kd_fetch_merged(gck_ctx *ctx, gck_kd_entry *dst, uint64_t cap, uint8_t *keys, uint64_t keys_cap,
                        uint64_t *n, uint64_t *n_key_bytes) {
    if (!ctx || !n || !n_key_bytes) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    *n = c->n_merged;
    *n_key_bytes = c->merged_key_bytes;
    if (!dst && !keys) return GCK_OK;  // size query
    if (c->n_merged > cap || c->merged_key_bytes > keys_cap || (c->n_merged && (!dst || !keys))) return GCK_EINVAL;
    if (c->n_merged) {
        GCK_HIP(hipSetDevice(c->device));
        GCK_HIP(hipMemcpy(dst, c->d_mhdr.p, c->n_merged * sizeof(gck_kd_entry), hipMemcpyDeviceToHost));
        GCK_HIP(hipMemcpy(keys, c->d_mkeys.p, c->merged_key_bytes, hipMemcpyDeviceToHost));
    }
    return GCK_OK;
}

}  // extern "C"
