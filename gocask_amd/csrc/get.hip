// get.hip — batched DB.Get and keydir scrub on the device.
//
// DB.Get (core/db.go:287-316): an empty key is ErrInvalidKey; a key missing from
// the keydir is ErrKeyNotFound; otherwise ValueSize bytes are read from the
// entry's File at ValuePos (a short read is an error of the file system) and
// crc32.ChecksumIEEE of them must equal the entry's CRC (ErrCRCFailed).  Here
// the keydir is the device table of gck_ctx_keydir and the files are the
// resident arena, so a batch of Gets is one lookup kernel and one verify
// kernel; gck_ctx_scrub_keydir runs the verify over every live entry.
#include "kd_common.h"
#include "gck_crc_lds.h"

namespace gck {

// LDS tables: the conflict-free slicing-by-4 image (gck_crc_lds.h, 128 KiB,
// from the context's global tables) and multiplication by the constant Z_1008
// as four byte tables: Z(A) = XOR_k Zs[k][byte k of A] (Z is linear in A).
struct CrcTabs {
    uint32_t S[kSliceLdsWords];
    uint32_t Zs[4][256];
};

__device__ void crc_tables(CrcTabs &t, const uint32_t *__restrict__ g_slice) {
    fill_slice_lds(t.S, g_slice);
    const uint32_t z = xpow8n(1008);
    for (uint32_t e = threadIdx.x; e < 1024; e += blockDim.x) t.Zs[e >> 8][e & 0xFF] = multmodp(z, (e & 0xFF) << (8 * (e >> 8)));
    __syncthreads();
}

// a * b mod P (reflected), 32 steps without early exit (a varies by lane).
__device__ __forceinline__ uint32_t gmul(uint32_t a, uint32_t b) {
    uint32_t p = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
        p ^= (a & (0x80000000u >> i)) ? b : 0u;
        b = (b >> 1) ^ ((b & 1u) ? kPoly : 0u);
    }
    return p;
}

__device__ __forceinline__ uint32_t zmul(const uint32_t (*Z)[256], uint32_t a) {
    return Z[0][a & 0xFF] ^ Z[1][(a >> 8) & 0xFF] ^ Z[2][(a >> 16) & 0xFF] ^ Z[3][a >> 24];
}

// The 16 bytes of virtual position v (value p[0, L) zero-padded in front by
// pad bytes), plus the next dword for the byte shift: one 16 B and one 4 B
// load (dword aligned), unconditional.  A lane wholly in the padding loads
// the value's first dwords instead (never before the arena; wave_crc masks its
// bytes); a lane straddling the value start reads up to 15 bytes before it
// (the record's header and key: inside the arena).
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
// (Pointer arithmetic only, never an integer cast back to a pointer: that
// would make the loads flat, and flat loads also count on lgkmcnt, so every
// LDS table wait would wait for HBM too.)
__device__ __forceinline__ void stripe_load(const uint8_t *p, uint64_t v, uint64_t pad, uint32_t d[5]) {
    const uint8_t *q = p + v - pad;
    q = v + 16 <= pad ? p : q;
    const uint8_t *a = q - (reinterpret_cast<uintptr_t>(q) & 3);
    const u32x4_a4 x = *reinterpret_cast<const u32x4_a4 *>(a);
    d[0] = x.x;
    d[1] = x.y;
    d[2] = x.z;
    d[3] = x.w;
    d[4] = *reinterpret_cast<const uint32_t *>(a + 16);
}

// Start of a value's CRC: J = ceil(L / 1 KiB) stripes, pad = J KiB - L.
struct CrcJob {
    const uint8_t *p;
    uint64_t L, J, pad;
    __device__ CrcJob(const uint8_t *p_, uint64_t L_) : p(p_), L(L_), J((L_ + 1023) >> 10), pad((J << 10) - L_) {}
};

// crc32.ChecksumIEEE of a value by one wavefront.  The value is read as a
// virtual buffer of J stripes of 1 KiB, zero-padded at the FRONT (F(0, .)
// ignores leading zeros), lane l taking the 16 bytes at 16 l of every stripe
// (coalesced loads).  Lane state: A <- F(Z_1008(A), chunk), i.e. Horner over
// the lane's chunks 1 KiB apart.  The 0xFFFFFFFF init is the complement of the
// value's first 4 bytes (F(~0, V) = F(0, V with bytes 0..3 ^ 0xFF)).  Lane l's
// part is finally shifted past the 16 (63-l) bytes after it (kl = x^(8 * 16
// (63-l))) and the lanes XOR-reduced: F(~0, V); crc = ~that.
//
// One stripe of the value at virtual stripe j into A:
__device__ __forceinline__ uint32_t fold_stripe(const CrcJob &jb, uint64_t j, const uint32_t d[5], uint32_t A,
                                                const CrcTabs &t, uint32_t lb0, uint32_t lb1) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t v = (j << 10) + 16ull * lane;  // virtual position of this lane's chunk
    const uint32_t sh = (uint32_t)((reinterpret_cast<uintptr_t>(jb.p) + v - jb.pad) & 3);
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
    if (v < jb.pad + 4) {  // chunks at the value's start: bytes before it are zero, its first 4 complemented
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int64_t lead = (int64_t)jb.pad - (int64_t)(v + 4 * i);  // bytes of dword i before the value
            const uint32_t keep = lead >= 4 ? 0u : lead <= 0 ? 0xFFFFFFFFu : 0xFFFFFFFFu << (8 * lead);
            const int64_t cl = lead + 4;  // bytes of dword i before the value's byte 4
            const uint32_t flip = cl <= 0 ? 0u : cl >= 4 ? 0xFFFFFFFFu : 0xFFFFFFFFu >> (8 * (4 - cl));
            w[i] = (w[i] & keep) ^ (flip & keep);
        }
    }
    uint32_t c = zmul(t.Zs, A) ^ w[0];
    c = slice4x(t.S, lb0, lb1, c, w[1]);
    c = slice4x(t.S, lb0, lb1, c, w[2]);
    c = slice4x(t.S, lb0, lb1, c, w[3]);
    return slice4x(t.S, lb0, lb1, c, 0u);
}

// The large values of a wavefront's 64 items (mask todo), one after another,
// with kRing stripes in flight across value boundaries: the stripe folded now
// was loaded kRing stripes earlier (16 KiB per CU in flight with one stripe
// ahead is far below what HBM latency needs).  All control is wave-uniform;
// every load is issued unconditionally (a dummy reload past the last stripe),
// so the compiler's vmcnt counts stay exact.  Item t's CRC lands in lane t.
#ifndef GCK_RING
#define GCK_RING 4
#endif
constexpr int kRing = GCK_RING;
__device__ uint32_t wave_crcs(uint64_t todo, const uint8_t *arena, uint64_t off, uint32_t len, uint32_t kl,
                              const CrcTabs &t, uint32_t lb0, uint32_t lb1) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t out = 0;
    auto job = [&](int it) { return CrcJob(arena + __shfl(off, it), __shfl(len, it)); };
    // load cursor
    uint64_t lrem = todo;
    int lt = __builtin_ctzll(todo);
    CrcJob lj = job(lt);
    uint64_t ls = 0;
    auto load_next = [&](uint32_t d[5]) {
        stripe_load(lj.p, (ls << 10) + 16ull * lane, lj.pad, d);
        if (lrem && ++ls == lj.J) {  // the next value (or stay on the last stripe: dummy reloads)
            lrem &= lrem - 1;
            if (lrem) {
                lt = __builtin_ctzll(lrem);
                lj = job(lt);
                ls = 0;
            } else {
                ls = lj.J - 1;
            }
        }
    };
    uint32_t ring[kRing][5];
#pragma unroll
    for (int k = 0; k < kRing; ++k) load_next(ring[k]);
    // compute cursor
    uint64_t crem = todo;
    int ct = __builtin_ctzll(todo);
    CrcJob cj = job(ct);
    uint64_t cs = 0;
    uint32_t A = 0;
    while (crem) {
#pragma unroll
        for (int k = 0; k < kRing; ++k) {
            if (crem) {
                A = fold_stripe(cj, cs, ring[k], A, t, lb0, lb1);
                load_next(ring[k]);
                if (++cs == cj.J) {  // value done
                    uint32_t f = gmul(kl, A);
#pragma unroll
                    for (int m = 32; m >= 1; m >>= 1) f ^= __shfl_xor(f, m);
                    if (lane == (uint32_t)ct) out = ~f;
                    A = 0;
                    cs = 0;
                    crem &= crem - 1;
                    if (crem) {
                        ct = __builtin_ctzll(crem);
                        cj = job(ct);
                    }
                }
            }
        }
    }
    return out;
}

constexpr uint32_t kLaneMax = 256;  // values up to this size: one lane each

// crc32.ChecksumIEEE of a small value by one lane (lanes run different
// values): aligned dwords, 64 bytes of loads in flight per round, slicing-by-4
// per word, the last 0..3 bytes one at a time.
__device__ uint32_t lane_crc(const uint8_t *p, uint32_t L, bool act, const CrcTabs &t, uint32_t lb0, uint32_t lb1) {
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
    const uint32_t *a = reinterpret_cast<const uint32_t *>(p - sh);
    const uint32_t nw = act ? (sh + L + 3) >> 2 : 0u;  // dwords covering the value
    uint32_t c = 0xFFFFFFFFu, pos = 0;
    for (uint32_t b = 0; __ballot(b < nw); b += 16) {
        uint32_t d[17];
#pragma unroll
        for (int i = 0; i < 17; ++i) d[i] = b + i < nw ? a[b + i] : 0u;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const uint32_t w = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
            if (pos + 4 <= L) {
                c = slice4x(t.S, lb0, lb1, c ^ w, 0u);
            } else {
                for (uint32_t k = 0; pos + k < L; ++k) c = byte1x(t.S, lb1, c, w >> (8 * k));
            }
            pos = pos + 4 <= L ? pos + 4 : L;
        }
    }
    return ~c;
}

// k_get_lookup: one lane per query key (keys: a blob padded by 8 bytes, koff:
// n+1 offsets).  Probes the keydir table like k_kd_insert; a key whose winning
// record is a tombstone is not in the keydir.  Found keys become verify items:
// the arena offset of ValueSize bytes at ValuePos of the entry's file.
__global__ __launch_bounds__(256) void k_get_lookup(const uint8_t *__restrict__ keys,
                                                    const uint64_t *__restrict__ koff, uint32_t n,
                                                    const unsigned long long *__restrict__ table, uint64_t slots,
                                                    const uint8_t *__restrict__ arena,
                                                    const uint64_t *__restrict__ rec_off,
                                                    const uint2 *__restrict__ rec_kv,
                                                    const gck_rec *__restrict__ recs,
                                                    const uint64_t *__restrict__ fbase,
                                                    const uint64_t *__restrict__ flen, int32_t *__restrict__ status,
                                                    uint64_t *__restrict__ item, uint32_t *__restrict__ vsize,
                                                    uint32_t *__restrict__ expect) {
    for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < n; q += gridDim.x * blockDim.x) {
        const uint64_t len64 = koff[q + 1] - koff[q];
        vsize[q] = 0;
        if (len64 == 0) {
            status[q] = GCK_EINVALID_KEY;  // core/db.go:295-297
            continue;
        }
        int32_t st = GCK_EKEY_NOT_FOUND;
        if (slots && len64 < 0xFFFFFFFFull) {
            const uint32_t len = (uint32_t)len64;
            const KeyWords k(keys, koff[q], len);
            const uint64_t h = key_hash(k, len), mask = slots - 1;
            const uint32_t tag = slot_tag(h);
            for (uint64_t s = h & mask;; s = (s + 1) & mask) {
                const unsigned long long v = table[s];
                if (v == kEmptySlot) break;
                const uint32_t cur = (uint32_t)v;
                if ((uint32_t)(v >> 32) != tag || key_len(rec_kv[cur]) != len) continue;
                const KeyWords a(arena, rec_off[cur] + 16, len);
                bool same = true;
                for (uint32_t i = 0; same && 4 * i < len; ++i) same = a[i] == k[i];
                if (!same) continue;
                const gck_rec r = recs[cur];
                if (!(r.flags & GCK_F_TOMBSTONE)) {
                    // os.File.ReadAt into an empty buffer returns (0, nil) at any
                    // offset, so an empty value is never a short read
                    if (r.value_size && (uint64_t)r.value_pos + r.value_size > flen[r.file]) {
                        st = GCK_EIO;  // Disk.ReadFileAt short read
                    } else {
                        st = GCK_OK;   // pending the CRC
                        item[q] = fbase[r.file] + r.value_pos;
                        vsize[q] = r.value_size;
                        expect[q] = r.crc;
                    }
                }
                break;
            }
        }
        status[q] = st;
    }
}

// k_scrub_items: the live keydir entries as verify items (Get of every key).
__global__ __launch_bounds__(256) void k_scrub_items(const gck_rec *__restrict__ live, uint64_t n,
                                                     const uint64_t *__restrict__ fbase,
                                                     const uint64_t *__restrict__ flen, int32_t *__restrict__ status,
                                                     uint64_t *__restrict__ item, uint32_t *__restrict__ vsize,
                                                     uint32_t *__restrict__ expect) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const gck_rec r = live[i];
        const bool ok = !r.value_size || (uint64_t)r.value_pos + r.value_size <= flen[r.file];  // see k_get_lookup
        status[i] = ok ? GCK_OK : GCK_EIO;
        item[i] = ok ? fbase[r.file] + r.value_pos : 0;
        vsize[i] = ok ? r.value_size : 0;
        expect[i] = r.crc;
    }
}

// k_verify: a wavefront takes 64 items (one per lane: status, location, size,
// expected CRC in one coalesced load each), then the CRC of every item still
// GCK_OK in turn, all lanes on one value; a mismatch is GCK_ECRC_FAILED, a
// match copies the value to dst + dst_off (if dst).
__global__ __launch_bounds__(1024) void k_verify(const uint8_t *__restrict__ arena, const uint32_t *__restrict__ g_slice,
                                                 uint64_t n,
                                                const uint64_t *__restrict__ item,
                                                const uint32_t *__restrict__ vsize,
                                                const uint32_t *__restrict__ expect, int32_t *__restrict__ status,
                                                uint32_t *__restrict__ crc_out, const uint64_t *__restrict__ dst_off,
                                                uint8_t *__restrict__ dst) {
    __shared__ CrcTabs T;
    crc_tables(T, g_slice);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t lb0, lb1;
    slice_bases(lane, lb0, lb1);
    const uint32_t kl = xpow8n(16ull * (63 - lane));  // lane l's chunk is followed by 16 (63-l) bytes of its stripe
    const uint64_t groups = (n + 63) >> 6, waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t gi = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); gi < groups; gi += waves) {
        const uint64_t mine = (gi << 6) + lane;
        const bool have = mine < n;
        const bool ok = have && status[mine] == GCK_OK;
        const uint64_t off = ok ? item[mine] : 0;
        const uint32_t len = ok ? vsize[mine] : 0u, want = ok ? expect[mine] : 0u;
        const uint64_t doff = ok && dst ? dst_off[mine] : 0;
        uint32_t crc = 0;
        const bool small = ok && len <= kLaneMax;
        const uint64_t todo = __ballot(ok && !small);
        if (__ballot(small)) {  // small values: a lane each, all at once
            const uint32_t c = lane_crc(arena + off, len, small, T, lb0, lb1);
            if (small) crc = c;
        }
        if (todo) {
            const uint32_t c = wave_crcs(todo, arena, off, len, kl, T, lb0, lb1);
            if ((todo >> lane) & 1) crc = c;
        }
        if (dst) {  // the values that passed, copied by the whole wave
            for (uint64_t cp = __ballot(ok && crc == want); cp; cp &= cp - 1) {
                const int t = __builtin_ctzll(cp);
                uint8_t *d = dst + __shfl(doff, t);
                const uint8_t *src = arena + __shfl(off, t);
                const uint32_t L = __shfl(len, t);
                for (uint64_t j = lane; j < L; j += 64) d[j] = src[j];
            }
        }
        if (have) {
            crc_out[mine] = crc;
            if (ok && crc != want) status[mine] = GCK_ECRC_FAILED;  // core/db.go:311-313
        }
    }
}

}  // namespace gck

using namespace gck;

extern "C" {

int gck_ctx_get_batch(gck_ctx *ctx, const uint8_t *keys, const uint64_t *key_off, uint32_t n, int32_t *status,
                      uint32_t *value_size, uint32_t *crc_calc, uint8_t *values, uint64_t values_cap,
                      uint64_t *val_off, double *ms) {
    if (!ctx || !key_off || !status || !value_size || !crc_calc || (values && !val_off)) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    if (!c->kd_valid) return GCK_EINVAL;  // gck_ctx_keydir after the run first
    if (ms) *ms = 0;
    if (!n) return GCK_OK;
    for (uint32_t i = 0; i < n; ++i)
        if (key_off[i + 1] < key_off[i]) return GCK_EINVAL;
    const uint64_t kb = key_off[n];
    if (kb && !keys) return GCK_EINVAL;
    int rc;
    if ((rc = c->d_gkeys.ensure(kb + 16)) || (rc = c->d_gkoff.ensure((n + 1) * 8ull)) ||
        (rc = c->d_gstat.ensure(n * 4ull)) || (rc = c->d_gitem.ensure(n * 8ull)) ||
        (rc = c->d_gvsize.ensure(n * 4ull)) || (rc = c->d_gexp.ensure(n * 4ull)) ||
        (rc = c->d_gcrc.ensure(n * 4ull)) || (rc = c->d_gvoff.ensure(n * 8ull)))
        return rc;
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    hipEvent_t a, b;
    GCK_HIP(hipEventCreate(&a));
    GCK_HIP(hipEventCreate(&b));
    GCK_HIP(hipEventRecord(a, s));
    GCK_HIP(hipMemsetAsync(c->d_gkeys.p, 0, kb + 16, s));
    if (kb) GCK_HIP(hipMemcpyAsync(c->d_gkeys.p, keys, kb, hipMemcpyHostToDevice, s));
    GCK_HIP(hipMemcpyAsync(c->d_gkoff.p, key_off, (n + 1) * 8ull, hipMemcpyHostToDevice, s));
    k_get_lookup<<<(n + 255) / 256, 256, 0, s>>>(
        c->d_gkeys.as<uint8_t>(), c->d_gkoff.as<uint64_t>(), n, c->d_ktab.as<unsigned long long>(), c->kd_slots,
        c->arena.as<uint8_t>(), c->d_rec_off.as<uint64_t>(), c->d_rec_kv.as<uint2>(),
        c->d_out.as<gck_rec>(), c->d_fbase.as<uint64_t>(), c->d_flen.as<uint64_t>(), c->d_gstat.as<int32_t>(),
        c->d_gitem.as<uint64_t>(), c->d_gvsize.as<uint32_t>(), c->d_gexp.as<uint32_t>());
    uint8_t *dvals = nullptr;
    if (values) {  // value offsets of the found keys, back to back
        GCK_HIP(hipMemcpyAsync(status, c->d_gstat.p, n * 4ull, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipMemcpyAsync(value_size, c->d_gvsize.p, n * 4ull, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipStreamSynchronize(s));
        uint64_t tot = 0;
        for (uint32_t i = 0; i < n; ++i) {
            val_off[i] = status[i] == GCK_OK ? tot : ~0ull;
            if (status[i] == GCK_OK) tot += value_size[i];
        }
        if (tot > values_cap) {
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
            return GCK_EINVAL;
        }
        if ((rc = c->d_gvals.ensure(tot))) return rc;
        GCK_HIP(hipMemcpyAsync(c->d_gvoff.p, val_off, n * 8ull, hipMemcpyHostToDevice, s));
        dvals = c->d_gvals.as<uint8_t>();
    }
    // one 1024-thread workgroup per CU (the tables take 132 KiB of LDS)
    const uint32_t grid = std::min<uint32_t>((n + 1023) / 1024, (uint32_t)c->n_cu);
    k_verify<<<grid, 1024, 0, s>>>(c->arena.as<uint8_t>(), c->d_slice.as<uint32_t>(), n, c->d_gitem.as<uint64_t>(), c->d_gvsize.as<uint32_t>(),
                                  c->d_gexp.as<uint32_t>(), c->d_gstat.as<int32_t>(), c->d_gcrc.as<uint32_t>(),
                                  c->d_gvoff.as<uint64_t>(), dvals);
    GCK_HIP(hipEventRecord(b, s));
    GCK_HIP(hipMemcpyAsync(status, c->d_gstat.p, n * 4ull, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipMemcpyAsync(value_size, c->d_gvsize.p, n * 4ull, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipMemcpyAsync(crc_calc, c->d_gcrc.p, n * 4ull, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    if (values) {
        uint64_t tot = 0;
        for (uint32_t i = 0; i < n; ++i)
            if (val_off[i] != ~0ull) {
                if (status[i] != GCK_OK) val_off[i] = ~0ull;  // CRC failed: no value
                tot = std::max(tot, (val_off[i] == ~0ull ? 0 : val_off[i] + value_size[i]));
            }
        if (tot) GCK_HIP(hipMemcpy(values, dvals, tot, hipMemcpyDeviceToHost));
    }
    GCK_HIP(hipGetLastError());
    float t = 0;
    (void)hipEventElapsedTime(&t, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (ms) *ms = t;
    return GCK_OK;
}

int gck_ctx_scrub_keydir(gck_ctx *ctx, int32_t *status, uint32_t *crc_calc, uint64_t *n_bad, double *ms) {
    if (!ctx || !n_bad) return GCK_EINVAL;
    Ctx *c = &ctx->c;
    if (!c->kd_valid) return GCK_EINVAL;
    *n_bad = 0;
    if (ms) *ms = 0;
    const uint64_t n = c->n_live;
    if (!n) return GCK_OK;
    int rc;
    if ((rc = c->d_gstat.ensure(n * 4)) || (rc = c->d_gitem.ensure(n * 8)) || (rc = c->d_gvsize.ensure(n * 4)) ||
        (rc = c->d_gexp.ensure(n * 4)) || (rc = c->d_gcrc.ensure(n * 4)))
        return rc;
    GCK_HIP(hipSetDevice(c->device));
    hipStream_t s = c->stream;
    hipEvent_t a, b;
    GCK_HIP(hipEventCreate(&a));
    GCK_HIP(hipEventCreate(&b));
    GCK_HIP(hipEventRecord(a, s));
    k_scrub_items<<<(uint32_t)c->n_cu * 8, 256, 0, s>>>(c->d_kdout.as<gck_rec>(), n, c->d_fbase.as<uint64_t>(),
                                                       c->d_flen.as<uint64_t>(), c->d_gstat.as<int32_t>(),
                                                       c->d_gitem.as<uint64_t>(), c->d_gvsize.as<uint32_t>(),
                                                       c->d_gexp.as<uint32_t>());
    k_verify<<<(uint32_t)c->n_cu, 1024, 0, s>>>(c->arena.as<uint8_t>(), c->d_slice.as<uint32_t>(), n, c->d_gitem.as<uint64_t>(),
                                                    c->d_gvsize.as<uint32_t>(), c->d_gexp.as<uint32_t>(),
                                                    c->d_gstat.as<int32_t>(), c->d_gcrc.as<uint32_t>(), nullptr,
                                                    nullptr);
    GCK_HIP(hipEventRecord(b, s));
    std::vector<int32_t> st(status ? 0 : n);
    int32_t *sp = status ? status : st.data();
    GCK_HIP(hipMemcpyAsync(sp, c->d_gstat.p, n * 4, hipMemcpyDeviceToHost, s));
    if (crc_calc) GCK_HIP(hipMemcpyAsync(crc_calc, c->d_gcrc.p, n * 4, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipStreamSynchronize(s));
    GCK_HIP(hipGetLastError());
    uint64_t bad = 0;
    for (uint64_t i = 0; i < n; ++i) bad += sp[i] != GCK_OK;
    *n_bad = bad;
    float t = 0;
    (void)hipEventElapsedTime(&t, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    if (ms) *ms = t;
    return GCK_OK;
}

}  // extern "C"
