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
#include "gck_crc_wave.h"

namespace gck {

// k_get_lookup: one lane per query key (keys: a blob padded by 8 bytes, koff:
// n+1 offsets).  Probes the keydir table like k_kd_insert; a key whose winning
// record is a tombstone is not in the keydir.  Found keys become verify items:
// the arena offset of ValueSize bytes at ValuePos of the entry's file.
__global__ __launch_bounds__(256) void k_get_lookup(const uint8_t *__restrict__ keys,
                                                    const uint64_t *__restrict__ koff, uint32_t n,
                                                    const unsigned long long *__restrict__ table, uint64_t slots,
                                                    uint64_t bound,
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
            const unsigned long long want = slot_word0(h, len, 0, false) >> 32;  // tag | length
            uint64_t s = h & mask;
            for (uint64_t probe = 0; probe < bound; ++probe, s = (s + 1) & mask) {  // (the build's longest probe)
                const unsigned long long *slot = table + kSlotWords * s;
                const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(slot);
                if (a.x == kEmptySlot) break;
                if ((a.x >> 32) != want) continue;
                const ulonglong2 b = *reinterpret_cast<const ulonglong2 *>(slot + 2);
                const unsigned long long w[3] = {a.y, b.x, b.y};
                const uint32_t cur = slot_rec(a.x);
                if (!slot_key_equal(arena, rec_off, rec_kv, w, cur, [&](uint32_t i) { return k[i]; }, len)) continue;
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

// The values' offsets in the caller's buffer, on the device: an exclusive
// scan of ValueSize over the keys the lookup found (UINT64_MAX for the
// others), blocks of 1024, then the block sums by one wavefront, then the
// add; res[0] = the bytes of all found values.  (The host had read back
// status and sizes, summed them and sent the offsets down: a round trip of
// 16 B per key in the middle of the call.)
constexpr uint32_t kVoffBlock = 1024;
__global__ __launch_bounds__(kVoffBlock) void k_voff_block(const int32_t *__restrict__ status,
                                                           const uint32_t *__restrict__ vsize, uint32_t n,
                                                           uint64_t *__restrict__ voff, uint64_t *__restrict__ bsum) {
    __shared__ uint64_t ws[kVoffBlock / 64];
    const uint32_t i = blockIdx.x * kVoffBlock + threadIdx.x, lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const uint64_t v = i < n && status[i] == GCK_OK ? vsize[i] : 0;
    uint64_t inc = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t y = __shfl_up(inc, d, 64);
        if (lane >= (uint32_t)d) inc += y;
    }
    if (lane == 63) ws[wid] = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint64_t run = 0;
        for (uint32_t k = 0; k < kVoffBlock / 64; ++k) {
            const uint64_t t = ws[k];
            ws[k] = run;
            run += t;
        }
        bsum[blockIdx.x] = run;
    }
    __syncthreads();
    if (i < n) voff[i] = ws[wid] + inc - v;
}
__global__ void k_voff_top(uint64_t *__restrict__ bsum, uint32_t nb, uint64_t *__restrict__ res) {
    const uint32_t lane = threadIdx.x;
    uint64_t run = 0;
    for (uint32_t b0 = 0; b0 < nb; b0 += 64) {
        const uint32_t b = b0 + lane;
        const uint64_t v = b < nb ? bsum[b] : 0;
        uint64_t inc = v;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t y = __shfl_up(inc, d, 64);
            if (lane >= (uint32_t)d) inc += y;
        }
        if (b < nb) bsum[b] = run + inc - v;
        run += __shfl(inc, 63, 64);
    }
    if (lane == 0) res[0] = run;
}
__global__ __launch_bounds__(256) void k_voff_add(const int32_t *__restrict__ status, uint32_t n,
                                                  uint64_t *__restrict__ voff, const uint64_t *__restrict__ bsum) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n) voff[i] = status[i] == GCK_OK ? voff[i] + bsum[i / kVoffBlock] : ~0ull;
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
// match copies the value to dst + dst_off (if dst).  Groups of 64 items: the
// first one per wavefront static, the rest from an atomic queue (zeroed by
// the caller), claimed one group ahead: value sizes are heavy-tailed, so a
// fixed stride left the kernel waiting for the wavefronts that drew the
// largest values.
// Copy (Get with values): every found value is also copied to dst + dst_off
// from the registers its CRC is computed in -- a large one by the stripe
// stores of wave_crcs, a small one's whole 16 B pieces by lane_crc, the rest
// (a large value's first 16 bytes, a small one's last L % 16) by its lane.
// A value whose CRC fails is copied too; the caller reports no value for it.
// GS: items per wavefront group (64: a lane each; fewer when a batch is too
// small to give every wavefront of the chip a group of 64).
template <bool Copy, int GS = 64>
__global__ __launch_bounds__(1024) void k_verify(const uint8_t *__restrict__ arena, const uint32_t *__restrict__ g_slice,
                                                 uint64_t n,
                                                const uint64_t *__restrict__ item,
                                                const uint32_t *__restrict__ vsize,
                                                const uint32_t *__restrict__ expect, int32_t *__restrict__ status,
                                                uint32_t *__restrict__ crc_out, const uint64_t *__restrict__ dst_off,
                                                uint8_t *__restrict__ dst, uint32_t *__restrict__ queue) {
    __shared__ CrcTabs T;
    crc_tables(T, g_slice);
    const uint32_t lane = threadIdx.x & 63;
    uint32_t lb0, lb1;
    slice_bases(lane, lb0, lb1);
    const uint64_t groups = (n + GS - 1) / GS, waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    uint64_t gi = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    uint32_t claim = 0;
    if (gi < groups && lane == 0) claim = atomicAdd(queue, 1u);
    while (gi < groups) {
        const uint64_t mine = gi * GS + lane;
        const bool have = lane < (uint32_t)GS && mine < n;
        const bool ok = have && status[mine] == GCK_OK;
        const uint64_t off = ok ? item[mine] : 0;
        const uint32_t len = ok ? vsize[mine] : 0u, want = ok ? expect[mine] : 0u;
        const uint64_t doff = ok && dst ? dst_off[mine] : 0;
        uint32_t crc = 0;
        const bool small = ok && len <= kLaneMax;
        const uint64_t todo = __ballot(ok && !small);
        if (__ballot(small)) {  // small values: a lane each, all at once
            const uint32_t c = lane_crc<true, Copy, 32>(arena + off, len, small, T, lb0, lb1, dst + doff);  // (the arena is padded)
            if (small) crc = c;
        }
        if (todo) {
            const uint32_t c = wave_crcs<false, Copy>(todo, [&](int it) { return arena + lane_u64(off, it); }, len, T,
                                                      lb0, lb1, [&](uint32_t A) { return lanes_combine(T, lb0, A); },
                                                      [&](int it) { return dst + lane_u64(doff, it); });
            if ((todo >> lane) & 1) crc = c;
        }
        if constexpr (Copy) {
            if (ok && len >= 16 && (!small || (len & 15))) {  // a large value's first 16 bytes, a small one's last
                const uint32_t at = small ? len - 16 : 0u;
                const uint8_t *p = arena + off + at;
                const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
                const uint32_t *a = reinterpret_cast<const uint32_t *>(p - sh);
                store16u(dst + doff + at, __builtin_amdgcn_alignbyte(a[1], a[0], sh), __builtin_amdgcn_alignbyte(a[2], a[1], sh),
                            __builtin_amdgcn_alignbyte(a[3], a[2], sh), __builtin_amdgcn_alignbyte(a[4], a[3], sh));
            } else if (ok && len < 16) {
                for (uint32_t j = 0; j < len; ++j) dst[doff + j] = arena[off + j];
            }
        }
        if (have) {
            crc_out[mine] = crc;
            if (ok && crc != want) status[mine] = GCK_ECRC_FAILED;  // core/db.go:311-313
        }
        gi = waves + (uint32_t)__builtin_amdgcn_readfirstlane((int)claim);
        if (gi < groups && lane == 0) claim = atomicAdd(queue, 1u);
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
    if (!c->kd_valid || c->from_hints) return GCK_EINVAL;  // gck_ctx_keydir after the run first (values: data files)
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
        (rc = c->d_gcrc.ensure(n * 4ull)) || (rc = c->d_gvoff.ensure(n * 8ull)) ||
        (rc = c->d_gscan.ensure(((n + kVoffBlock - 1) / kVoffBlock + 1) * 8ull + 8)))
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
        c->kd_probe_bound,
        c->arena.as<uint8_t>(), c->d_rec_off.as<uint64_t>(), c->d_rec_kv.as<uint2>(),
        c->d_out.as<gck_rec>(), c->d_fbase.as<uint64_t>(), c->d_flen.as<uint64_t>(), c->d_gstat.as<int32_t>(),
        c->d_gitem.as<uint64_t>(), c->d_gvsize.as<uint32_t>(), c->d_gexp.as<uint32_t>());
    uint8_t *dvals = nullptr;
    if (values) {  // value offsets of the found keys, back to back (on the device; 8 B come back)
        const uint32_t nb = (n + kVoffBlock - 1) / kVoffBlock;
        uint64_t *bsum = c->d_gscan.as<uint64_t>(), *res = bsum + nb + 1;
        k_voff_block<<<nb, kVoffBlock, 0, s>>>(c->d_gstat.as<int32_t>(), c->d_gvsize.as<uint32_t>(), n,
                                               c->d_gvoff.as<uint64_t>(), bsum);
        k_voff_top<<<1, 64, 0, s>>>(bsum, nb, res);
        k_voff_add<<<(n + 255) / 256, 256, 0, s>>>(c->d_gstat.as<int32_t>(), n, c->d_gvoff.as<uint64_t>(), bsum);
        uint64_t tot = 0;
        GCK_HIP(hipMemcpyAsync(&tot, res, 8, hipMemcpyDeviceToHost, s));
        GCK_HIP(hipStreamSynchronize(s));
        if (tot > values_cap) {  // status / value_size of the lookup, for a retry
            GCK_HIP(hipMemcpyAsync(status, c->d_gstat.p, n * 4ull, hipMemcpyDeviceToHost, s));
            GCK_HIP(hipMemcpyAsync(value_size, c->d_gvsize.p, n * 4ull, hipMemcpyDeviceToHost, s));
            GCK_HIP(hipStreamSynchronize(s));
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
            return GCK_EINVAL;
        }
        if ((rc = c->d_gvals.ensure(tot))) return rc;
        dvals = c->d_gvals.as<uint8_t>();
    }
    // one 1024-thread workgroup per CU (the tables take 132 KiB of LDS)
    // groups of 16 when 64 would leave wavefronts idle (65,536 keys: 1,024
    // groups of 64 for 4,096 wavefronts; k_verify 383 us, profiles/r4zzb)
    const bool g16 = n < 64ull * 16 * c->n_cu;
    const uint32_t grid = std::min<uint32_t>(g16 ? (n + 255) / 256 : (n + 1023) / 1024, (uint32_t)c->n_cu);
    uint32_t *queue = c->d_queue.as<uint32_t>() + kQueueVerify;
    GCK_HIP(hipMemsetAsync(queue, 0, 4, s));
    (dvals ? (g16 ? k_verify<true, 16> : k_verify<true, 64>) : (g16 ? k_verify<false, 16> : k_verify<false, 64>))<<<grid, 1024, 0, s>>>(c->arena.as<uint8_t>(), c->d_slice.as<uint32_t>(), n, c->d_gitem.as<uint64_t>(), c->d_gvsize.as<uint32_t>(),
                                  c->d_gexp.as<uint32_t>(), c->d_gstat.as<int32_t>(), c->d_gcrc.as<uint32_t>(),
                                  c->d_gvoff.as<uint64_t>(), dvals, queue);
    GCK_HIP(hipEventRecord(b, s));
    GCK_HIP(hipMemcpyAsync(status, c->d_gstat.p, n * 4ull, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipMemcpyAsync(value_size, c->d_gvsize.p, n * 4ull, hipMemcpyDeviceToHost, s));
    GCK_HIP(hipMemcpyAsync(crc_calc, c->d_gcrc.p, n * 4ull, hipMemcpyDeviceToHost, s));
    if (values) GCK_HIP(hipMemcpyAsync(val_off, c->d_gvoff.p, n * 8ull, hipMemcpyDeviceToHost, s));
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
    if (!c->kd_valid || c->from_hints) return GCK_EINVAL;  // (a hint replay's arena holds no values)
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
    uint32_t *queue = c->d_queue.as<uint32_t>() + kQueueVerify;
    GCK_HIP(hipMemsetAsync(queue, 0, 4, s));
    k_verify<false><<<(uint32_t)c->n_cu, 1024, 0, s>>>(c->arena.as<uint8_t>(), c->d_slice.as<uint32_t>(), n, c->d_gitem.as<uint64_t>(),
                                                    c->d_gvsize.as<uint32_t>(), c->d_gexp.as<uint32_t>(),
                                                    c->d_gstat.as<int32_t>(), c->d_gcrc.as<uint32_t>(), nullptr,
                                                    nullptr, queue);
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
