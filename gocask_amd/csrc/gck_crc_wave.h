// gck_crc_wave.h — CRC-32/IEEE of many byte ranges by wavefronts: a lane per
// small range, the whole wavefront per large one in 1 KiB stripes with a ring
// of stripes in flight (k_verify's Get / scrub, k_encode_batch's records).
#pragma once
#include "gck_crc_lds.h"
#include "gck_math.h"

namespace gck {

// LDS tables: the conflict-free slicing-by-4 image (gck_crc_lds.h, 128 KiB,
// from the context's global tables); multiplication by the constant Z_1024
// as four byte tables, Z(A) = XOR_k Zs[k][byte k of A] (Z is linear in A);
// the lane shifts Z_{16 (31 - (l & 31))} as eight nibble tables per lane
// (entry (q, v) of lane l at word 512 q + 32 v + (l & 31): each lane of a
// 32-lane LDS group on its own bank, 16 KiB); Z_512 as four byte tables
// (lanes 0..31 are a further 512 bytes from the stripe end; read with a
// wave-uniform address only, so one copy has no conflicts).  152 KiB.  Ls and
// Z512 follow the slicing tables in the context's global table (built once
// per process on the host, replay.hip make_tables): kGLs, kGZ512 words in.
constexpr uint32_t kLaneShiftWords = 8 * 16 * 32;
constexpr uint32_t kGLs = 1024, kGZ512 = kGLs + kLaneShiftWords, kGTabWords = kGZ512 + 1024;
struct CrcTabs {
    uint32_t S[kSliceLdsWords];
    uint32_t Zs[4][256];
    uint32_t Ls[kLaneShiftWords];
    uint32_t Z512[4][256];
};
__device__ inline void fill_zs(CrcTabs &t) {
    const uint32_t z = xpow8n(1024);
    for (uint32_t e = threadIdx.x; e < 1024; e += blockDim.x) t.Zs[e >> 8][e & 0xFF] = multmodp(z, (e & 0xFF) << (8 * (e >> 8)));
}

// All of CrcTabs from the context's global table.
__device__ inline void crc_tables(CrcTabs &t, const uint32_t *__restrict__ g_tab) {
    fill_slice_lds(t.S, g_tab);
    fill_zs(t);
    for (uint32_t e = threadIdx.x; e < kLaneShiftWords; e += blockDim.x) t.Ls[e] = g_tab[kGLs + e];
    for (uint32_t e = threadIdx.x; e < 1024; e += blockDim.x) (&t.Z512[0][0])[e] = g_tab[kGZ512 + e];
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

// Inclusive XOR prefix within each 16-lane row (DPP row shifts), then row 0's
// total into row 1 and row 2's into row 3 (row_bcast:15): lane 31 = XOR of
// lanes 0..31, lane 63 = XOR of lanes 32..63.  DPP moves data in the VALU;
// __shfl_xor compiles to ds_bpermute through the LDS crossbar.  All lanes
// must be active (callers run it in wave-uniform control flow).
__device__ __forceinline__ uint32_t half_xor(uint32_t f) {
    f ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)f, 0x111, 0xF, 0xF, false);  // row_shr:1
    f ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)f, 0x112, 0xF, 0xF, false);  // row_shr:2
    f ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)f, 0x114, 0xF, 0xF, false);  // row_shr:4
    f ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)f, 0x118, 0xF, 0xF, false);  // row_shr:8
    f ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)f, 0x142, 0xA, 0xF, false);  // row_bcast:15 -> rows 1, 3
    return f;
}

__device__ __forceinline__ uint32_t zmul(const uint32_t (*Z)[256], uint32_t a) {
    return Z[0][a & 0xFF] ^ Z[1][(a >> 8) & 0xFF] ^ Z[2][(a >> 16) & 0xFF] ^ Z[3][a >> 24];
}

// crc32.ChecksumIEEE from the lanes' stripe registers A (lane l's chunk is
// followed by 16 (63 - l) bytes of the value): Z_{16 (31 - (l & 31))}(A) by
// the lane's nibble tables (address: nibble at bits 7..10 merged with the
// lane's bank offset lb0 in one v_bitop3, table q at + 2048 q bytes), XOR over
// each half-wave, then Z_512 of the lower half's sum (uniform), complemented.
// Replaces a 32-step branch-free multiply by the lane constant (~160 VALU per
// value; lanes_combine_gmul, for kernels without the tables).
__device__ __forceinline__ uint32_t lanes_combine(const CrcTabs &t, uint32_t lb0, uint32_t A) {
    uint32_t x8[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const int sh = 4 * q;
        const uint32_t x = sh >= 7 ? A >> (sh - 7) : A << (7 - sh);
        x8[q] = lds_at(t.Ls + q * 512, __builtin_amdgcn_bitop3_b32(x, 0x780u, lb0, 0xEA));
    }
    uint32_t f = xor3(xor3(x8[0], x8[1], x8[2]), xor3(x8[3], x8[4], x8[5]), x8[6] ^ x8[7]);
    // XOR over each half-wave by DPP (row prefixes, then row 0 into row 1 and
    // row 2 into row 3): lane 31 holds lanes 0..31, lane 63 lanes 32..63
    f = half_xor(f);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)f, 31), hi = (uint32_t)__builtin_amdgcn_readlane((int)f, 63);
    return ~(zmul(t.Z512, lo) ^ hi);
}
__device__ __forceinline__ uint32_t lanes_combine_gmul(uint32_t kl, uint32_t A) {
    uint32_t f = half_xor(gmul(kl, A));  // kl = x^(8 * 16 (63 - lane))
    return ~((uint32_t)__builtin_amdgcn_readlane((int)f, 31) ^ (uint32_t)__builtin_amdgcn_readlane((int)f, 63));
}

// Lane it's x, it wave-uniform: v_readlane into a scalar register, so the
// values derived from it (a value's stripe count, padding, shift and base) and
// the branches on them stay scalar.  __shfl would be a ds_bpermute whose
// result the compiler treats as divergent: the per-value bookkeeping then ran
// in VALU 64-bit arithmetic and every branch on it under an exec mask.
__device__ __forceinline__ uint32_t lane_u32(uint32_t x, int it) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, it);
}
__device__ __forceinline__ uint64_t lane_u64(uint64_t x, int it) {
    return ((uint64_t)lane_u32((uint32_t)(x >> 32), it) << 32) | lane_u32((uint32_t)x, it);
}

// The 16 bytes of virtual position v (value p[0, L) zero-padded in front by
// pad bytes), plus the next dword for the byte shift: one 16 B and one 4 B
// load (dword aligned), unconditional.  A lane wholly in the padding loads
// the value's first dwords instead (never before the arena; wave_crc masks its
// bytes); a lane straddling the value start reads up to 15 bytes before it
// (the record's header and key: inside the arena).
typedef uint32_t u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
// 16 bytes to any byte address: one dwordx4 store (gfx9 global stores need no
// alignment; the amdhsa target compiles a 1-byte-aligned vector access to it).
// The copies built on it (the encoder's records, Get's values) rely on one
// thread's overlapping stores landing in program order.
typedef uint32_t u32x4_a1 __attribute__((ext_vector_type(4), aligned(1)));
__device__ __forceinline__ void store16u(uint8_t *dst, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    u32x4_a1 x;
    x.x = a;
    x.y = b;
    x.z = c;
    x.w = d;
    *reinterpret_cast<u32x4_a1 *>(dst) = x;
}
__device__ __forceinline__ void store16u(uint8_t *dst, uint4 v) { store16u(dst, v.x, v.y, v.z, v.w); }
// (Pointer arithmetic only, never an integer cast back to a pointer: that
// would make the loads flat, and flat loads also count on lgkmcnt, so every
// LDS table wait would wait for HBM too.)
// Start of a value's CRC: J = ceil(L / 1 KiB) stripes, pad = J KiB - L; all
// wave-uniform, so the byte shift sh and the dword-aligned base b of the
// virtual buffer (b + v = the dword holding virtual byte v, sh its offset)
// are scalars.
// Stripe indices and in-value positions are 32-bit (L < 2^32, so J <= 2^22
// and j << 10 < 2^32): gfx9's scalar unit has no 64-bit less-than, and the
// 64-bit head-stripe test (j << 10) < pad + 4 was a VALU compare on every
// stripe.  head4 / head16: the stripes that hold bytes of [0, pad + 4) /
// [0, pad + 16) (1 or 2).
struct CrcJob {
    const uint8_t *p, *b;
    uint32_t J, pad, sh, head4, head16;
    __device__ CrcJob(const uint8_t *p_, uint32_t L)
        : p(p_), J((uint32_t)(((uint64_t)L + 1023) >> 10)), pad((J << 10) - L),
          sh((uint32_t)((reinterpret_cast<uintptr_t>(p_) - pad) & 3)),
          head4((pad + 4 + 1023) >> 10), head16((pad + 16 + 1023) >> 10) {
        b = p - pad - sh;
    }
};
// NT: non-temporal stripe loads.  Both callers now keep the default policy:
// a stripe's 1 KiB starts anywhere, so its first and last lines are shared
// with the neighbouring stripes (and the fifth dword load reads the next
// lane's line again) -- non-temporal loads re-fetch them: C3 scrub 2.83-2.92
// against 3.21-3.27 ms (profiles/r4zy), the encoder 0.77 against 0.83 ms.
template <bool NT = true>
__device__ __forceinline__ void stripe_load(const CrcJob &jb, uint32_t j, uint32_t d[5]) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t v = (j << 10) + 16u * lane;
    const uint8_t *a = jb.b + v;
    if (j < jb.head16) {  // (uniform) the value's first stripe(s): lanes wholly in the padding
        const uint8_t *p0 = jb.p - (reinterpret_cast<uintptr_t>(jb.p) & 3);
        a = v + 16 <= jb.pad ? p0 : a;
    }
    // (NT: round 2 measured 4.92 -> 4.76-4.90 ms for the scrub of then; round 4 reversed it, above)
    u32x4_a4 x;
    if constexpr (NT)
        x = __builtin_nontemporal_load(reinterpret_cast<const u32x4_a4 *>(a));
    else
        x = *reinterpret_cast<const u32x4_a4 *>(a);
    d[0] = x.x;
    d[1] = x.y;
    d[2] = x.z;
    d[3] = x.w;
    // the dword after the chunk when the shift needs it, else one inside it
    // (alignbyte by 0 ignores d[4]): nothing past a value's last dword is read
    d[4] = *reinterpret_cast<const uint32_t *>(a + (jb.sh ? 16 : 12));
}

// crc32.ChecksumIEEE of a value by one wavefront.  The value is read as a
// virtual buffer of J stripes of 1 KiB, zero-padded at the FRONT (F(0, .)
// ignores leading zeros), lane l taking the 16 bytes at 16 l of every stripe
// (coalesced loads).  Lane state: A <- Z_1024(A) ^ F(0, chunk), i.e. Horner
// over the lane's chunks 1 KiB apart (= F(Z_1008(A), chunk); the chunk's CRC
// does not wait for A, whose only dependent step is the one Z_1024 multiply).  The 0xFFFFFFFF init is the complement of the
// value's first 4 bytes (F(~0, V) = F(0, V with bytes 0..3 ^ 0xFF)).  Lane l's
// part is finally shifted past the 16 (63-l) bytes after it and the lanes
// XOR-reduced (lanes_combine): F(~0, V); crc = ~that.
//
// One stripe of the value at virtual stripe j into A.  Store: the value's
// bytes also go to ob (the value's copy, any alignment) -- every lane whose 16
// bytes lie inside the value writes them (the value's first < 16 bytes are the
// caller's); one buffer store per stripe on every path (lanes in the padding
// at an offset past the stripe's 1 KiB window: dropped by the bounds check),
// so the vmcnt counts stay exact.
typedef uint32_t u32x4_st __attribute__((ext_vector_type(4)));
template <bool Store = false>
__device__ __forceinline__ uint32_t fold_stripe(const CrcJob &jb, uint32_t j, const uint32_t d[5], uint32_t A,
                                                const CrcTabs &t, uint32_t lb0, uint32_t lb1,
                                                uint8_t *ob = nullptr) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t v = (j << 10) + 16u * lane;  // virtual position of this lane's chunk
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], jb.sh);
    if constexpr (Store) {
        // the stripe's window in the copy: ob + (j KiB - pad), never read or
        // written outside [ob, ob + L) (the padding lanes are dropped)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(ob + (j << 10) - jb.pad, 0, 1024, 0x00020000);
        const u32x4_st x = {w[0], w[1], w[2], w[3]};
        // (non-temporal: written once; 0.717-0.719 against 0.732-0.737 ms per GB)
        __builtin_amdgcn_raw_buffer_store_b128(x, rs, (int)(v >= jb.pad ? 16u * lane : 0x800u), 0, 2);
    }
    // (uniform) the stripes that hold the value's first 4 bytes; then per lane:
    // bytes before the value are zero, its first 4 complemented
    if (j < jb.head4) {  // (a scalar branch, then the lanes)
      if (v < jb.pad + 4) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int32_t lead = (int32_t)jb.pad - (int32_t)(v + 4 * i);  // bytes of dword i before the value (v < 2 KiB here)
            const uint32_t keep = lead >= 4 ? 0u : lead <= 0 ? 0xFFFFFFFFu : 0xFFFFFFFFu << (8 * lead);
            const int32_t cl = lead + 4;  // bytes of dword i before the value's byte 4
            const uint32_t flip = cl <= 0 ? 0u : cl >= 4 ? 0xFFFFFFFFu : 0xFFFFFFFFu >> (8 * (4 - cl));
            w[i] = (w[i] & keep) ^ (flip & keep);
        }
      }
    }
    uint32_t c = slice4x(t.S, lb0, lb1, w[0], w[1]);
    c = slice4x(t.S, lb0, lb1, c, w[2]);
    c = slice4x(t.S, lb0, lb1, c, w[3]);
    return slice4x(t.S, lb0, lb1, c, zmul(t.Zs, A));
}

// The large values of a wavefront's 64 items (mask todo; ptr_of(i) = item i's
// bytes, a global pointer built by pointer arithmetic), one after another,
// with kRing stripes in flight across value boundaries: the stripe folded now
// was loaded kRing stripes earlier (16 KiB per CU in flight with one stripe
// ahead is far below what HBM latency needs).  All control is wave-uniform;
// every load is issued unconditionally (a dummy reload past the last stripe),
// so the compiler's vmcnt counts stay exact.  Item t's CRC lands in lane t.
constexpr int kRing = 4;  // ring depths 2, 4 and 8 measured the same (again in round 3)
struct NoCopy {
    __device__ uint8_t *operator()(int) const { return nullptr; }
};
template <bool NT = true, bool Store = false, class PtrOf, class Combine, class OutOf = NoCopy>
__device__ uint32_t wave_crcs(uint64_t todo, PtrOf ptr_of, uint32_t len, const CrcTabs &t, uint32_t lb0,
                              uint32_t lb1, Combine combine, OutOf out_of = OutOf()) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t out = 0;
    auto job = [&](int it) { return CrcJob(ptr_of(it), lane_u32(len, it)); };
    // load cursor
    uint64_t lrem = todo;
    int lt = __builtin_ctzll(todo);
    CrcJob lj = job(lt);
    uint32_t ls = 0;
    auto load_next = [&](uint32_t d[5]) {
        stripe_load<NT>(lj, ls, d);
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
    uint8_t *ob = out_of(ct);
    uint32_t cs = 0;
    uint32_t A = 0;
    while (crem) {
#pragma unroll
        for (int k = 0; k < kRing; ++k) {
            // the fold (and a value's end) only while values remain; the
            // reload of ring[k] on every pass, so every path issues the same
            // loads in the same order and the compiler's vmcnt waits stay
            // exact (a load inside the branch made the merge at the loop head
            // wait for every load in flight: the ring drained once per round)
            if (crem) {
                A = fold_stripe<Store>(cj, cs, ring[k], A, t, lb0, lb1, ob);
                if (++cs == cj.J) {  // value done
                    const uint32_t f = combine(A);
                    if (lane == (uint32_t)ct) out = f;
                    A = 0;
                    cs = 0;
                    crem &= crem - 1;
                    if (crem) {
                        ct = __builtin_ctzll(crem);
                        cj = job(ct);
                        ob = out_of(ct);
                    }
                }
            }
            load_next(ring[k]);
        }
    }
    return out;
}

constexpr uint32_t kLaneMax = 256;  // values up to this size: one lane each

// crc32.ChecksumIEEE of a small value by one lane (lanes run different
// values): aligned dwords, 4 R bytes of loads in flight per round (R = 32:
// a 256 B value in two round trips; scrub and encoder about 1 % faster than
// R = 16, profiles/r4zs), slicing-by-4
// per word, the last 0..3 bytes one at a time.  Wide: the round's dwords as
// four 16 B loads (each lane's address is its own line, so one instruction
// per 16 B instead of per 4 B); reads up to 12 bytes past the value's last
// dword, so only for buffers padded past their end (the replay arena).
// Store: the value's whole 16 B pieces also go to op (any alignment), from
// the same registers; the last L % 16 bytes are the caller's.
template <bool Wide = false, bool Store = false, int R = 16>
__device__ inline uint32_t lane_crc(const uint8_t *p, uint32_t L, bool act, const CrcTabs &t, uint32_t lb0, uint32_t lb1,
                                    uint8_t *op = nullptr) {
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
    const uint32_t *a = reinterpret_cast<const uint32_t *>(p - sh);
    const uint32_t nw = act ? (sh + L + 3) >> 2 : 0u;  // dwords covering the value
    uint32_t c = 0xFFFFFFFFu, pos = 0;
    for (uint32_t b = 0; __ballot(b < nw); b += R) {
        uint32_t d[R + 1];
        if constexpr (Wide) {
#pragma unroll
            for (int k = 0; k < R / 4; ++k) {
                u32x4_a4 x = {0u, 0u, 0u, 0u};
                if (b + 4 * k < nw) x = *reinterpret_cast<const u32x4_a4 *>(a + b + 4 * k);
                d[4 * k] = x.x;
                d[4 * k + 1] = x.y;
                d[4 * k + 2] = x.z;
                d[4 * k + 3] = x.w;
            }
            d[R] = b + R < nw ? a[b + R] : 0u;
        } else {
#pragma unroll
            for (int i = 0; i < R + 1; ++i) d[i] = b + i < nw ? a[b + i] : 0u;
        }
        if constexpr (Store) {
#pragma unroll
            for (int q = 0; q < R / 4; ++q) {
                if (act && 4 * b + 16 * q + 16 <= L)
                    store16u(op + 4 * b + 16 * q, __builtin_amdgcn_alignbyte(d[4 * q + 1], d[4 * q], sh),
                             __builtin_amdgcn_alignbyte(d[4 * q + 2], d[4 * q + 1], sh),
                             __builtin_amdgcn_alignbyte(d[4 * q + 3], d[4 * q + 2], sh),
                             __builtin_amdgcn_alignbyte(d[4 * q + 4], d[4 * q + 3], sh));
            }
        }
#pragma unroll
        for (int i = 0; i < R; ++i) {
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


}  // namespace gck
