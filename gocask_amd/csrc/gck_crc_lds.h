// gck_crc_lds.h — bank-conflict-free slicing-by-4 CRC-32/IEEE tables in LDS,
// shared by the kernels that fold bytes at stream rate (k_crc_rows, k_verify).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gck {

// LDS image of the slicing-by-4 tables: two 64 KiB regions; in region r,
// entry b of half h, copy l31 sits at byte address r*65536 + b*256 + h*128 +
// l31*4 (tables T3, T2 in region 0, T1, T0 in region 1).  Every lane of a
// 32-lane LDS group reads its own bank, so lookups are conflict free
// (MI355X_MICROARCH.md §LDS), and the address of a lookup is ONE v_perm_b32:
// byte 0 = the lane's l31*4, byte 1 = the index byte, byte 2 = the region
// (from the lane base lb0 = l31*4 or lb1 = 65536 + l31*4); the half is the
// ds_read immediate offset.  128 KiB: kSliceLdsWords dwords.
constexpr uint32_t kSliceLdsWords = 32768;

__device__ __forceinline__ uint32_t lds_at(const uint32_t *lds, uint32_t byte_addr) {
    return *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(lds) + byte_addr);
}
template <int K>
__device__ __forceinline__ uint32_t tbl_addr(uint32_t c, uint32_t lb) {
    return __builtin_amdgcn_perm(c, lb, 0x0C020000u | ((4u + K) << 8));
}
// a ^ b ^ c in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
// One slicing-by-4 step on a = crc ^ word, with the next word x folded in:
// T3[a0] ^ T2[a1] ^ T1[a2] ^ T0[a3] ^ x.  4 v_perm + 4 ds_read + 2 v_bitop3.
__device__ __forceinline__ uint32_t slice4x(const uint32_t *lds, uint32_t lb0, uint32_t lb1, uint32_t a,
                                            uint32_t x) {
    return xor3(xor3(lds_at(lds, tbl_addr<0>(a, lb0)), lds_at(lds, tbl_addr<1>(a, lb0) + 128),
                     lds_at(lds, tbl_addr<2>(a, lb1))),
                lds_at(lds, tbl_addr<3>(a, lb1) + 128), x);
}
// One byte: T0[(c ^ x) & 0xFF] ^ (c >> 8)
__device__ __forceinline__ uint32_t byte1x(const uint32_t *lds, uint32_t lb1, uint32_t c, uint32_t x) {
    return lds_at(lds, tbl_addr<0>(c ^ x, lb1) + 128) ^ (c >> 8);
}
// The lane's table bases.
__device__ __forceinline__ void slice_bases(uint32_t lane, uint32_t &lb0, uint32_t &lb1) {
    lb0 = (lane & 31) * 4;
    lb1 = 65536 + (lane & 31) * 4;
}
// Fill the image from the four 256-entry tables in global memory (T[k*256+b]
// = Tk[b], as make_tables builds them).  No barrier.
__device__ __forceinline__ void fill_slice_lds(uint32_t *lds, const uint32_t *__restrict__ g_slice) {
    for (uint32_t i = threadIdx.x; i < kSliceLdsWords; i += blockDim.x)
        lds[i] = g_slice[(3 - ((i >> 13) & 2) - ((i >> 5) & 1)) * 256 + ((i >> 6) & 255)];
}

}  // namespace gck
