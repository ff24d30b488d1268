// gck_math.h — CRC-32/IEEE algebra shared by host setup code and gfx950 kernels.
//
// The reference computes crc32.Checksum(val, IEEETable) (internal/crc/crc.go:8-10).
// Device code never walks a value byte-by-byte: it evaluates the same function
// through its GF(2) structure.  Notation (reflected domain, x^0 = 0x80000000):
//   F(c, B)   raw register update over bytes B from state c (no init / xorout)
//   Z_n(c)    = F(c, 0^n) = c * x^(8n) mod P        (linear, invertible)
//   crc(V)    = F(0, V) ^ Z_|V|(0xFFFFFFFF) ^ 0xFFFFFFFF
// F(0, .) ignores leading zero bytes, so masked (non-value) bytes that precede a
// value cost nothing; trailing masked bytes are removed with Z_{-m}.
// multmodp is the published zlib crc32_combine multiply (zlib 1.2.12+ crc32.c).
#pragma once
#include <stdint.h>

#ifndef GCK_HD
#if defined(__HIPCC__)
#define GCK_HD __host__ __device__
#else
#define GCK_HD
#endif
#endif

namespace gck {

constexpr uint32_t kPoly = 0xEDB88320u;
constexpr uint32_t kX0 = 0x80000000u;      // x^0
constexpr uint32_t kXinv = 0xDB710641u;    // x^-1 mod P (checked at setup)

// Data layout constants of the device pipeline.
constexpr int kSlab = 64;                  // bytes per lane per row (16 words)
constexpr int kRow = 64 * kSlab;           // 4096 B per wavefront row
constexpr uint32_t kNone32 = 0xFFFFFFFFu;
constexpr uint64_t kNone = ~0ull;

// a * b mod P (reflected).  Exits early when a's remaining bits are zero.
GCK_HD inline uint32_t multmodp(uint32_t a, uint32_t b) {
    if (a == 0) return 0;
    uint32_t m = kX0, p = 0;
    for (;;) {
        if (a & m) {
            p ^= b;
            if ((a & (m - 1)) == 0) break;
        }
        m >>= 1;
        b = (b & 1) ? (b >> 1) ^ kPoly : b >> 1;
    }
    return p;
}

// x^(8n) mod P by square-and-multiply.
GCK_HD inline uint32_t xpow8n(uint64_t n) {
    uint32_t r = kX0, base = kX0 >> 8;  // x^8
    while (n) {
        if (n & 1) r = multmodp(base, r);
        base = multmodp(base, base);
        n >>= 1;
    }
    return r;
}

GCK_HD inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Keyed counter hash of the corpus spec (DESIGN.md "Corpus").
GCK_HD inline uint64_t H(uint64_t seed, uint64_t tag, uint64_t i) {
    return mix64(mix64(seed ^ (tag * 0xD6E8FEB86659FD93ull)) + i);
}

}  // namespace gck
