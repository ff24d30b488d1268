// kd_common.h — key hashing shared by the device keydir (keydir.hip) and the
// batched Get (get.hip): both must hash a key to the same table slot.
#pragma once
#include "gck_internal.h"

namespace gck {

constexpr uint32_t kEmpty = 0xFFFFFFFFu;
constexpr int kKdTile = 1024;  // records per compaction tile (one workgroup)

// Key of a record: KeySize bytes after the header, or ValueSize bytes for a
// tombstone (KeySize 0; core/db.go:151-155).
__device__ __forceinline__ uint32_t key_len(const uint2 &kv) { return kv.x ? kv.x : kv.y; }  // (KeySize, ValueSize)

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

// 64-bit hash of a key's bytes (the table slot is its low bits, the merge
// partition its bits 40..63).
__device__ __forceinline__ uint64_t key_hash(const KeyWords &k, uint32_t len) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)len << 32);
    for (uint32_t i = 0; 4 * i < len; ++i) h = mix64d(h ^ k[i]) + i;
    return mix64d(h);
}

// Table slot: the key's hash tag (bits 32..63 of its hash, never all ones)
// above the index of its record; all ones = empty.  Same key => same tag, so
// a 64-bit max keeps the larger record index.
constexpr unsigned long long kEmptySlot = ~0ull;
// A slot is two words (GCK_KD_WIDE): (tag, record index) and the key's arena
// offset with its length in the top 16 bits (0xFFFF: 65,535 or longer, look
// the length up), written by the lane that claimed the slot right after its
// CAS (all ones until then: a probe then reads the record table instead), so
// a probe compares key bytes without two random record-table reads: C3 keydir
// 2.03-2.08 -> 1.81-1.87 ms, the rebuild of a run 1.51 -> 1.37 (profiles/r5p)
#ifndef GCK_KD_WIDE
#define GCK_KD_WIDE 1
#endif
constexpr uint32_t kSlotWords = GCK_KD_WIDE ? 2 : 1;
constexpr uint64_t kKeyOffMask = (1ull << 48) - 1;
__device__ __forceinline__ unsigned long long slot_key_word(uint64_t key_off, uint32_t len) {
    return (key_off & kKeyOffMask) | ((unsigned long long)(len < 0xFFFFu ? len : 0xFFFFu) << 48);
}
__device__ __forceinline__ uint32_t slot_tag(uint64_t h) {
    const uint32_t t = (uint32_t)(h >> 32);
    return t == 0xFFFFFFFFu ? 0xFFFFFFFEu : t;
}

}  // namespace gck
