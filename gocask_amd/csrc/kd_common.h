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

// The same words with the first 28 bytes in registers: two 16-byte loads at
// construction, so a probe's compare does not start a memory round trip after
// the slot read (k_kd_insert); words 7.. from memory.
typedef uint32_t kd_u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));
struct KeyRegs {
    KeyWords m;
    uint32_t v0, v1, v2, v3, v4, v5, v6;
    __device__ KeyRegs(const uint8_t *arena, uint64_t o, uint32_t n) : m(arena, o, n) {
        const kd_u32x4_a4 *p = reinterpret_cast<const kd_u32x4_a4 *>(m.w);
        const kd_u32x4_a4 a = p[0], b = p[1];
        v0 = __builtin_amdgcn_alignbyte(a.y, a.x, m.sh);
        v1 = __builtin_amdgcn_alignbyte(a.z, a.y, m.sh);
        v2 = __builtin_amdgcn_alignbyte(a.w, a.z, m.sh);
        v3 = __builtin_amdgcn_alignbyte(b.x, a.w, m.sh);
        v4 = __builtin_amdgcn_alignbyte(b.y, b.x, m.sh);
        v5 = __builtin_amdgcn_alignbyte(b.z, b.y, m.sh);
        v6 = __builtin_amdgcn_alignbyte(b.w, b.z, m.sh);
    }
    __device__ __forceinline__ uint32_t operator()(uint32_t i) const {
        if (i >= 7) return m[i];
        const uint32_t v = i == 0 ? v0 : i == 1 ? v1 : i == 2 ? v2 : i == 3 ? v3 : i == 4 ? v4 : i == 5 ? v5 : v6;
        const uint32_t left = m.len - 4 * i;
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

// Table slot, 32 bytes: word 0 = the key's hash tag (bits 48..63 of its
// hash) | its length (16 bits, 0xFFFF: 65,535 or longer) | the index of its
// record (31 bits) | 1 if that record is a tombstone; all ones = empty.  Same
// key => same tag and length, so a 64-bit max on word 0 keeps the larger
// record index (the tombstone bit never decides: indices differ), and the
// marking reads the winner's kind from the slot, not from the record table.  Words 1..3 = the key's first 24
// bytes (zero past its end), written by the lane that claimed the slot right
// after its CAS: a probe compares keys of up to 24 bytes without reading the
// arena.  A word still all ones (not landed yet, or a key whose 8 bytes are
// all 0xFF) is compared from the arena instead.  C3: the byte compares of a
// key's earlier records against its winner were 0.53 of the 1.37 ms keydir
// (profiles/r5u); the 16-byte slots of profiles/r5p (tag, index; key offset,
// length) saved the record-table reads but not the arena's.
constexpr unsigned long long kEmptySlot = ~0ull;
constexpr uint32_t kSlotWords = 4, kInlineKey = 24;
constexpr uint64_t kKdMaxRecs = 1ull << 31;  // record indices in 31 bits
__device__ __forceinline__ unsigned long long slot_word0(uint64_t h, uint32_t len, uint64_t r, bool tomb) {
    return ((h >> 48) << 48) | ((unsigned long long)(len < 0xFFFFu ? len : 0xFFFFu) << 32) |
           ((uint32_t)r << 1) | (tomb ? 1u : 0u);
}
__device__ __forceinline__ uint32_t slot_rec(unsigned long long w0) { return (uint32_t)w0 >> 1; }

// Table slots for an expected number of distinct keys: a power of two, load
// <= 0.8.  A table sized for the keys expected, not for every record (C3: 4.4
// M keys of 10.24 M records -> 8 M slots, 256 MiB: it stays in the Infinity
// Cache, which 16 M slots of 32 B did not).  A key that finds no empty slot
// within kMaxProbe probes sets the overflow word and the table is built again
// for every record distinct (kd_table_slots(n), load <= 0.8); that last build
// probes without a bound (a crafted or unlucky key set whose hashes cluster
// still gets a keydir, as the reference's Go map would) and records its
// longest probe past kMaxProbe, which is then the lookups' bound
// (Ctx::kd_probe_bound).
constexpr uint32_t kMaxProbe = 256;
inline uint64_t kd_table_slots(uint64_t keys) {
    uint64_t slots = 1024;
    while (slots < keys + keys / 4) slots <<= 1;
    return slots;
}
// keys expected: the last keydir's count on this context, else half the records
inline uint64_t kd_keys_expected(uint64_t hint, uint64_t n) { return hint ? hint + hint / 8 : n / 2; }

__device__ __forceinline__ bool same_key(const uint8_t *__restrict__ arena, const uint64_t *__restrict__ rec_off,
                                         uint64_t a, uint64_t b, uint32_t len) {
    const KeyWords ka(arena, rec_off[a] + 16, len), kb(arena, rec_off[b] + 16, len);
    for (uint32_t i = 0; 4 * i < len; ++i)
        if (ka[i] != kb[i]) return false;
    return true;
}

// 8-byte word j of a key given its 4-byte words (bytes past the key zero)
template <class Words>
__device__ __forceinline__ unsigned long long key_word8(const Words &k, uint32_t len, uint32_t j) {
    const uint32_t lo = 8 * j < len ? k(2 * j) : 0u, hi = 8 * j + 4 < len ? k(2 * j + 1) : 0u;
    return ((unsigned long long)hi << 32) | lo;
}

// Does the slot's key (words w1..w3, record ci) equal key k (len bytes)?
// Inline words first; a word not landed, or a key past 24 bytes, from the arena.
template <class Words>
__device__ __forceinline__ bool slot_key_equal(const uint8_t *__restrict__ arena, const uint64_t *__restrict__ rec_off,
                                               const uint2 *__restrict__ rec_kv, const unsigned long long w[3],
                                               uint32_t ci, const Words &k, uint32_t len) {
    if (len >= 0xFFFFu && key_len(rec_kv[ci]) != len) return false;  // word 0 holds 0xFFFF for both
    bool known = true;
#pragma unroll
    for (uint32_t j = 0; j < 3; ++j) {
        if (8 * j >= len) break;
        if (w[j] == kEmptySlot) {
            known = false;
        } else if (w[j] != key_word8(k, len, j)) {
            return false;  // a landed word differs: another key
        }
    }
    if (known && len <= kInlineKey) return true;
    const KeyWords a(arena, rec_off[ci] + 16, len);
    for (uint32_t i = known ? kInlineKey / 4 : 0; 4 * i < len; ++i)
        if (a[i] != k(i)) return false;
    return true;
}

// Record r (key hash h, key of len bytes, its 4-byte words k(i)) into the
// open-addressing table: a slot is claimed by CAS on word 0; a probe compares
// word 0's tag and length before any key bytes; records of the same key keep
// the largest index with a 64-bit atomicMax, so the last writer in walk order
// wins whatever order the lanes run in.  Keys are never removed, so a probe
// sequence never skips a key's slot.  False: no slot within `bound` probes.
// Probes past kMaxProbe (the unbounded last build) are recorded in *longest.
// (k_kd_insert, and k_finalize when the run builds the table: gck_ctx_keydir_hash)
template <class Words>
__device__ __forceinline__ bool kd_insert_rec(const uint8_t *__restrict__ arena, const uint64_t *__restrict__ rec_off,
                                              const uint2 *__restrict__ rec_kv, unsigned long long *__restrict__ table,
                                              uint64_t mask, uint64_t h, uint64_t r, bool tomb, const Words &k,
                                              uint32_t len, uint64_t bound = kMaxProbe, uint32_t *longest = nullptr) {
    const unsigned long long mine = slot_word0(h, len, r, tomb);
    uint64_t s = h & mask;
    for (uint64_t probe = 0; probe < bound; ++probe, s = (s + 1) & mask) {
        if (probe >= kMaxProbe && longest) atomicMax(longest, (uint32_t)min(probe + 1, (uint64_t)0xFFFFFFFFu));
        unsigned long long *slot = table + kSlotWords * s;
        // plain reads: word 0 only goes EMPTY -> (tag, len, i) -> (tag, len,
        // larger i), the key words EMPTY -> the claimer's key, so a stale word
        // 0 is EMPTY (the CAS then returns the truth) or an older record of
        // the same key, and a stale key word is all ones (compared from the arena)
        const ulonglong2 a = *reinterpret_cast<const ulonglong2 *>(slot);
        const ulonglong2 b = *reinterpret_cast<const ulonglong2 *>(slot + 2);
        unsigned long long cur = a.x, w[3] = {a.y, b.x, b.y};
        if (cur == kEmptySlot) {
            const unsigned long long prev = atomicCAS(slot, kEmptySlot, mine);
            if (prev == kEmptySlot) {  // claimed: the key's first 24 bytes
                slot[1] = key_word8(k, len, 0);
                slot[2] = key_word8(k, len, 1);
                slot[3] = key_word8(k, len, 2);
                return true;
            }
            cur = prev;
            const ulonglong2 a2 = *reinterpret_cast<const ulonglong2 *>(slot);
            const ulonglong2 b2 = *reinterpret_cast<const ulonglong2 *>(slot + 2);
            w[0] = a2.y;
            w[1] = b2.x;
            w[2] = b2.y;
        }
        if ((cur >> 32) != (mine >> 32)) continue;  // tag or length differ
        const uint32_t ci = slot_rec(cur);
        if (slot_key_equal(arena, rec_off, rec_kv, w, ci, k, len)) {
            if (ci < r) atomicMax(slot, mine);  // same key: the later record wins
            return true;
        }
    }
    return false;  // overflow: the caller flags it, the table is built again larger
}

}  // namespace gck
