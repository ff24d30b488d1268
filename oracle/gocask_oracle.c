/*
 * gocask_oracle.c — TEST INFRASTRUCTURE ONLY (see gocask_oracle.h).
 *
 * CPU restatement of aneshas/gocask's replay path.  Every function cites the
 * reference lines it restates.  Go stdlib semantics that the reference relies
 * on (binary.Read / io.ReadFull / bufio.Reader.Discard EOF classes, hash/crc32
 * IEEE) are restated from their published behaviour; the reference's own
 * tests pin the result (tests/golden/, tests/test_oracle_golden.py).
 */
#include "gocask_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- CRC --- */
/* internal/crc/crc.go:5-10: crc32.Checksum(val, MakeTable(0xedb88320)).
 * MakeTable(IEEE) is the reflected table for poly 0xEDB88320; Checksum runs
 * crc = ^0, per byte crc = T[(crc^b)&0xff] ^ crc>>8, returns ^crc. */
static uint32_t T8[8][256];
static int tables_ready = 0;

static void init_tables(void) {
    if (tables_ready) return;
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : c >> 1;
        T8[0][n] = c;
    }
    for (int t = 1; t < 8; t++)
        for (uint32_t n = 0; n < 256; n++)
            T8[t][n] = (T8[t - 1][n] >> 8) ^ T8[0][T8[t - 1][n] & 0xff];
    tables_ready = 1;
}

uint32_t orc_crc32(const uint8_t *p, uint64_t n) {
    init_tables();
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < n; i++) c = T8[0][(c ^ p[i]) & 0xff] ^ (c >> 8);
    return ~c;
}

uint32_t orc_crc32_fast(const uint8_t *p, uint64_t n) {
    init_tables();
    uint32_t c = 0xFFFFFFFFu;
    while (n && ((uintptr_t)p & 7)) { c = T8[0][(c ^ *p++) & 0xff] ^ (c >> 8); n--; }
    while (n >= 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        lo ^= c;
        c = T8[7][lo & 0xff] ^ T8[6][(lo >> 8) & 0xff] ^ T8[5][(lo >> 16) & 0xff] ^
            T8[4][lo >> 24] ^ T8[3][hi & 0xff] ^ T8[2][(hi >> 8) & 0xff] ^
            T8[1][(hi >> 16) & 0xff] ^ T8[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) c = T8[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    return ~c;
}

/* CPU-baseline CRC (bench.py cpu_baseline "ref_crc"): Go's hash/crc32 on
 * amd64 computes IEEE CRCs of 64 bytes or more with PCLMULQDQ folding
 * (archUpdateIEEE -> ieeeCLMUL: the len & ~15 prefix by carry-less multiply,
 * the rest by slicing-by-8).  This is the same published algorithm (Gopal et
 * al., "Fast CRC Computation for Generic Polynomials Using PCLMULQDQ", the
 * bit-reflected constants for 0xEDB88320), so the baseline's CRC runs at Go's
 * speed class instead of a table loop's.  Checked against zlib.crc32 in
 * tests/test_oracle_golden.py.  Falls back to slicing-by-8 without CLMUL. */
#if defined(__x86_64__)
#include <immintrin.h>
__attribute__((target("pclmul,sse4.1"))) static uint32_t clmul_fold(const uint8_t *buf, uint64_t len, uint32_t crc) {
    /* len >= 64, a multiple of 16; crc is the register (pre-inverted) */
    const __m128i k1k2 = _mm_set_epi64x(0x01c6e41596ll, 0x0154442bd4ll);
    const __m128i k3k4 = _mm_set_epi64x(0x00ccaa009ell, 0x01751997d0ll);
    const __m128i k5k0 = _mm_set_epi64x(0, 0x0163cd6124ll);
    const __m128i poly = _mm_set_epi64x(0x01f7011641ll, 0x01db710641ll);
    __m128i x0, x1, x2, x3, x4, x5, x6, x7, x8;
    x1 = _mm_loadu_si128((const __m128i *)(buf + 0x00));
    x2 = _mm_loadu_si128((const __m128i *)(buf + 0x10));
    x3 = _mm_loadu_si128((const __m128i *)(buf + 0x20));
    x4 = _mm_loadu_si128((const __m128i *)(buf + 0x30));
    x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)crc));
    x0 = k1k2;
    buf += 64;
    len -= 64;
    while (len >= 64) { /* four lanes of 128 bits folded 512 bits forward */
        x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
        x6 = _mm_clmulepi64_si128(x2, x0, 0x00);
        x7 = _mm_clmulepi64_si128(x3, x0, 0x00);
        x8 = _mm_clmulepi64_si128(x4, x0, 0x00);
        x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
        x2 = _mm_clmulepi64_si128(x2, x0, 0x11);
        x3 = _mm_clmulepi64_si128(x3, x0, 0x11);
        x4 = _mm_clmulepi64_si128(x4, x0, 0x11);
        x1 = _mm_xor_si128(_mm_xor_si128(x1, x5), _mm_loadu_si128((const __m128i *)(buf + 0x00)));
        x2 = _mm_xor_si128(_mm_xor_si128(x2, x6), _mm_loadu_si128((const __m128i *)(buf + 0x10)));
        x3 = _mm_xor_si128(_mm_xor_si128(x3, x7), _mm_loadu_si128((const __m128i *)(buf + 0x20)));
        x4 = _mm_xor_si128(_mm_xor_si128(x4, x8), _mm_loadu_si128((const __m128i *)(buf + 0x30)));
        buf += 64;
        len -= 64;
    }
    x0 = k3k4; /* the four lanes into one */
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x2), x5);
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x3), x5);
    x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x4), x5);
    while (len >= 16) { /* single 128-bit folds */
        x2 = _mm_loadu_si128((const __m128i *)buf);
        x5 = _mm_clmulepi64_si128(x1, x0, 0x00);
        x1 = _mm_clmulepi64_si128(x1, x0, 0x11);
        x1 = _mm_xor_si128(_mm_xor_si128(x1, x2), x5);
        buf += 16;
        len -= 16;
    }
    /* 128 -> 64 bits, then Barrett reduction to 32 */
    x2 = _mm_clmulepi64_si128(x1, x0, 0x10);
    x3 = _mm_setr_epi32(~0, 0, ~0, 0);
    x1 = _mm_srli_si128(x1, 8);
    x1 = _mm_xor_si128(x1, x2);
    x0 = k5k0;
    x2 = _mm_srli_si128(x1, 4);
    x1 = _mm_and_si128(x1, x3);
    x1 = _mm_clmulepi64_si128(x1, x0, 0x00);
    x1 = _mm_xor_si128(x1, x2);
    x0 = poly;
    x2 = _mm_and_si128(x1, x3);
    x2 = _mm_clmulepi64_si128(x2, x0, 0x10);
    x2 = _mm_and_si128(x2, x3);
    x2 = _mm_clmulepi64_si128(x2, x0, 0x00);
    x1 = _mm_xor_si128(x1, x2);
    return (uint32_t)_mm_extract_epi32(x1, 1);
}
#endif

static uint32_t slice8_update(uint32_t c, const uint8_t *p, uint64_t n) {
    while (n >= 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        lo ^= c;
        c = T8[7][lo & 0xff] ^ T8[6][(lo >> 8) & 0xff] ^ T8[5][(lo >> 16) & 0xff] ^
            T8[4][lo >> 24] ^ T8[3][hi & 0xff] ^ T8[2][(hi >> 8) & 0xff] ^
            T8[1][(hi >> 16) & 0xff] ^ T8[0][hi >> 24];
        p += 8;
        n -= 8;
    }
    while (n--) c = T8[0][(c ^ *p++) & 0xff] ^ (c >> 8);
    return c;
}

uint32_t orc_crc32_clmul(const uint8_t *p, uint64_t n) {
    init_tables();
    uint32_t c = 0xFFFFFFFFu;
#if defined(__x86_64__)
    static int have = -1;
    if (have < 0) have = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
    if (have && n >= 64) {
        const uint64_t body = n & ~(uint64_t)15;
        c = clmul_fold(p, body, c);
        p += body;
        n -= body;
    }
#endif
    return ~slice8_update(c, p, n);
}

/* ------------------------------------------------------------- header --- */
/* core/header.go:9-16,58-62: 16-byte little-endian {CRC, Timestamp, KeySize,
 * ValueSize} read with binary.Read(r, LittleEndian, &h). */
static inline uint32_t le32(const uint8_t *p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
}

/* ------------------------------------------------------------- replay --- */
/* core/db.go:110-123 (init), 125-143 (walkFile), 145-178 (readEntry),
 * core/keydir.go:22-34 (set), 45-53 (unset/resetOffset).
 * EOF classes (Go stdlib):
 *   binary.Read -> io.ReadFull(16): 0 bytes io.EOF (clean stop), 1-15 bytes
 *   io.ErrUnexpectedEOF (walkFile returns "gocask: startup error").
 *   io.ReadFull(key): 0 bytes with len>0 -> io.EOF (clean stop), partial ->
 *   io.ErrUnexpectedEOF.  bufio.Reader.Discard(n) short -> io.EOF (clean stop,
 *   record not inserted).  A walk error aborts filepath.Walk, so later files
 *   are not replayed and resetOffset is not reached. */
int orc_replay(const orc_file *files, uint32_t nfiles, int verify_crc, orc_rec *out,
               uint64_t cap, orc_status *st) {
    uint32_t last = 0; /* keyDir.lastOffset (core/keydir.go:12) */
    uint64_t n = 0;
    memset(st, 0, sizeof(*st));
    for (uint32_t f = 0; f < nfiles; f++) {
        const uint8_t *d = files[f].data;
        const uint64_t len = files[f].len;
        uint64_t p = 0;
        st->files_walked = f + 1;
        for (;;) {
            uint64_t rem = len - p;
            if (rem == 0) break;                       /* io.EOF: clean      */
            if (rem < 16) {                            /* ErrUnexpectedEOF   */
                st->status = ORC_EUNEXPECTED_EOF;
                st->err_file = f;
                st->err_off = p;
                goto done;
            }
            const uint64_t rec = p;
            const uint32_t hcrc = le32(d + p), ts = le32(d + p + 4);
            const uint32_t ks = le32(d + p + 8), vs = le32(d + p + 12);
            p += 16;
            const int tomb = (ks == 0);                /* header.go:54-56    */
            const uint32_t klen = tomb ? vs : ks;      /* db.go:151-155      */
            rem = len - p;
            if (klen > 0 && rem == 0) break;           /* ReadFull -> io.EOF */
            if (rem < klen) {                          /* partial key        */
                st->status = ORC_EUNEXPECTED_EOF;
                st->err_file = f;
                st->err_off = rec;
                goto done;
            }
            p += klen;
            if (!tomb) {
                if (len - p < vs) break;               /* Discard -> io.EOF  */
                p += vs;
            }
            if (out && n < cap) {
                orc_rec *r = &out[n];
                r->rec_off = rec;
                r->file = f;
                r->key_len = klen;
                r->value_pos = last + 16u + ks;        /* keydir.go:25       */
                r->value_size = vs;
                r->crc = hcrc;
                r->ts = ts;
                r->flags = tomb ? ORC_F_TOMBSTONE : 0;
                r->crc_calc = 0;
                if (verify_crc) {                      /* db.go:311 rule     */
                    r->crc_calc = orc_crc32(d + p - vs, vs);
                    if (r->crc_calc == hcrc) r->flags |= ORC_F_CRC_OK;
                }
            }
            n++;
            if (tomb) last += 16u + klen;              /* keydir.go:48       */
            else last += 16u + ks + vs;                /* keydir.go:31       */
        }
        if (files[f].reset_after) last = 0;            /* db.go:117-119      */
    }
done:
    st->n_recs = n;
    st->final_last_offset = last;
    if (out && n > cap) return ORC_ECAPACITY;
    return st->status;
}

/* ----------------------------------------------------------- hash map --- */
/* keyDir.entries map[string]kdEntry (core/keydir.go:11-14).  Open addressing,
 * linear probing, backward-shift delete. */
typedef struct {
    uint64_t *slot; /* (idx+1) or 0 for empty */
    uint64_t *hash;
    uint64_t mask;
    const uint8_t **kp;
    uint32_t *kl;
} hmap;

static uint64_t hkey(const uint8_t *p, uint32_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ ((uint64_t)n * 0xff51afd7ed558ccdull);
    while (n >= 8) {
        uint64_t w;
        memcpy(&w, p, 8);
        h = (h ^ w) * 0xbf58476d1ce4e5b9ull;
        h ^= h >> 29;
        p += 8;
        n -= 8;
    }
    uint64_t w = 0;
    memcpy(&w, p, n);
    h = (h ^ w) * 0x94d049bb133111ebull;
    return h ^ (h >> 32);
}

static int hm_init(hmap *m, uint64_t n_keys) {
    uint64_t cap = 16;
    while (cap < n_keys * 2 + 16) cap <<= 1;
    m->mask = cap - 1;
    m->slot = calloc(cap, sizeof(uint64_t));
    m->hash = calloc(cap, sizeof(uint64_t));
    return m->slot && m->hash ? 0 : -1;
}
static void hm_free(hmap *m) { free(m->slot); free(m->hash); }

/* keyed by record index; key bytes looked up through kp/kl */
static inline int hm_eq(const hmap *m, uint64_t a, const uint8_t *p, uint32_t n) {
    return m->kl[a] == n && memcmp(m->kp[a], p, n) == 0;
}

/* returns 1 when idx's key was not in the map */
static int hm_set(hmap *m, uint64_t idx) {
    const uint8_t *p = m->kp[idx];
    uint32_t n = m->kl[idx];
    uint64_t h = hkey(p, n), i = h & m->mask;
    for (;;) {
        if (!m->slot[i]) { m->slot[i] = idx + 1; m->hash[i] = h; return 1; }
        if (m->hash[i] == h && hm_eq(m, m->slot[i] - 1, p, n)) { m->slot[i] = idx + 1; return 0; }
        i = (i + 1) & m->mask;
    }
}

/* double the slots (the timed baseline grows its map as Go's does) */
static int hm_grow(hmap *m) {
    const uint64_t ocap = m->mask + 1, cap = ocap * 2;
    uint64_t *slot = calloc(cap, sizeof(uint64_t)), *hash = calloc(cap, sizeof(uint64_t));
    if (!slot || !hash) { free(slot); free(hash); return -1; }
    for (uint64_t j = 0; j < ocap; j++) {
        if (!m->slot[j]) continue;
        uint64_t i = m->hash[j] & (cap - 1);
        while (slot[i]) i = (i + 1) & (cap - 1);
        slot[i] = m->slot[j];
        hash[i] = m->hash[j];
    }
    free(m->slot);
    free(m->hash);
    m->slot = slot;
    m->hash = hash;
    m->mask = cap - 1;
    return 0;
}

/* returns 1 when the key was present */
static int hm_del(hmap *m, const uint8_t *p, uint32_t n) {
    uint64_t h = hkey(p, n), i = h & m->mask;
    for (;;) {
        if (!m->slot[i]) return 0; /* delete of an absent key is a no-op */
        if (m->hash[i] == h && hm_eq(m, m->slot[i] - 1, p, n)) break;
        i = (i + 1) & m->mask;
    }
    uint64_t j = i;
    for (;;) { /* backward-shift deletion */
        j = (j + 1) & m->mask;
        if (!m->slot[j]) break;
        uint64_t home = m->hash[j] & m->mask;
        if (((j - home) & m->mask) >= ((j - i) & m->mask)) {
            m->slot[i] = m->slot[j];
            m->hash[i] = m->hash[j];
            i = j;
        }
    }
    m->slot[i] = 0;
    return 1;
}

static int cmp_u64(const void *a, const void *b) {
    uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
    return x < y ? -1 : x > y;
}

/* core/keydir.go:22-49: set overwrites (last writer wins), unset deletes. */
uint64_t orc_keydir(const orc_file *files, const orc_rec *recs, uint64_t n, uint64_t *live_out) {
    hmap m;
    if (hm_init(&m, n)) return 0;
    m.kp = malloc(sizeof(*m.kp) * (n ? n : 1));
    m.kl = malloc(sizeof(*m.kl) * (n ? n : 1));
    for (uint64_t r = 0; r < n; r++) {
        m.kp[r] = files[recs[r].file].data + recs[r].rec_off + 16;
        m.kl[r] = recs[r].key_len;
    }
    for (uint64_t r = 0; r < n; r++) {
        if (recs[r].flags & ORC_F_TOMBSTONE) hm_del(&m, m.kp[r], m.kl[r]);
        else hm_set(&m, r);
    }
    uint64_t k = 0;
    for (uint64_t i = 0; i <= m.mask; i++)
        if (m.slot[i]) live_out[k++] = m.slot[i] - 1;
    qsort(live_out, k, sizeof(uint64_t), cmp_u64);
    free(m.kp);
    free(m.kl);
    hm_free(&m);
    return k;
}

/* Timed CPU baseline: the same loop as orc_replay, but with the keydir map
 * update inline and no per-record output array (what the single-goroutine
 * reference does in core/db.go:131-140 + keydir.go:22-49). */
/* flags: 1 = CRC verdict per record; 2 = copy the key and value bytes
 * through a 4 KiB buffer, as walkFile's bufio.Reader (core/db.go:126) does
 * for ReadFull(key) and Discard(ValueSize). */
uint64_t orc_baseline(const orc_file *files, uint32_t nfiles, int flags, orc_status *st) {
    const int verify_crc = flags & 1, bufio = flags & 2;
    uint8_t buf[4096];
    uint64_t sink = 0;
    /* the map and the key arrays grow as the reference's map does (doubling),
     * instead of being sized for the worst case of 16-byte records */
    hmap m;
    uint64_t kcap = 1u << 16, keys = 0;
    if (hm_init(&m, kcap / 2)) return 0;
    m.kp = malloc(sizeof(*m.kp) * kcap);
    m.kl = malloc(sizeof(*m.kl) * kcap);
    uint32_t last = 0;
    uint64_t n = 0, bad = 0;
    memset(st, 0, sizeof(*st));
    for (uint32_t f = 0; f < nfiles; f++) {
        const uint8_t *d = files[f].data;
        const uint64_t len = files[f].len;
        uint64_t p = 0;
        for (;;) {
            uint64_t rem = len - p;
            if (rem == 0) break;
            if (rem < 16) { st->status = ORC_EUNEXPECTED_EOF; goto out; }
            const uint32_t hcrc = le32(d + p), ks = le32(d + p + 8), vs = le32(d + p + 12);
            p += 16;
            const int tomb = ks == 0;
            const uint32_t klen = tomb ? vs : ks;
            rem = len - p;
            if (klen > 0 && rem == 0) break;
            if (rem < klen) { st->status = ORC_EUNEXPECTED_EOF; goto out; }
            const uint8_t *key = d + p;
            p += klen;
            if (bufio) { /* the record's bytes through the reader's buffer */
                const uint64_t e = tomb ? p : (len - p < vs ? len : p + vs);
                for (uint64_t q = p - klen - 16; q < e; q += sizeof buf) {
                    const uint64_t k = e - q < sizeof buf ? e - q : sizeof buf;
                    memcpy(buf, d + q, k);
                    sink += buf[k - 1];
                }
            }
            if (tomb) {
                keys -= (uint64_t)hm_del(&m, key, klen);
                last += 16u + klen;
            } else {
                if (len - p < vs) break;
                p += vs;
                if (n >= kcap) {
                    kcap *= 2;
                    m.kp = realloc(m.kp, sizeof(*m.kp) * kcap);
                    m.kl = realloc(m.kl, sizeof(*m.kl) * kcap);
                    if (!m.kp || !m.kl) { st->status = -1; goto out; }
                }
                m.kp[n] = key;
                m.kl[n] = klen;
                keys += (uint64_t)hm_set(&m, n);
                if (keys * 2 > m.mask + 1 && hm_grow(&m)) { st->status = -1; goto out; }
                last += 16u + ks + vs;
            }
            if (verify_crc && orc_crc32_clmul(d + p - vs, vs) != hcrc) bad++;
            n++;
        }
        if (files[f].reset_after) last = 0;
    }
out:
    st->n_recs = n;
    st->final_last_offset = last;
    uint64_t live = 0;
    for (uint64_t i = 0; i <= m.mask; i++) live += m.slot[i] != 0;
    st->err_off = bad; /* baseline: number of CRC rejects (diagnostic) */
    st->err_file = (uint32_t)sink; /* keeps the buffered copies live */
    free(m.kp);
    free(m.kl);
    hm_free(&m);
    return live;
}

/* ------------------------------------------------------------- corpus --- */
/* This repo's synthetic corpus spec (DESIGN.md "Corpus").  Records are
 * serialized exactly as core/db.go:257-284 (serializeEntry) and
 * core/testutil/utils.go:10-19 (Entry) do: header || key || value, CRC over
 * the value (core/header.go:18-28); a Delete writes header{CRC(key), t, 0,
 * len(key)} || key (core/db.go:245-247).  Files rotate when
 * size + entrySize > MaxDataFileSize (core/db.go:214-232). */
static inline uint64_t mix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
static inline uint64_t H(uint64_t seed, uint64_t tag, uint64_t i) {
    return mix64(mix64(seed ^ (tag * 0xD6E8FEB86659FD93ull)) + i);
}

#define ZIPF_N 65473u
static uint32_t zipf_thr[ZIPF_N - 1];
static int zipf_ready = 0;

void orc_zipf_table(uint32_t *thr) {
    if (!zipf_ready) {
        double *cum = malloc(sizeof(double) * ZIPF_N);
        double acc = 0.0;
        for (uint32_t r = 1; r <= ZIPF_N; r++) {
            acc += pow((double)r, -1.1);
            cum[r - 1] = acc;
        }
        for (uint32_t k = 0; k + 1 < ZIPF_N; k++) {
            double v = floor(cum[k] / acc * 4294967296.0);
            zipf_thr[k] = v >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)v;
        }
        free(cum);
        zipf_ready = 1;
    }
    if (thr) memcpy(thr, zipf_thr, sizeof(zipf_thr));
}

static uint32_t zipf_sample(uint32_t u) {
    /* r = 1 + #{k : thr[k] <= u} */
    uint32_t lo = 0, hi = ZIPF_N - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi) / 2;
        if (zipf_thr[mid] <= u) lo = mid + 1;
        else hi = mid;
    }
    return 1 + lo;
}

typedef struct {
    int tomb;
    uint64_t keyid;
    uint32_t klen, vlen;
    uint64_t entry;
} op_t;

static uint64_t kseed(const orc_corpus_cfg *c) { return c->key_seed ? c->key_seed : c->seed; }

static void op_describe(const orc_corpus_cfg *c, uint64_t i, op_t *o) {
    const uint64_t kidx = c->key_seed ? ((uint64_t)c->key_file << 32 | i) : i;
    o->tomb = c->tomb_permille && (H(c->seed, 3, i) % 1000u) < c->tomb_permille;
    o->keyid = c->key_universe ? H(kseed(c), 1, kidx) % c->key_universe : kidx;
    o->klen = c->key_min + (c->key_max > c->key_min
                                ? (uint32_t)(H(kseed(c), 6, o->keyid) % (c->key_max - c->key_min + 1))
                                : 0);
    if (o->tomb) o->vlen = o->klen;
    else o->vlen = c->val_fixed ? c->val_fixed : 63u + zipf_sample((uint32_t)(H(c->seed, 2, i) >> 32));
    o->entry = 16ull + (o->tomb ? 0 : o->klen) + o->vlen;
}

static void key_bytes(const orc_corpus_cfg *c, uint64_t keyid, uint32_t klen, uint8_t *k) {
    uint64_t w0 = mix64(keyid ^ H(kseed(c), 7, 0));
    for (uint32_t j = 0; j < klen; j++) {
        uint64_t w = j < 8 ? w0 : H(kseed(c), 8, keyid * 64 + j / 8);
        k[j] = (uint8_t)(w >> (8 * (j % 8)));
    }
}

static void put32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)v; p[1] = (uint8_t)(v >> 8); p[2] = (uint8_t)(v >> 16); p[3] = (uint8_t)(v >> 24);
}

/* Walk ops in order, applying the rotation rule; calls back per op. */
static int plan(const orc_corpus_cfg *c, uint64_t *file_sizes, uint32_t max_files,
                uint32_t *n_files, uint64_t *n_ops, uint8_t *const *bufs) {
    orc_zipf_table(NULL);
    uint32_t cur = 0;
    uint64_t size = 0, i = 0;
    uint8_t kb[512];
    if (c->key_min < 8 || c->key_max > 512 || c->key_max < c->key_min) return -1;
    if (!c->n_ops && !c->n_files) return -1;
    for (;; i++) {
        if (c->n_ops && i >= c->n_ops) break;
        op_t o;
        op_describe(c, i, &o);
        if (size + o.entry > c->max_file_size) {
            if (c->n_files && cur + 1 >= c->n_files) break;
            if (file_sizes && cur < max_files) file_sizes[cur] = size;
            cur++;
            size = 0;
            if (cur >= max_files) return -2;
        }
        if (bufs) {
            uint8_t *p = bufs[cur] + size;
            uint32_t ts = c->ts_base + (uint32_t)i;
            key_bytes(c, o.keyid, o.klen, kb);
            if (o.tomb) {
                put32(p, orc_crc32(kb, o.klen));
                put32(p + 4, ts);
                put32(p + 8, 0);
                put32(p + 12, o.klen);
                memcpy(p + 16, kb, o.klen);
            } else {
                uint8_t *v = p + 16 + o.klen;
                for (uint32_t j = 0; j < o.vlen; j += 8) {
                    uint64_t w = H(c->seed, 5, (i << 20) | (j / 8));
                    for (uint32_t b = 0; b < 8 && j + b < o.vlen; b++) v[j + b] = (uint8_t)(w >> (8 * b));
                }
                put32(p, orc_crc32(v, o.vlen));
                put32(p + 4, ts);
                put32(p + 8, o.klen);
                put32(p + 12, o.vlen);
                memcpy(p + 16, kb, o.klen);
                if (c->flip_permille && o.vlen && (H(c->seed, 4, i) % 1000u) < c->flip_permille) {
                    uint64_t bit = H(c->seed, 9, i) % (8ull * o.vlen);
                    v[bit / 8] ^= (uint8_t)(1u << (bit % 8));
                }
            }
        }
        size += o.entry;
    }
    if (file_sizes && cur < max_files) file_sizes[cur] = size;
    if (n_files) *n_files = cur + 1;
    if (n_ops) *n_ops = i;
    return 0;
}

int orc_gen_sizes(const orc_corpus_cfg *cfg, uint64_t *n_ops, uint64_t *file_sizes,
                  uint32_t max_files, uint32_t *n_files) {
    return plan(cfg, file_sizes, max_files, n_files, n_ops, NULL);
}

int orc_gen_fill(const orc_corpus_cfg *cfg, uint8_t *const *file_bufs, uint32_t n_files) {
    return plan(cfg, NULL, n_files, NULL, NULL, file_bufs);
}
