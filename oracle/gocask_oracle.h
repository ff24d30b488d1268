/*
 * gocask_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's cold-start replay path
 * (aneshas/gocask: core/db.go:110-178, core/keydir.go:22-53, core/header.go:9-62,
 * internal/crc/crc.go:5-10) plus an independent CPU implementation of this
 * repo's synthetic corpus spec.  It is the CHECKER: only tests/, the
 * __graft_entry__.smoke() check and bench.py's cpu_baseline leg may load it.
 * The product library (gocask_amd/libgocask_hip.so) never links or calls it.
 *
 * Pinning: the Go toolchain is absent here, so the reference cannot be run.
 * The restatement is pinned against (a) the known answers of the reference's
 * own replay tests (core/db_test.go:140-500, db_test.go:39-74), committed as
 * fixtures under tests/golden/, and (b) the published CRC-32/IEEE check value
 * crc32("123456789") = 0xCBF43926 that Go's hash/crc32 (the algorithm behind
 * internal/crc/crc.go:9) is specified to produce.  See DESIGN.md "Oracle".
 */
#ifndef GOCASK_ORACLE_H
#define GOCASK_ORACLE_H
#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One data file in walk order (internal/fs/disk.go:122-145).  reset_after
 * mirrors `file.Name() != activeFile.Name()` (core/db.go:117). */
typedef struct {
    const uint8_t *data;
    uint64_t len;
    uint8_t reset_after;
} orc_file;

/* Record tuple; byte-identical layout to gck_rec in include/gocask_hip.h. */
typedef struct {
    uint64_t rec_off;    /* header offset within its file                      */
    uint32_t file;       /* index into the files[] array (walk order)          */
    uint32_t key_len;    /* KeySize, or ValueSize for a tombstone              */
    uint32_t value_pos;  /* kdEntry.ValuePos, u32 wrap (core/keydir.go:25)      */
    uint32_t value_size; /* header ValueSize                                   */
    uint32_t crc;        /* header CRC (kdEntry.CRC)                           */
    uint32_t ts;         /* header Timestamp                                   */
    uint32_t flags;      /* ORC_F_TOMBSTONE | ORC_F_CRC_OK                      */
    uint32_t crc_calc;   /* CRC-32/IEEE of the record's last ValueSize bytes   */
} orc_rec;

#define ORC_F_TOMBSTONE 1u
#define ORC_F_CRC_OK 2u

enum { ORC_OK = 0, ORC_EUNEXPECTED_EOF = 1, ORC_ECAPACITY = 2 };

typedef struct {
    int32_t status;            /* ORC_OK or ORC_EUNEXPECTED_EOF               */
    uint32_t err_file;         /* file index of the startup error             */
    uint64_t err_off;          /* offset of the record that failed            */
    uint64_t n_recs;           /* records emitted (walk order)                */
    uint32_t final_last_offset;/* keyDir.lastOffset after replay              */
    uint32_t files_walked;     /* files fully or partially walked             */
} orc_status;

/* CRC-32/IEEE (internal/crc/crc.go:8-10 -> Go hash/crc32 IEEE). */
uint32_t orc_crc32(const uint8_t *p, uint64_t n);
/* Same result, slicing-by-8 (used by the timed CPU baseline). */
uint32_t orc_crc32_fast(const uint8_t *p, uint64_t n);
/* Go's amd64 speed class: PCLMULQDQ folding for >= 64 bytes (cpu baseline). */
uint32_t orc_crc32_clmul(const uint8_t *p, uint64_t n);

/* Replay the files in walk order.  verify_crc computes the per-record verdict
 * (the core/db.go:311 rule applied to every record).  out may be NULL to only
 * count.  Returns status code. */
int orc_replay(const orc_file *files, uint32_t nfiles, int verify_crc,
               orc_rec *out, uint64_t cap, orc_status *st);

/* Keydir after replay: last-writer-wins in walk order, tombstones delete
 * (core/keydir.go:22-49).  Writes the indices (into recs) of the live entries
 * in ascending order; returns their count. */
uint64_t orc_keydir(const orc_file *files, const orc_rec *recs, uint64_t n,
                    uint64_t *live_out);

/* Faithful timed CPU baseline: replay + hash-map keydir, the way the
 * single-goroutine reference does it (one pass, map insert per record, the
 * map grown by doubling).  flags: 1 = CRC verdict per record, 2 = every
 * record byte through a 4 KiB buffer (the reference's bufio.Reader).
 * Returns number of live keys. */
uint64_t orc_baseline(const orc_file *files, uint32_t nfiles, int flags, orc_status *st);

/* ------------------------------------------------------------------------
 * Synthetic corpus spec (see DESIGN.md "Corpus").  Independent CPU
 * implementation used to cross-check the product's device encoder.
 * ---------------------------------------------------------------------- */
typedef struct {
    uint64_t seed;
    uint64_t max_file_size;   /* rotation threshold (core/db.go:214-232)     */
    uint64_t n_ops;           /* stop after n ops (0: use n_files)            */
    uint32_t n_files;         /* stop when this many files are full          */
    uint32_t key_min, key_max;/* key length range (>= 8)                     */
    uint64_t key_universe;    /* 0: unique keys                               */
    uint32_t val_fixed;       /* >0 fixed value size, 0 = bounded Zipf(1.1)   */
    uint32_t tomb_permille;
    uint32_t flip_permille;
    uint32_t ts_base;
    uint64_t key_seed;        /* 0: keys from seed; else key ids / lengths /  */
                              /* bytes from key_seed, op i drawing key id     */
                              /* H(key_seed, 1, key_file << 32 | i)           */
    uint32_t key_file;        /* the file id of a per-file corpus (C4)        */
    uint32_t pad_;
} orc_corpus_cfg;

/* Dry run: number of ops and per-file sizes (creation order). */
int orc_gen_sizes(const orc_corpus_cfg *cfg, uint64_t *n_ops, uint64_t *file_sizes,
                  uint32_t max_files, uint32_t *n_files);
/* Fill file buffers (creation order), sized by orc_gen_sizes. */
int orc_gen_fill(const orc_corpus_cfg *cfg, uint8_t *const *file_bufs, uint32_t n_files);
/* The Zipf threshold table (65472 entries) so tests can compare encoders. */
void orc_zipf_table(uint32_t *thr);

#ifdef __cplusplus
}
#endif
#endif
