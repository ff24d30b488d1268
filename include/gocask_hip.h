/*
 * gocask_hip.h — C-ABI of libgocask_hip.so, the MI355X-native replacement for
 * aneshas/gocask's cold-start log replay.
 *
 * What it replaces (reference file:line):
 *   - gck_replay / gck_ctx_*  replace the body of the unexported
 *     (*DB).init(activeFile File) (core/db.go:110-123) together with
 *     walkFile/readEntry (core/db.go:125-178), keyDir.set/unset/resetOffset
 *     (core/keydir.go:22-53) and, per record, the crc.CalcCRC32 check that
 *     (*DB).get applies lazily (core/db.go:304-313, internal/crc/crc.go:8-10).
 *   - gck_db_*  mirror the public surface that sits on top of that seam:
 *     core.NewDB (core/db.go:90-108) / gocask.Open (db.go:29-59) with the Disk
 *     and InMemory file systems (internal/fs/disk.go:50-145,
 *     internal/fs/memory.go:46-80), DB.Get (core/db.go:287-316) and DB.Keys
 *     (core/db.go:318-324).
 *   - gck_encode_* is the device-side record encoder (serializeEntry,
 *     core/db.go:272-284, core/header.go:18-48) used for bulk corpus builds.
 *
 * Plain pointers and sizes only; no framework types cross this boundary.  The
 * Go-side cgo binding a maintainer would add is shown in INTEGRATION.md.
 *
 * Errors never fall back to a CPU path: without a usable gfx950 device every
 * compute entry point returns GCK_EDEVICE.
 */
#ifndef GOCASK_HIP_H
#define GOCASK_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes --------------------------------------------------------- */
enum {
    GCK_OK = 0,
    GCK_EUNEXPECTED_EOF = 1, /* "gocask: startup error: unexpected EOF" (core/db.go:138)   */
    GCK_EDEVICE = 2,         /* no gfx950 device / HIP runtime failure                       */
    GCK_EINVAL = 3,          /* bad argument                                                 */
    GCK_ENOMEM = 4,          /* device or host allocation failed                             */
    GCK_EIO = 5,             /* file system error (open/stat/mmap/readdir)                   */
    GCK_EKEY_NOT_FOUND = 6,  /* core.ErrKeyNotFound (core/db.go:17)                          */
    GCK_ECRC_FAILED = 7,     /* core.ErrCRCFailed (core/db.go:24)                            */
    GCK_EINVALID_KEY = 8,    /* core.ErrInvalidKey (core/db.go:27)                           */
    GCK_ENOT_DIR = 9         /* "file exists and it's not a folder" (internal/fs/disk.go:116) */
};

/* ---- replay input / output ---------------------------------------------- */

/* One data file, in FS.Walk order (internal/fs/disk.go:122-145).  data must stay
 * valid for the whole call (mmap'd or host memory).  reset_after mirrors
 * `file.Name() != activeFile.Name()` (core/db.go:117): 1 = lastOffset resets to 0
 * after this file. */
typedef struct gck_file {
    const uint8_t *data;
    uint64_t len;
    uint8_t reset_after;
} gck_file;

#define GCK_F_TOMBSTONE 1u /* header KeySize == 0 (core/header.go:54-56)              */
#define GCK_F_CRC_OK 2u    /* CRC-32/IEEE(last ValueSize bytes) == header CRC           */
#define GCK_F_HINT 4u      /* from a hint file (gck_ctx_replay_hints): value not read   */

/* One record per header decoded, in walk order (superseded records and tombstones
 * included).  40 bytes, no padding. */
typedef struct gck_rec {
    uint64_t rec_off;    /* header offset within its file                                  */
    uint32_t file;       /* index into files[] (walk order); kdEntry.File = its Name()      */
    uint32_t key_len;    /* KeySize, or ValueSize for a tombstone (core/db.go:151-155)     */
    uint32_t value_pos;  /* kdEntry.ValuePos = lastOffset + 16 + KeySize mod 2^32          */
    uint32_t value_size; /* header ValueSize (kdEntry.ValueSize)                           */
    uint32_t crc;        /* header CRC (kdEntry.CRC)                                       */
    uint32_t ts;         /* header Timestamp (kdEntry.Timestamp)                           */
    uint32_t flags;      /* GCK_F_*                                                        */
    uint32_t crc_calc;   /* CRC-32/IEEE of the record's last ValueSize bytes               */
} gck_rec;

/* gck_opts.flags: gck_replay / gck_replay_into / gck_replay_paths also return
 * the records' key bytes (gck_result.keys), so a caller that never maps the
 * files (gck_replay_paths) can fill its keydir map. */
#define GCK_OPT_KEYS 1u
/* gck_opts.flags: gck_replay / gck_replay_into / gck_replay_paths return the
 * live keydir instead of every record (SURVEY.md §8f f1 on the one-GPU drop-in
 * path; replaces applying every record with keyDir.set / unset,
 * core/keydir.go:22-49): one gck_rec per live key -- its last record in walk
 * order, a Put (a key whose last record is a Delete is absent) -- with
 * rec.file the walk index; with GCK_OPT_KEYS the live keys' bytes in the
 * order of the records.  Each file group's keydir is built on the device as
 * the group replays and the groups are merged there in walk order (the
 * one-device form of gck_replay_multi, no RCCL), so only live entries cross
 * PCIe and the caller's map takes one insert per live key.  status, err_*,
 * files_walked, final_last_offset and n_crc_fail (rejects among all replayed
 * records) as without the flag. */
#define GCK_OPT_LIVE 2u

/* Tuning knobs; zero fields take the defaults.  Results never depend on them
 * (GCK_OPT_KEYS adds an output). */
typedef struct gck_opts {
    int32_t device;        /* HIP device ordinal (default 0)                               */
    uint32_t chunk_bytes;  /* boundary-speculation chunk (pow2 >= 4 KiB; default 512 KiB)  */
    uint32_t max_key;      /* speculation plausibility bound on key length (default 64K)  */
    uint32_t chunk_cap;    /* records staged per chunk before a re-walk (default 1024)    */
    uint32_t flags;        /* GCK_OPT_*                                                    */
    uint32_t spec_window;  /* bytes from a chunk's start searched for its first record    */
                           /* (rounded up to 4 KiB; default 0 = the whole chunk).  A      */
                           /* chunk whose first record lies further in is covered by the  */
                           /* walk of the chunk before it.                                 */
    uint64_t max_resident; /* gck_replay / gck_replay_into: data-file bytes resident on   */
                           /* the device at once (0 = 60 % of free device memory); a     */
                           /* larger database streams through a ring of file groups      */
} gck_opts;

typedef struct gck_result {
    gck_rec *recs;              /* library-owned host array; free with gck_result_free  */
    uint64_t n;                 /* records in recs                                      */
    uint64_t n_crc_fail;        /* records whose verdict is a reject                    */
    uint32_t final_last_offset; /* keyDir.lastOffset after replay (later Puts use it)   */
    int32_t status;             /* GCK_OK or GCK_EUNEXPECTED_EOF                        */
    uint32_t err_file;          /* file index of the startup error                      */
    uint32_t files_walked;      /* files the reference would have walked                */
    uint64_t err_off;           /* header offset of the record that hit the error       */
    uint32_t n_groups;          /* gck_replay*: file groups the files were cut into     */
    uint32_t n_resident;        /* gck_replay*: groups resident at once (the ring)      */
    uint8_t *keys;              /* GCK_OPT_KEYS: the records' key bytes back to back in */
    uint64_t keys_len;          /* record order (record i's key_len bytes); freed by    */
                                /* gck_result_free (gck_replay_into callers too)        */
} gck_result;

/* One-shot host-in/host-out replay: H2D, device pipeline, D2H.  Pipelined over
 * groups of files (about a quarter of the database, >= 1 GiB, or a third of
 * opts->max_resident; cut after files that reset lastOffset): each group
 * replays as soon as its own files are resident, while later groups still
 * cross PCIe.  Registered memory (gck_host_register) goes by DMA as is; other
 * memory is staged by the library's host threads through page-locked buffers
 * (no registration needed).  A ring of groups bounds the device
 * memory (opts->max_resident): a database larger than it streams through.
 * Results are those of one replay of all files in walk order.  GCK_ENOMEM:
 * the device could not hold even one group (a caller may fall back to the CPU
 * path, as for GCK_EDEVICE). */
int gck_replay(const gck_file *files, uint32_t nfiles, const gck_opts *opts, gck_result *out);
/* The same, tuples into caller memory dst (cap records; pin it for DMA rate);
 * out->recs = NULL.  Each group's tuples leave as soon as it has replayed.
 * GCK_EINVAL (out->n = records needed, dst contents unspecified) when
 * cap < out->n. */
int gck_replay_into(const gck_file *files, uint32_t nfiles, const gck_opts *opts, gck_rec *dst, uint64_t cap,
                    gck_result *out);
/* A data file by name (filepath.Walk's path) for gck_replay_paths. */
typedef struct gck_path {
    const char *path;
    uint8_t reset_after; /* Name() != activeFile.Name() (core/db.go:117) */
} gck_path;
/* gck_replay of files named by path: the library opens them, reads them with
 * pread into page-locked staging buffers (host threads, GCK_COPY_THREADS) and
 * streams them to the device, so nothing has to be mapped or registered;
 * GCK_EIO when a file cannot be opened or read. */
int gck_replay_paths(const gck_path *files, uint32_t nfiles, const gck_opts *opts, gck_result *out);
void gck_result_free(gck_result *res);
/* gck_replay / gck_replay_into keep their device contexts (arenas, tables) for
 * the next call with the same options, so a repeated Open allocates nothing;
 * this frees them (call it when no replay will follow, or to return HBM). */
void gck_replay_release_cache(void);

/* ---- device-resident context (benchmarks, repeated replays) ---------------- */
typedef struct gck_ctx gck_ctx;

typedef struct gck_stats {
    uint64_t bytes;         /* data-file bytes replayed                               */
    uint64_t n_recs;        /* records decoded                                         */
    uint64_t n_crc_fail;    /* verdict rejects                                         */
    uint64_t n_chunks;      /* speculation chunks                                      */
    uint64_t n_fixups;      /* chunks whose speculative entry was wrong (re-walked)   */
    uint64_t n_overflow;    /* chunks whose records exceeded chunk_cap (re-walked)    */
    double ms_total;        /* last gck_ctx_run wall time (host clock)                */
    double ms_kernel[12];   /* per-phase device time (HIP events), see gck_phase_name; */
                            /* a device-path run (no host round trip) times only the */
                            /* CRC pass unless gck_ctx_phase_timing is on (the other */
                            /* phases and "pipeline" are 0); a host-path run all     */
    uint32_t device_path;   /* 1: the last run had no host round trip (record table sized by an earlier run) */
    uint32_t n_reruns;      /* device-only runs redone on the host path (capacity / unsettled speculation)  */
    /* the last run's outcome, as gck_result reports it (no records copied):   */
    int32_t status;              /* GCK_OK or GCK_EUNEXPECTED_EOF                 */
    uint32_t err_file;           /* file index of the startup error               */
    uint64_t err_off;            /* header offset of the record that hit it       */
    uint32_t files_walked;       /* files the reference would have walked         */
    uint32_t final_last_offset;  /* keyDir.lastOffset after replay                */
    uint32_t n_files;            /* files in the arena                            */
    uint32_t kd_longest_probe;   /* last keydir build: its longest table probe past 256 (0: none) */
    uint64_t n_runs;             /* runs of this context so far                   */
    double ms_crc_rows_sum;      /* k_crc_rows time (HIP events) summed over them */
} gck_stats;

int gck_ctx_create(const gck_opts *opts, gck_ctx **out);
void gck_ctx_destroy(gck_ctx *ctx);
/* Copy files into the device arena (H2D). */
int gck_ctx_load(gck_ctx *ctx, const gck_file *files, uint32_t nfiles);
/* Run the device pipeline on the resident arena.  Blocks until done. */
int gck_ctx_run(gck_ctx *ctx);
/* Events between every phase of the next runs (on) or only around the CRC pass
 * and the whole run (off, the default: each event costs ~6 us of a run). */
int gck_ctx_phase_timing(gck_ctx *ctx, int on);
/* Copy the tuples of the last run to host memory. */
int gck_ctx_fetch(gck_ctx *ctx, gck_result *out);
/* Copy the tuples of the last run into caller memory (dst holds cap records;
 * register it with gck_host_register for DMA rate); *n = records of the run.
 * GCK_EINVAL (and nothing copied) when cap < *n. */
int gck_ctx_fetch_into(gck_ctx *ctx, gck_rec *dst, uint64_t cap, uint64_t *n);

/* Device keydir of the last run (replaces applying every
 * record with keyDir.set / unset, core/keydir.go:22-49): for every key its
 * last record in walk order, kept if it is a Put (with GCK_KD_KEEP_TOMBSTONES
 * tombstones are kept too, as delete markers for a merge across shards).
 * *n_live = the entries; *ms (optional) = device time.  The entries, in walk
 * order of their records, are fetched with gck_ctx_fetch_keydir; a Go caller
 * sets db.kd.entries[key] for each (key bytes at rec_off + 16 in the file).
 * GCK_EINVAL for a run of 2^31 records or more (the table's record index is
 * 31 bits); GCK_EDEVICE if keys keep finding no free slot within 256 probes
 * after the table was rebuilt for every record distinct (a hash flood). */
#define GCK_KD_KEEP_TOMBSTONES 1u
int gck_ctx_keydir(gck_ctx *ctx, uint32_t flags, uint64_t *n_live, double *ms);
/* on: the next runs also hash every record's key in their finalize pass (the
 * key bytes are in registers there) and insert the record into the keydir
 * table, so gck_ctx_keydir only marks the winners and compacts them; off (the
 * default) for runs that build no keydir.  gck_replay* with GCK_OPT_LIVE and
 * gck_replay_multi* turn it on for their groups.  A second gck_ctx_keydir of
 * the same run (either way) reuses the table. */
int gck_ctx_keydir_hash(gck_ctx *ctx, int on);
int gck_ctx_fetch_keydir(gck_ctx *ctx, gck_rec *dst, uint64_t cap, uint64_t *n);

/* ---- merge (compaction) and hint files ------------------
 * The reference lists "merging and hint files" as future work (README.md:60);
 * this is the device form of that roadmap item.  After gck_ctx_keydir (without
 * GCK_KD_KEEP_TOMBSTONES: a merge keeps live Puts only), the live records in
 * walk order are written as new data files exactly as DB.Put would write them
 * into a fresh database with MaxDataFileSize = max_file_size (an entry that does
 * not fit rotates first, core/db.go:214-231; a first record larger than the
 * limit leaves the first file empty), each record's bytes verbatim (header,
 * key, value: CRCs and timestamps unchanged).  One hint file per data file
 * (format invented here, parity unpinned: the reference has no hint files),
 * little-endian:
 *   entries [Timestamp u32][KeySize u32][ValueSize u32][ValuePos u32][CRC u32][key bytes]
 *   index   [hint-file offset u64][data-file offset u64][check u64] of entries
 *           0, B, 2B, ... (B = GCK_HINT_BLOCK); check = the XOR over the
 *           block's entries of a 64-bit mix of each entry's header words and
 *           key (gck_internal.h hint_entry_check): a reader refuses a block
 *           whose entries do not give it
 *   tail    [entries u64][entry bytes u64][data-file bytes u64][GCK_HINT_MAGIC u32]
 *           [GCK_HINT_VERSION u32]
 * (ValuePos = the value's offset in its merged file mod 2^32, as
 * core/keydir.go:25 sets it on a replay of the merged files; CRC = the
 * record header's, kdEntry.CRC), so gck_replay_hints fills the keydir without
 * reading the data files, in parallel over the index's blocks.  The outputs stay
 * on the device: *n_files, *data_bytes (all files back to back), *hint_bytes;
 * gck_ctx_fetch_compact copies them and the per-file sizes out (any pointer
 * may be NULL).  *ms (optional) = device time. */
#define GCK_HINT_BLOCK 16u
#define GCK_HINT_MAGIC 0x484B4347u /* "GCKH" */
#define GCK_HINT_VERSION 3u
int gck_ctx_compact(gck_ctx *ctx, uint64_t max_file_size, uint32_t *n_files, uint64_t *data_bytes,
                    uint64_t *hint_bytes, double *ms);
int gck_ctx_fetch_compact(gck_ctx *ctx, uint8_t *data, uint64_t *file_sizes, uint8_t *hints, uint64_t *hint_sizes);

/* Hint-driven replay (row f4; the reference's roadmap "hint files",
 * README.md:60): the tuples of a database whose data files all have hint files
 * (gck_ctx_compact's), from the hints alone -- no data-file byte is read.
 * The context's arena holds the hint files (gck_ctx_load, in walk order, each
 * with its data file's reset_after); afterwards the context's tuples are one
 * gck_rec per hint entry in walk order, each equal to the one gck_ctx_run
 * gives for that record on the data files (rec_off, file, key_len, value_pos
 * with the carried lastOffset, value_size, crc, ts) except flags = GCK_F_HINT
 * and crc_calc = 0 (the value is not read, so there is no CRC verdict), with
 * status GCK_OK, files_walked and final_last_offset as a replay; gck_ctx_fetch,
 * gck_ctx_keydir (last entry per key across several merges' hints) and the
 * rest work on them as on a run's.  GCK_EINVAL when a hint file is malformed
 * (tail, index and entries must agree).  *ms (optional) = device time. */
int gck_ctx_replay_hints(gck_ctx *ctx, double *ms);
/* One-shot form (host hint files in, tuples out, as gck_replay; GCK_OPT_KEYS
 * returns the key bytes, GCK_OPT_LIVE the keydir: last entry per key). */
int gck_replay_hints(const gck_file *files, uint32_t nfiles, const gck_opts *opts, gck_result *out);

/* ---- batched Get / keydir scrub -------------------------
 * DB.Get (core/db.go:287-316) for n keys against the device keydir of the last
 * run (call gck_ctx_keydir first, any flags): keys[key_off[i], key_off[i+1]) is
 * key i.  Per key: status[i] = GCK_OK, GCK_EINVALID_KEY (empty key),
 * GCK_EKEY_NOT_FOUND (absent or deleted), GCK_EIO (ValuePos + ValueSize past the
 * end of the entry's file: Disk.ReadFileAt's short read) or GCK_ECRC_FAILED;
 * value_size[i] = the entry's ValueSize; crc_calc[i] = CRC-32/IEEE recomputed
 * on the device from the resident file bytes at (File, ValuePos).  With values
 * != NULL the values of the GCK_OK keys are copied back to back, val_off[i]
 * their offsets (UINT64_MAX for the others); GCK_EINVAL if they exceed
 * values_cap (status / value_size are then filled, for a retry).
 * File resolution: the device reads the value from the walked file the entry's
 * record came from (its index in walk order).  Disk.ReadFileAt opens
 * <path>/<Name()>.csk instead (internal/fs/disk.go:147-148), which is the same
 * file for every .csk directly in the DB directory (the layout Disk writes);
 * for a .csk nested in a subdirectory (Disk.Walk recurses, disk.go:122-145) the
 * reference would read the top-level file of that name, or fail: not mirrored
 * here.  gck_db_get (the host mirror) opens by name as the reference does. */
int gck_ctx_get_batch(gck_ctx *ctx, const uint8_t *keys, const uint64_t *key_off, uint32_t n, int32_t *status,
                      uint32_t *value_size, uint32_t *crc_calc, uint8_t *values, uint64_t values_cap,
                      uint64_t *val_off, double *ms);
/* Integrity scrub: Get of every live keydir entry (gck_ctx_keydir order);
 * status / crc_calc (optional, n_live each) as above; *n_bad = entries not OK. */
int gck_ctx_scrub_keydir(gck_ctx *ctx, int32_t *status, uint32_t *crc_calc, uint64_t *n_bad, double *ms);

/* ---- keydir merge across shards ----------------------------
 * Files shard over GPUs in walk order: shard s holds a contiguous run of files,
 * every one but the last shard's last file with reset_after = 1, so each shard
 * replays on its own.  The merged keydir equals the one keyDir.set / unset
 * (core/keydir.go:22-49) would build over all files in walk order:
 *   1. every shard: gck_ctx_run, then gck_ctx_keydir(GCK_KD_KEEP_TOMBSTONES)
 *      (a shard's last word on a key may be a delete that hides an earlier
 *      shard's Put);
 *   2. gck_kd_pack_sizes / gck_kd_pack: the shard's entries as gck_kd_entry
 *      records plus a key blob, partitioned by key hash over nparts owners
 *      (partition-major, walk order within a partition);
 *   3. the caller exchanges partitions (all-to-all, e.g. RCCL over xGMI), each
 *      owner concatenating what it receives in shard order;
 *   4. gck_kd_merge on the owner: per key, the entry of the highest shard wins;
 *      a winning tombstone drops the key.  gck_kd_fetch_merged copies the
 *      owner's live entries (shard order, then walk order) and their keys.
 * The partition of a key is (hash >> 40) % nparts on every shard. */
typedef struct gck_kd_entry {
    uint64_t hash;    /* 64-bit hash of the key bytes                                */
    uint64_t key_off; /* offset of the key in its blob (8-byte aligned, zero padded) */
    uint32_t key_len; /* key bytes                                                   */
    uint32_t shard;   /* shard that wrote the entry                                  */
    gck_rec rec;      /* the record; rec.file is global (file_base + walk index)     */
} gck_kd_entry;       /* 64 bytes */

/* After gck_ctx_keydir: partition the keydir entries over nparts (1..64)
 * owners; counts[p] entries and key_bytes[p] blob bytes go to owner p. */
int gck_kd_pack_sizes(gck_ctx *ctx, uint32_t nparts, uint64_t *counts, uint64_t *key_bytes);
/* Fill DEVICE buffers: entries (>= sum counts) partition-major, keys (>= sum
 * key_bytes) partition-major; key_off is relative to the partition's blob. */
int gck_kd_pack(gck_ctx *ctx, uint32_t shard, uint32_t file_base, gck_kd_entry *d_entries, uint64_t entries_cap,
                uint8_t *d_keys, uint64_t keys_cap);
/* Merge the partitions an owner received: DEVICE arrays of nsrc sources in
 * shard order, src_counts[s] entries / src_key_bytes[s] blob bytes each
 * (fewer than 2^31 - 1 entries in all, else GCK_EINVAL). */
int gck_kd_merge(gck_ctx *ctx, const gck_kd_entry *d_entries, const uint8_t *d_keys, const uint64_t *src_counts,
                 const uint64_t *src_key_bytes, uint32_t nsrc, uint64_t *n_live, double *ms);
/* Host copies of the merged entries (key_off into the merged blob) and keys;
 * dst = keys = NULL only reports the sizes. */
int gck_kd_fetch_merged(gck_ctx *ctx, gck_kd_entry *dst, uint64_t cap, uint8_t *keys, uint64_t keys_cap,
                        uint64_t *n, uint64_t *n_key_bytes);

/* ---- several GPUs in one call ------------------------------
 * gck_replay over ndev devices (one rank per device): the files (walk order)
 * are cut into ndev contiguous shards of about equal bytes, only after files
 * that reset lastOffset (gck_plan_shards), and shard s replays on devices[s]
 * (a host thread per device).  The first startup error in walk order ends the
 * walk (core/db.go:134-138): its records before the error count, later shards
 * nothing.  Then the keydir merge above runs inside the library: per shard the
 * keydir with tombstones, partitioned by key hash over the devices, exchanged
 * with RCCL (ncclCommInitAll over the devices, grouped ncclSend / ncclRecv over
 * xGMI; librccl.so.1 is loaded at the first call), merged per owner.
 * out->recs = the global live keydir, one gck_rec per live key (rec.file = the
 * walk index into files[]; any order), out->n = live keys; n_crc_fail = CRC
 * rejects among the replayed records; status, err_file, err_off, files_walked
 * and final_last_offset as gck_replay reports them.  Free with
 * gck_result_free.  GCK_EDEVICE when RCCL cannot be loaded or a device fails. */
int gck_replay_multi(const gck_file *files, uint32_t nfiles, const int32_t *devices, uint32_t ndev,
                     const gck_opts *opts, gck_result *out);
/* gck_replay_multi of files named by path (read by the library, as
 * gck_replay_paths); with GCK_OPT_KEYS the live entries' key bytes come back
 * in out->keys, in the order of out->recs (either call). */
int gck_replay_multi_paths(const gck_path *files, uint32_t nfiles, const int32_t *devices, uint32_t ndev,
                           const gck_opts *opts, gck_result *out);
/* gck_replay_multi's keydir merge over shards that are already resident and
 * replayed: ctxs[s] holds shard s (a contiguous walk-order run of files, each
 * but the last shard's last file resetting lastOffset) after gck_ctx_run, on
 * its own device (several contexts on one device: every pair a device copy).
 * Per shard the keydir with tombstones packed over the n owners
 * (gck_ctx_keydir, gck_kd_pack), the partitions exchanged (RCCL across
 * devices, as gck_replay_multi), per owner the merge in ctxs[p] (gck_kd_merge).
 * out: status, err_file / files_walked (global walk indices), err_off,
 * final_last_offset and n_crc_fail resolved over the shards in order; n = live
 * keys; with GCK_MULTI_FETCH recs = the live entries (rec.file global; freed by
 * gck_result_free), with GCK_MULTI_KEYS also their key bytes.  ms (optional, 4
 * doubles): wall ms of keydir + pack, exchange, merge, fetch.  This is the
 * one-process multi-GPU path's exchange step, timed by bench.py --lib-multi. */
#define GCK_MULTI_FETCH 1u
#define GCK_MULTI_KEYS 2u
int gck_ctx_multi_keydir(gck_ctx *const *ctxs, uint32_t n, uint32_t flags, gck_result *out, double *ms);
/* The shard plan (host only, no device): shard s = files [ranges[2 s],
 * ranges[2 s + 1]); empty shards when there are fewer allowed cuts than
 * shards.  A cut at i needs reset_after[i - 1] (core/db.go:117-119). */
int gck_plan_shards(const uint64_t *sizes, const uint8_t *reset_after, uint32_t nfiles, uint32_t world,
                    uint32_t *ranges);
int gck_ctx_stats(gck_ctx *ctx, gck_stats *out);
const char *gck_phase_name(int phase);
/* Device pointers of the last run's outputs (gck_rec array, n records) and the
 * HIP stream the pipeline runs on (hipStream_t, as void*). */
int gck_ctx_device_recs(gck_ctx *ctx, const gck_rec **recs, uint64_t *n);
void *gck_ctx_stream(gck_ctx *ctx);
/* Copy `len` bytes of file `file` (as resident in the arena) back to host. */
int gck_ctx_read_file(gck_ctx *ctx, uint32_t file, uint64_t off, uint8_t *dst, uint64_t len);

/* ---- device record encoder (serializeEntry, core/db.go:272-284) ----------- */
/* Synthetic corpus spec (DESIGN.md "Corpus"): op i is a Put (or, with
 * tomb_permille, a Delete) written exactly as DB.Put/DB.Delete serialize it;
 * files rotate when size + entry > max_file_size (core/db.go:214-232). */
typedef struct gck_corpus_cfg {
    uint64_t seed;
    uint64_t max_file_size;
    uint64_t n_ops;         /* stop after n ops (0: use n_files)                  */
    uint32_t n_files;       /* stop when this many files are full                 */
    uint32_t key_min, key_max;
    uint64_t key_universe;  /* 0: unique keys                                     */
    uint32_t val_fixed;     /* >0: fixed value size; 0: bounded Zipf(1.1) 64..64K */
    uint32_t tomb_permille;
    uint32_t flip_permille; /* single-bit flips inside values, after the CRC     */
    uint32_t ts_base;
    uint64_t key_seed;      /* 0: key ids, lengths and bytes from seed (op i:    */
                            /* key id H(seed, 1, i)); else from key_seed, op i   */
                            /* of file id f drawing H(key_seed, 1, f << 32 | i): */
                            /* one key universe across gck_encode_files' per-   */
                            /* file corpora (BASELINE C4; f = 0 in               */
                            /* gck_encode_corpus)                                */
} gck_corpus_cfg;

/* Plan the corpus (host) and encode it straight into the context's device arena.
 * Files are placed in lexical (walk) order of their names data_<n>_<ts_base+n>;
 * the lexically last one is the active file.  n_files_out / file_sizes (creation
 * order, may be NULL) report the layout. */
int gck_encode_corpus(gck_ctx *ctx, const gck_corpus_cfg *cfg, uint32_t *n_files_out,
                      uint64_t *n_ops_out, uint64_t *file_sizes, uint32_t max_files);
/* Encode n independent one-file corpora into the context's arena, in the given
 * order (the caller's walk order): slot k is file data_<id>_<ts_base+id> with
 * file_ids[k] = id, generated by the spec of cfg with seed cfg->seed + id and
 * n_files = 1 (BASELINE C4: per-file seed 4 + n).  Every file resets lastOffset
 * except the last when last_is_active.  n_ops_out / file_sizes (n entries,
 * optional) report the ops and bytes per slot. */
int gck_encode_files(gck_ctx *ctx, const gck_corpus_cfg *cfg, const uint32_t *file_ids, uint32_t n,
                     uint32_t last_is_active, uint64_t *n_ops_out, uint64_t *file_sizes);
/* Walk-order index -> creation index n of file data_<n>_... in the last encoded corpus. */
int gck_encode_walk_order(gck_ctx *ctx, uint32_t *creation_index, uint32_t n);
/* The encoder's Zipf threshold table (65472 u32), for cross-checks. */
void gck_encode_zipf_table(uint32_t *thr);

/* Bulk serializeEntry (row f4; replaces the per-record encode of DB.Put /
 * DB.Delete, core/db.go:185-212 and :245-247, serializeEntry :272-284, header
 * encode core/header.go:38-48, for bulk loads and compaction).  Record i is a
 * Put of key i / value i, or, when tomb[i] != 0, a Delete of key i
 * (header{CRC32(key), ts, 0, len(key)} || key), written back to back into out
 * in order.  keys/vals are concatenated bytes with n+1 offsets
 * (key_off/val_off); every pointer except total is DEVICE memory, keys and
 * vals 4-byte aligned and readable 4 bytes past their last byte (the kernel
 * reads whole dwords); out_off (n+1) receives each record's offset in out;
 * *total = bytes written (or needed: GCK_EINVAL with nothing written to out
 * when out_cap < *total; GCK_EINVALID_KEY and nothing written to out when a
 * key is empty, as DB.Put / DB.Delete refuse it, core/db.go:186-188,
 * :294-297).  Offsets, CRCs and bytes are all computed on the device (16 B of
 * results cross PCIe).  stream: a hipStream_t, NULL for the default stream;
 * returns after the bytes are written. */
int gck_encode_batch(const uint8_t *keys, const uint64_t *key_off, const uint8_t *vals,
                     const uint64_t *val_off, const uint32_t *ts, const uint8_t *tomb, uint64_t n,
                     uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint64_t *total, void *stream);

/* ---- host-side DB mirror (core.NewDB / gocask.Open / Get / Keys) ------------ */
typedef struct gck_db gck_db;

typedef struct gck_config {
    int64_t max_data_file_size; /* core.Config.MaxDataFileSize (core/db.go:84-87)     */
    const char *data_dir;       /* core.Config.DataDir; joined with db_path           */
} gck_config;

/* core.NewDB(dbpath, fs.NewDisk(), time, cfg): create the dir if needed, pick the
 * active file (lexically last entry, created as data_<n>_<unix>.csk when the dir is
 * empty), walk every *.csk in lexical order and replay them on the GPU.  On a
 * startup error *out is still set (like NewDB returning &db, err) and the
 * message "gocask: startup error: unexpected EOF" is written to errbuf. */
int gck_db_open(const char *db_path, const gck_config *cfg, const gck_opts *opts, gck_db **out,
                char *errbuf, size_t errlen);
/* In-memory file system (internal/fs/memory.go): one file "data" (also active). */
int gck_db_open_mem(const uint8_t *data, uint64_t len, const gck_opts *opts, gck_db **out,
                    char *errbuf, size_t errlen);
/* DB.Get: GCK_EINVALID_KEY for an empty key, GCK_EKEY_NOT_FOUND, GCK_ECRC_FAILED.
 * On success *val (library-owned until the next call or close) holds *vlen bytes. */
int gck_db_get(gck_db *db, const uint8_t *key, uint32_t klen, const uint8_t **val, uint64_t *vlen);
/* DB.Keys: number of live keys; gck_db_key(i) returns the i-th (any order). */
uint64_t gck_db_keys(gck_db *db);
int gck_db_key(gck_db *db, uint64_t i, const uint8_t **key, uint32_t *klen);
/* kdEntry of a key (CRC, Timestamp, ValuePos, ValueSize, file name). */
int gck_db_entry(gck_db *db, const uint8_t *key, uint32_t klen, uint32_t *crc, uint32_t *ts,
                 uint32_t *value_pos, uint32_t *value_size, const char **file);
uint32_t gck_db_last_offset(gck_db *db);
const char *gck_db_active_file(gck_db *db);
uint32_t gck_db_nfiles(gck_db *db);
const char *gck_db_file_name(gck_db *db, uint32_t i);
void gck_db_close(gck_db *db);

/* Library/device info. */
int gck_device_count(void);
/* Pin (page-lock) caller memory, e.g. mmap'd data files, so gck_ctx_load /
 * gck_replay copy it by DMA at PCIe rate instead of through staging buffers;
 * unregister before unmapping.  Thin wrappers over hipHostRegister. */
int gck_host_register(const void *p, uint64_t len);
int gck_host_unregister(const void *p);
const char *gck_version(void);
/* Text of the last HIP failure on this thread (GCK_EDEVICE diagnostics). */
const char *gck_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
