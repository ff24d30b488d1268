// gck_internal.h — device context shared by the replay pipeline and the encoder.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/gocask_hip.h"
#include "gck_math.h"

#define GCK_HIP(x)                                         \
    do {                                                   \
        hipError_t e_ = (x);                               \
        if (e_ != hipSuccess) {                            \
            gck::set_error(#x, e_, __FILE__, __LINE__);    \
            return GCK_EDEVICE;                            \
        }                                                  \
    } while (0)

namespace gck {

void set_error(const char *what, hipError_t e, const char *file, int line);
const char *last_error();

// Grow-only device buffer.
struct DBuf {
    void *p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return GCK_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = bytes < 256 ? 256 : bytes;
        if (hipMalloc(&p, want) != hipSuccess) return GCK_ENOMEM;
        cap = want;
        return GCK_OK;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T>
    T *as() const { return static_cast<T *>(p); }
};

enum Phase {
    PH_BOUNDARY = 0,  // k_spec_entry, k_walk, k_validate / k_fixup rounds
    PH_SCAN,          // record slots per chunk, per-file summary
    PH_HOST,          // D2H summary + host bookkeeping (device path: k_account_grp)
    PH_RECORDS,       // k_compact (record table + row index)
    PH_CRC,           // k_crc_rows: the HBM-bound kernel
    PH_FINAL,         // k_finalize: CRC verdict + tuples
    PH_END,           // (event) end of the run
    PH_PIPE = PH_END, // (time) device span of the whole run
    PH_NPHASE
};

// d_gbase: the record bases gb[0] (0) and gb[1], then the records' range
// (clamped to capacity) and the run's range.
constexpr uint32_t kGbSlots = 2, kGbWords = kGbSlots + 4;
// d_queue: atomic work queues, zeroed before each use: k_crc_rows' row
// blocks, k_verify's item groups, compaction.
constexpr uint32_t kQueueCrc = 0, kQueueVerify = 1, kQueueCompact = 2, kQueueSlots = 3;


// 64-bit finaliser (splitmix64): the keydir's key hash (kd_common.h) and the
// hint entries' integrity word
__device__ __forceinline__ uint64_t mix64d(uint64_t x) {
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// The integrity word of one hint entry (GCK_HINT_VERSION 3): its five header
// words and its key's 4-byte little-endian words k(i) (the last one zero past
// the key) folded by h = (h ^ w) * K + i, then one finaliser.  Every step is
// a bijection of h, so a change in any one word always changes the word.
// Each index entry of a hint file holds the XOR of its block's words; the
// writer (compact.hip) and the reader (hints.hip) compute it the same way, and
// oracle.hint_entry_check restates it.
template <class Words>
__device__ __forceinline__ uint64_t hint_entry_check(uint32_t ts, uint32_t ks, uint32_t vs, uint32_t vpos,
                                                     uint32_t crc, const Words &k) {
    constexpr uint64_t K = 0x9E3779B97F4A7C15ull;  // odd
    uint64_t h = 0x2545F4914F6CDD1Dull ^ ((uint64_t)ks << 32);
    h = (h ^ ts) * K + 1;
    h = (h ^ vs) * K + 2;
    h = (h ^ vpos) * K + 3;
    h = (h ^ crc) * K + 4;
    for (uint32_t i = 0; 4 * i < ks; ++i) h = (h ^ k(i)) * K + 5 + i;
    return mix64d(h);
}

struct Ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // end-of-run counters and results land here by a kernel's PCIe writes
    // (coherent pinned host memory, mapped): no DMA-engine copy, which would
    // queue behind any large H2D already queued (gck_replay's file groups)
    uint32_t *h_mbox = nullptr, *d_mbox = nullptr;
    // layout tables go up through pinned, mapped host memory read by a kernel
    // on `stream` (k_upload), not by DMA copies, which would queue behind any
    // large H2D in flight (gck_replay's file groups)
    uint8_t *h_up = nullptr, *d_up = nullptr;
    size_t up_cap = 0;
    gck_opts opts{};
    int n_cu = 256;
    int fin_blocks_per_cu = 4;       // resident k_finalize<false> workgroups per CU
    int fin_blocks_per_cu_hash = 4;  // the same for k_finalize<true> (hashing: more registers)

    // arena: files in walk order, each at a kRow-aligned offset
    DBuf arena;
    uint64_t arena_len = 0;  // bytes covered by rows (multiple of kRow)
    uint32_t nfiles = 0;
    std::vector<uint64_t> f_base, f_len;
    std::vector<uint8_t> f_reset;
    std::vector<uint32_t> f_first_chunk, f_nchunks;
    uint64_t data_bytes = 0;

    // chunk metadata
    uint32_t n_chunks = 0;
    DBuf d_fbase, d_flen, d_ffirst, d_fnch, d_fbad, d_fterm, d_ftpos, d_fnrec, d_ffirstrec, d_carry;
    DBuf d_ch_file, d_ch_start, d_ch_end, d_ch_entry, d_ch_exit, d_ch_count, d_ch_term, d_ch_tpos, d_ch_bad;
    DBuf d_ch_wend;              // where each chunk's walk stopped (its bound, walk_bound)
    DBuf d_ch_aentry;            // each chunk's walked entry as an arena offset (k_compact's record base)
    uint32_t chunk_shift = 17;   // log2(opts.chunk_bytes)
    DBuf d_rec_base, d_bsum, d_stage, d_counters;  // d_stage: (KeySize, ValueSize) per walked record (stage_slot)
    DBuf d_freset;                   // per file: 1 = lastOffset resets after it
    DBuf d_gbase;                    // record range of the run [0, n)

    // records
    uint64_t n_recs = 0;
    uint64_t rec_cap = 0;  // record-table capacity of the current run
    DBuf d_rec_off, d_rec_kv, d_rec_file, d_ep, d_out;  // record table: arena offset, (KeySize, ValueSize), file
    // rows
    uint64_t n_rows = 0;
    DBuf d_blk_first, d_rend, d_queue;  // d_blk_first: the first record ending past each 64-row block start

    // constant tables
    DBuf d_slice, d_nib, d_xinv, d_xa, d_xb, d_zrow;

    // device keydir (keydir.hip): key hashes, slot table, live flags, tile
    // ranks, the live records
    DBuf d_khash, d_ktab, d_live, d_ktile, d_kdout, d_kdidx;
    DBuf d_kdstat;  // keydir table: [0] overflow (a key found no slot in kMaxProbe), [1] keys (claimed slots)
    uint64_t n_live = 0;
    bool kd_hashed = false;  // d_khash holds the key hashes of the last run's records
    bool kd_inserted = false;  // d_ktab holds the last run's records (its finalize inserted them)
    bool kd_fin_table = false;  // the last finalize launch builds the keydir table
    uint64_t kd_tab_slots = 0;  // d_ktab's slots then
    uint64_t kd_keys_hint = 0;  // distinct keys of the last keydir built here (sizes the next table)
    bool hash_keys = false;  // runs hash every record's key in finalize (gck_ctx_keydir_hash)
    uint32_t kd_flags = 0;                                // flags of the last gck_ctx_keydir
    // compaction (compact.hip): record / hint-entry offsets, block sums, file
    // starts, file count, merged data and hint bytes
    DBuf d_cpos, d_chpos, d_cbsum, d_cfstart, d_cnf, d_cdata, d_chint, d_cfoot;
    DBuf d_cjmp, d_con;  // many-file rotation points: jump pointers (two copies), start marks
    uint32_t cmp_files = 0;
    uint64_t cmp_data = 0, cmp_hint = 0;
    // keydir merge across shards: pack partition of each live entry, the
    // merged headers / keys of the entries this rank owns
    DBuf d_kpart, d_kcrank, d_kbrank, d_kpsum, d_kptot;  // pack: partition, in-tile ranks, tile sums
    DBuf d_mkoff, d_mtab, d_mlive, d_msrc, d_mhdr, d_mkeys;  // merge
    DBuf d_mout;                                             // its gck_rec array (merged_out)
    uint32_t kd_nparts = 0;                               // of the last gck_kd_pack_sizes
    uint64_t kd_packed = 0;                               // entries it partitioned
    uint64_t kd_tot[128] = {};                            // its per-partition counts, key bytes
    uint64_t n_merged = 0, merged_key_bytes = 0;
    bool kd_valid = false;   // d_ktab / d_khash / d_kdout describe the last run
    uint64_t kd_slots = 0;   // table slots (power of two; 0: no records)
    uint64_t kd_probe_bound = 256;  // lookups probe at most this far (kMaxProbe, or the unbounded build's longest)
    // batched Get / scrub (get.hip): query keys, per-item state, values
    DBuf d_gkeys, d_gkoff, d_gstat, d_gitem, d_gvsize, d_gexp, d_gcrc, d_gvoff, d_gvals, d_gscan;
    // the key blob of gck_replay with GCK_OPT_KEYS: look-back words, offsets, bytes
    DBuf d_klb, d_koff, d_keyblob;

    // results of the last run
    int32_t status = 0;
    uint32_t err_file = 0, files_walked = 0, final_last_offset = 0;
    uint64_t err_off = 0, n_crc_fail = 0, n_fixups = 0, n_overflow = 0;
    bool device_path = false;  // the last run had no host round trip (ctx_run_device)
    bool from_hints = false;   // the tuples came from hint files (hints.hip): the arena holds no data files
    uint32_t n_reruns = 0;     // device-only runs redone on the host path
    double ms_total = 0, ms_phase[PH_NPHASE] = {};
    bool phase_timing = false;  // an event between every phase (gck_ctx_phase_timing)
    double ms_crc_sum = 0;      // k_crc_rows event time summed over runs
    uint64_t n_runs = 0;
    hipEvent_t ev[PH_END + 1] = {};


    // encoder bookkeeping
    std::vector<uint32_t> walk_to_creation;
};

int ctx_layout(Ctx *c, const uint64_t *lens, uint32_t nfiles, const uint8_t *reset_after);

// A data file: caller memory (data), or a path the copier opens per chunk it
// reads (no descriptor is held across the call: a database with more files
// than RLIMIT_NOFILE still opens, as the reference's Walk does, one at a time)
struct Src {
    const uint8_t *data;
    const char *path;
    uint64_t len;
    bool reset_after;
    uint64_t dev, ino;  // a path's file as stat saw it (each chunk's read checks it is the same)
};

// Host-to-device copies of gck_replay's file groups on one copy stream
// (staging.hip): registered memory by the DMA engine directly (direct), the
// rest through page-locked staging buffers filled by host threads (add:
// memcpy from src, or pread of its path when src is null).  Group g's event is
// recorded on the stream once every chunk of the group is queued (seal, then
// wait_recorded before a stream waits on it).
class Copier {
   public:
    Copier();
    ~Copier();
    int start(int dev, hipStream_t stream, std::vector<hipEvent_t> *group_ev);
    void add(uint32_t group, const Src &src, uint64_t off, uint64_t len, uint8_t *dst);
    int direct(const uint8_t *src, uint64_t len, uint8_t *dst);
    void seal(uint32_t group);
    int wait_recorded(uint32_t group);
    int finish();  // joins the threads; the first error of any copy

   private:
    struct Impl;
    Impl *p;
    int dev_ = 0;
};
void stage_release();  // frees the idle staging buffers (gck_replay_release_cache)
uint32_t stage_buffers_wanted();             // staging buffers a Copier takes
int stage_prealloc(int dev, uint32_t n);     // fill the idle pool ahead of a Copier
bool host_pinned(const void *p);  // page-locked (registered or hipHostMalloc) host memory
// gck_result arrays: page-locked or plain, both freed by res_free
void *res_alloc(uint64_t bytes, bool pinned);
void res_free(void *p);
// dst = the segments back to back (host threads for large totals)
void par_gather(uint8_t *dst, const std::vector<std::pair<const void *, uint64_t>> &segs);
std::vector<Src> mem_srcs(const gck_file *files, uint32_t nfiles);
// gck_replay's ring of file groups with a hook instead of tuple delivery:
// group(g, first file of the group, its context) runs after each group has
// replayed (on the context's stream, which the hook may use and synchronise);
// out receives the outcome (status, err_file / err_off / files_walked relative
// to files, final_last_offset, n_crc_fail, n_groups / n_resident), no records.
struct GroupSink {
    virtual ~GroupSink() = default;
    virtual int group(uint32_t g, uint32_t file0, gck_ctx *ctx) = 0;
};
int replay_groups_to(const Src *files, uint32_t nfiles, const gck_opts *opts, GroupSink *sink, gck_result *out);
// the ring's data-byte budget when gck_opts.max_resident is 0 (replay.hip)
int auto_budget(const gck_opts *opts, uint64_t *budget);
// gck_replay_multi (multi.hip): one shard's outcome, the global outcome over
// shards in walk order, the exchange's receive offsets, and the call itself
// (loopback: several shards may share a device; every pair is a device copy)
struct MultiOutcome {
    int32_t status;
    uint32_t nfiles, err_file, files_walked, final_last_offset;
    uint64_t err_off, n_crc_fail;
};
void multi_resolve(const MultiOutcome *sh, uint32_t n, uint32_t nfiles, gck_result *out, uint8_t *contrib);
void multi_recv_offsets(const uint64_t *counts, uint32_t nsrc, uint32_t nown, uint64_t *off);
int replay_multi(const Src *files, uint32_t nfiles, const std::vector<int> &devs, const gck_opts *opts,
                 gck_result *out, bool loopback);
// the pool of idle contexts behind gck_replay (per device, one options key each)
int pool_take(const gck_opts *o, gck_ctx **out);
void pool_give(const gck_opts *o, gck_ctx *c);
// the last run's key bytes back to back into a new pinned host buffer (replay.hip)
int ctx_gather_keys(Ctx *c, void **host, uint64_t *len);
// the last gck_kd_merge's live entries as a gck_rec array and (keys non-null)
// their key bytes back to back, shaped on the device: the entry count and key
// bytes first, then the copies into host memory of those sizes (replay.hip)
int merged_out_sizes(Ctx *c, bool want_keys, uint64_t *n, uint64_t *key_bytes);
int merged_out(Ctx *c, gck_rec *h, uint8_t *keys, uint64_t key_bytes);
// stats every path (GCK_EIO when one fails); the paths must outlive the call
int open_srcs(const gck_path *files, uint32_t nfiles, std::vector<Src> &out);
void close_srcs(std::vector<Src> &v);
// n files into device memory through a Copier on stream, then waits for them
int copy_files_sync(int dev, hipStream_t stream, const Src *src, uint8_t *const *dst, uint32_t n);
// gck_ctx_load of sources: layout, then the copies
int ctx_load_srcs(Ctx *c, const Src *src, uint32_t n);

}  // namespace gck

struct gck_ctx {
    gck::Ctx c;
};
