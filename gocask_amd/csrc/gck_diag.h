/*
 * gck_diag.h — measurement helpers of libgocask_diag.so (diag.hip), a separate
 * library next to libgocask_hip.so: not part of the product ABI
 * (include/gocask_hip.h) and not on the replay path.  bench.py uses
 * gck_diag_stream_read for the practical HBM read ceiling it reports beside
 * the spec peak; tools/chase.py the random-access probes.
 */
#ifndef GCK_DIAG_H
#define GCK_DIAG_H
#include "../../include/gocask_hip.h"
#ifdef __cplusplus
extern "C" {
#endif
/* A plain streaming read of the context's resident arena (16 B per lane,
 * non-temporal loads): ms per pass and GB/s. */
int gck_diag_stream_read(gck_ctx *ctx, int iters, double *ms_per_iter, double *gbs);
/* The XCD-balanced stream ceiling: k_crc_rows' geometry and work assignment
 * (64-row blocks, static_eighths / 8 of the full rounds static, the rest from
 * an atomic queue) without its compute.  stamp: the last pass records
 * per-wavefront clock stamps (gck_diag_clock_read). */
/* Stream probe: k_crc_rows' row loads, pf (1..3) rows in flight per
 * wavefront, no compute; blocks: 64-row blocks per wavefront (else rows
 * strided over the wavefronts); workgroups of `threads` with lds_kib of LDS,
 * wg_per_cu of them per CU in the grid. */
int gck_diag_stream_xp(gck_ctx *ctx, int pf, int blocks, int threads, int lds_kib, int wg_per_cu, int iters,
                       int stamp, double *ms_per_iter, double *gbs);
int gck_diag_stream_blocks(gck_ctx *ctx, int iters, uint32_t static_eighths, int stamp, double *ms_per_iter,
                           double *gbs);
/* Stamps of the last stamped gck_diag_stream_blocks pass: per wavefront 4 u64
 * (shader clock, 100 MHz real time at start; the same at end) and its XCC id;
 * cap_waves >= 16384. */
int gck_diag_clock_read(uint64_t *stamps, uint32_t *xcc, uint32_t cap_waves);
/* Read probes over the arena: 0 = the streaming read with the default cache
 * policy, 15 = with non-temporal loads (gck_diag_stream_read's kernel), 1 = a
 * lane-contiguous 64 B slab layout (lane stride 64 B), 2 = same geometry
 * coalesced, 16 / 17 = k_crc_rows' row geometry without compute, 3..14 =
 * random-access probes. */
int gck_diag_stream_pattern(gck_ctx *ctx, int pattern, int iters, double *ms_per_iter, double *gbs);
/* 65,536 dependent chains reading 16 x lpc bytes per round trip (lpc lanes per
 * chain), hops round trips each: the cost of a windowed header walk. */
int gck_diag_chase_win(gck_ctx *ctx, int lpc, uint32_t hops, int iters, double *ms_per_iter);
/* Per-chunk chain length (records k_walk staged) and final entry of the last
 * run; count / entry NULL: *n = chunks only. */
int gck_diag_chunks(gck_ctx *ctx, uint32_t *count, uint64_t *entry, uint64_t cap, uint64_t *n);
/* ---- gck_replay_multi's orchestration, testable on one GPU / the CPU ----
 * One shard's outcome as gck_replay reports it (gck::MultiOutcome). */
typedef struct gck_diag_outcome {
    int32_t status;
    uint32_t nfiles, err_file, files_walked, final_last_offset;
    uint64_t err_off, n_crc_fail;
} gck_diag_outcome;
/* The global outcome over n shards in walk order (host only): out's status,
 * err_file / err_off (rebased), files_walked, final_last_offset, n_crc_fail;
 * contrib[s] = 1 for the shards whose records count. */
int gck_diag_multi_resolve(const gck_diag_outcome *sh, uint32_t n, uint32_t nfiles, gck_result *out,
                           uint8_t *contrib);
/* Receive offsets of the exchange (host only): off[p * (nsrc + 1) + i] = items
 * owner p receives from sources before i; counts[i * nown + p]. */
int gck_diag_multi_recv_offsets(const uint64_t *counts, uint32_t nsrc, uint32_t nown, uint64_t *off);
/* gck_replay_multi with nshards logical shards on one device: the same plan,
 * ring replays, keydir packs, status resolution, receive layout and merges,
 * the partitions moved by device copies instead of RCCL (test entry). */
int gck_diag_replay_multi_loopback(const gck_file *files, uint32_t nfiles, uint32_t nshards, int32_t device,
                                   const gck_opts *opts, gck_result *out);
#ifdef __cplusplus
}
#endif
#endif
