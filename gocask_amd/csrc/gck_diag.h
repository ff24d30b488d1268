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
/* Read probes over the arena: 0 = the streaming read with the default cache
 * policy, 15 = with non-temporal loads (gck_diag_stream_read's kernel), 1 = a
 * lane-contiguous 64 B slab layout (lane stride 64 B), 2 = same geometry
 * coalesced, 16 / 17 = k_crc_rows' row geometry without compute, 3..14 =
 * random-access probes. */
int gck_diag_stream_pattern(gck_ctx *ctx, int pattern, int iters, double *ms_per_iter, double *gbs);
/* Per-chunk chain length (records k_walk staged) and final entry of the last
 * run; count / entry NULL: *n = chunks only. */
int gck_diag_chunks(gck_ctx *ctx, uint32_t *count, uint64_t *entry, uint64_t cap, uint64_t *n);
#ifdef __cplusplus
}
#endif
#endif
