/*
 * gprx_dev.h — developer hooks of libgprx (NOT part of the drop-in boundary in gprx.h).
 * Times individual device kernels in isolation so they can be tuned against their
 * roofline; used by scripts/devbench.py.  No reference counterpart.
 */
#ifndef GPRX_DEV_H
#define GPRX_DEV_H
#include "gprx.h"
#ifdef __cplusplus
extern "C" {
#endif
/* what: 0 = diagonal 128-block factor+inverse, 1 = gemm_nt (C -= A B^T), 2 = lower gemm_nt,
 *       3 = full potrf of an n x n SPD matrix (single stream), 4 = potrf with look-ahead,
 *       5 = back substitution (m = 1) of an n x n factor,
 *       6 = diagonal kernel phase profile: ms must hold 5 doubles, receiving the mean
 *           s_memtime ticks per launch of (load, solve phases, update phases, store, total),
 *       7 = potrf with look-ahead replayed from a captured hipGraph, 8 = backsolve from a graph.
 * For 1/2: (M, N, K) are the gemm sizes; for 3/4/5: M = n.  Returns the mean device time
 * per call over `iters` calls (HIP events) in *ms. */
gprx_status gprx_dev_bench(gprx_ctx* ctx, gprx_dtype dtype, int32_t what, int64_t M, int64_t N, int64_t K,
                           int32_t iters, double* ms);
#ifdef __cplusplus
}
#endif
#endif
