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
 *       7 = potrf with look-ahead replayed from a captured hipGraph, 8 = backsolve from a graph,
 *       9 = potrf as one persistent tile-dataflow launch (potrf_tiles),
 *      10 = back substitution as one flag-chained launch (launch_backsolve_chain),
 *      11 / 12 / 13 = the tile engine's diagonal-block factor, variant what - 11 (rank-8 /
 *           blocked / look-ahead): ms must hold 9 doubles: ms[0] = us per factor, ms[1..5] =
 *           phase ticks (100 MHz), ms[6..8] = fact32 core cycles (GPRX_FACT32_PROF builds).
 * For 1/2: (M, N, K) are the gemm sizes; for 3/4/5: M = n.  Returns the mean device time
 * per call over `iters` calls (HIP events) in *ms. */
gprx_status gprx_dev_bench(gprx_ctx* ctx, gprx_dtype dtype, int32_t what, int64_t M, int64_t N, int64_t K,
                           int32_t iters, double* ms);
/* Host-only: build the tile-dataflow potrf schedule for nc diagonal blocks, nr row blocks
 * and P workers (build bit 0: with the fused covariance-build tasks; bit 1: the last nc of
 * the nr row blocks are identity rows, the inverse riding along; bits 8..15: the update
 * chunk rule's ratio + 1, 0 = the rule the simulated makespan picks; bits 16..23: the paired
 * updates' first row below the diagonal + 1, 1 = no pairs, 0 = the simulation's choice); returns its task count
 * and simulated makespan (us).  Throws nothing, needs no
 * device: GPRX_ERR_ARG if the ticket order would violate a dependency. */
gprx_status gprx_dev_schedule(int32_t nc, int32_t nr, int32_t P, int32_t build, double* est_us, int64_t* ntasks);
/* Host-only: the same schedule's ticket list, 4 ints per ticket {type | chunk panels << 8, i, j,
 * first panel} (types 0 DIAGX, 1 TRSM, 2 UPD, 3 BUILD, 4 TPART with j = the part, 5 UPD2: the
 * tiles (i, j) and (i + 1, j) as one 256 x 128 update), at most max
 * tickets into out; returns the task count, -1 on bad arguments. */
int64_t gprx_dev_schedule_list(int32_t nc, int32_t nr, int32_t P, int32_t build, int32_t* out, int64_t max);
/* Host-only: the distributed factorisation's schedule (g ranks of P workers each, row blocks
 * grouped by gb, a window of ww panels; flags bit 0: with the fused covariance-build tasks,
 * bit 1: LML mode, the inverse's identity rows and the C = U U^T tiles riding along), simulated
 * over all ranks with the pushes and window releases as timed nodes; returns the simulated
 * makespan (us), the update chunk width and the task count -- the figures gprx_dist.cpp picks
 * gb and ww by.  GPRX_ERR_ARG if the ticket order would violate a dependency. */
gprx_status gprx_dev_dist_schedule(int32_t nc, int32_t P, int32_t g, int32_t gb, int32_t ww, int32_t flags,
                                   double* est_us, int32_t* chunk_w, int64_t* ntasks);
/* GPRX_PT_DEBUG=1: copy the per-workgroup status {ticket, phase, i, j} of the running (or last)
 * potrf_tiles launch out of pinned host memory, without synchronising; returns workgroups. */
int32_t gprx_dev_pt_debug(int32_t* out, int32_t max_wg);
/* GPRX_PT_TRACE=1: timeline of the last potrf_tiles launch.  tasks: 4 ints per ticket
 * {type | nb << 8, i, j, b0}; times: 4 int64 per ticket {taken, inputs ready, published,
 * workgroup} in 100 MHz wall-clock ticks.  Synchronises the device; returns tickets copied. */
int64_t gprx_dev_pt_trace(int32_t* tasks, int64_t* times, int64_t max);
/* GPRX_BS_TRACE=1: per block of the last back substitution {start, non-critical tiles done,
 * alpha_{k+1} seen, alpha_k published} (100 MHz wall clock); returns blocks. */
int64_t gprx_dev_bs_trace(int64_t* times, int64_t max_blocks);
/* Parity hook for the PRODUCTION covariance build (the fit never materialises K on its own):
 * K(X, X) + sigma^2 I of n samples (row-major host X, n x d) as the fit's MFMA pair-statistics
 * path writes it, returned as the full symmetric n x n row-major matrix.
 *   path 0: the BUILD tasks of the fused tile factorisation (potrf_tiles_kernel, the
 *           default fit path for sum-of-exp-leaf trees), launched with no other task;
 *   path 1: the stand-alone kbuild_mma_kernel (trees the fused build does not carry).
 * GPRX_ERR_ARG when the tree is not covered by that path; GPRX_ERR_NONFINITE as the fit. */
gprx_status gprx_dev_build_matrix(gprx_ctx* ctx, gprx_dtype dtype, const gprx_kernel_desc* kernel, const void* X,
                                  int64_t n, int32_t d, double sigma, int32_t path, void* K);
/* Device time (mean over `iters` launches, HIP events on the launch's stream) of the same
 * build alone, features already resident: bench.py reports the build's GB/s from it. */
gprx_status gprx_dev_build_time(gprx_ctx* ctx, gprx_dtype dtype, const gprx_kernel_desc* kernel, const void* X,
                                int64_t n, int32_t d, double sigma, int32_t path, int32_t iters, double* ms);
/* Test context for the distributed fit: `world` VIRTUAL ranks in this process, all on one
 * GPU -- each runs its own persistent tile launch over its row blocks (a share of the CUs),
 * with device copies in place of the RCCL broadcast / panel exchange (gprx_dist.cpp).  Models
 * of this context fit with the multi-GPU algorithm end to end on a single device. */
gprx_status gprx_ctx_create_virtual(int device, int world, gprx_ctx** out);
/* Layout and memory of a model's last distributed fit (gprx_dist.cpp), written to the first
 * min(nout, 11) slots of out: out[0] device bytes the engine holds per rank (max over this
 * process's ranks; the fit's buffers), out[1] of which the packed own row blocks, out[2] row-block
 * group gb, out[3] window panels ww, out[4] update chunk width, out[5] workgroups per rank, out[6]
 * simulated makespan (us), out[7] ranks, out[8] 1 when this process holds the dense N x N factor
 * (gathered for the core matrix or a VALU-gradient tree; the posterior covariance solves across
 * the ranks without it), out[9] query chunks of 128 one sharded posterior solve takes (0: none
 * on this layout), out[10] device bytes of the last sharded posterior solve's K(Z, X_own)
 * workspace per rank (its queries x this rank's own rows only). */
gprx_status gprx_dev_dist_info(gprx_model* model, int64_t* out, int32_t nout);
/* (round 6) out[11..13] of gprx_dev_dist_info: this process's rank's pushes per fit, from the
 * schedule of the last distributed fit -- out[11] Linv_k pushes (each own diagonal block to every
 * peer), out[12] final-tile pushes (each own tile L_ib, b < nc, to every peer that reads row i
 * through its window), out[13] their bytes; out[14] the rank these describe. */
/* Identity of a context, written to the first min(nout, 10) slots of out: out[0] rank, out[1]
 * world, out[2] HIP device ordinal, out[3] transport (0 single GPU, 1 RCCL, 2 peer context over
 * the caller's all-gather, 3 virtual ranks), out[4] ranks the RCCL communicator holds
 * (ncclCommCount; -1 when there is none), out[5] the rank RCCL assigned (ncclCommUserRank; -1),
 * out[6..8] the device's PCI domain, bus and device numbers (distinct GPUs have distinct
 * triples), out[9] the CU share index of a shared-GPU rehearsal (GPRX_DIST_SHARED_GPU; else 0).
 * Local: no collective. */
gprx_status gprx_dev_ctx_info(gprx_ctx* ctx, int64_t* out, int32_t nout);
/* Parity hook for the tile engine's diagonal-block factor: the 128 x 128 SPD block A (column-
 * major, host) factored by variant 0 (rank-8 register image), 1 (blocked) or 2 (blocked with
 * look-ahead): L (lower triangle meaningful, the upper keeps A), Linv = L^{-1} (column-major)
 * and info (INT_MAX when SPD, else the 1-based first non-positive pivot column). */
gprx_status gprx_dev_diag_factor(gprx_ctx* ctx, int32_t variant, const double* A, double* L, double* Linv,
                                 int32_t* info);
/* The pair-statistics epilogues' f64 exp (gprx_internal.h fexp) on n host values (accuracy
 * test against the C library). */
gprx_status gprx_dev_fexp(gprx_ctx* ctx, const double* x, int64_t n, double* y);
#ifdef __cplusplus
}
#endif
#endif
