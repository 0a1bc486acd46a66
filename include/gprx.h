/*
 * gprx.h — C ABI of libgprx, the MI355X (gfx950) numerics layer of gpr_amd.
 *
 * This is the drop-in boundary for the agiger/GPR hot path.  The reference crosses a
 * foreign ABI exactly once on this path — the Fortran LAPACK calls in
 * include/LAPACKUtils.h:13-27 (dgetrf_/dgetri_/dpotrf_/dpotri_/ilaenv_) — and otherwise
 * runs everything inside the templated C++ classes GaussianProcess<T>
 * (include/GaussianProcess.h:73-171, lib/GaussianProcess.cpp), Kernel<T>
 * (include/Kernel.h:40-146), GaussianLogLikelihood<T> (include/Likelihood.h:154-350) and
 * SparseGaussianProcess<T> (include/SparseGaussianProcess.h:33-411).  The C++ host layer
 * of this repo (include/gpr/) keeps those class signatures and calls the entry points
 * below instead of Eigen + LAPACK.  Each entry point names the reference code it replaces.
 *
 * Conventions
 *   - plain C types only; every matrix a caller passes is row-major, in the model's scalar
 *     type (float for GPRX_F32, double for GPRX_F64), exactly the layout of the reference's
 *     Eigen RowMajor MatrixType (include/GaussianProcess.h:42); it is HOST memory except where
 *     an entry point says "host or device memory" (gprx_model_set_data, gprx_sparse_fit: a
 *     pointer from gprx_device_alloc is read in HBM, without a PCIe transfer);
 *   - no entry point throws; each returns a gprx_status and records a message retrievable
 *     with gprx_last_error();
 *   - a model owns its device buffers (training inputs, labels, Cholesky factor, regression
 *     vectors) and keeps them resident in HBM between calls;
 *   - read-only model calls (predict, posterior covariance) may be issued concurrently from
 *     several host threads after a fit (the reference's tests do this,
 *     tests/PosteriorProcessTest.cpp:120-134); they are serialised internally.
 */
#ifndef GPRX_H
#define GPRX_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GPRX_ABI_VERSION 2

typedef enum gprx_status {
    GPRX_OK = 0,
    GPRX_ERR_NONFINITE = 1, /* lib/GaussianProcess.cpp:399-401 "kernel matrix contains entries which are not finite." */
    GPRX_ERR_NOT_SPD = 2,   /* Cholesky pivot <= 0 (dpotrf_ INFO > 0, include/LAPACKUtils.h:64) */
    GPRX_ERR_SINGULAR = 3,  /* LU pivot == 0 (dgetrf_ INFO > 0, include/LAPACKUtils.h:46-47) */
    GPRX_ERR_DIM = 4,       /* lib/GaussianProcess.cpp:709-724 dimension checks */
    GPRX_ERR_HIP = 5,
    GPRX_ERR_RCCL = 6,
    GPRX_ERR_OOM = 7,
    GPRX_ERR_ARG = 8,
    GPRX_ERR_STATE = 9,     /* e.g. predict before fit (lib/GaussianProcess.cpp:677-679) */
    GPRX_ERR_NO_DEVICE = 10
} gprx_status;

typedef enum gprx_dtype { GPRX_F32 = 0, GPRX_F64 = 1 } gprx_dtype;

/* Kernel identity.  Replaces virtual dispatch through Kernel<T>::operator() /
 * GetDerivative (include/Kernel.h:52-59) and the string form parsed by
 * KernelFactory<T>::GetKernel (include/KernelFactory.h:83-178).  A kernel is a POST-ORDER
 * program: leaves push a value, SUM/PRODUCT pop two.  Leaf parameters are stored in the
 * reference's GetParameters() order so gradient vectors line up:
 *   GAUSSIAN          p = (sigma, scale)        include/Kernel.h:483-488
 *   GAUSSIAN_EXP      p = (sigma, scale)        include/Kernel.h:602-607
 *   WHITE             p = (scale)               include/Kernel.h:717-720
 *   RATIONAL_QUADRATIC p = (scale, sigma, alpha) include/Kernel.h:812-819
 *   PERIODIC          p = (scale, b, sigma)     include/Kernel.h:950-960
 *   SUM / PRODUCT     gradient = [k1 params, k2 params] include/Kernel.h:169-178, 318-327 */
typedef enum gprx_kop {
    GPRX_K_GAUSSIAN = 1,
    GPRX_K_GAUSSIAN_EXP = 2,
    GPRX_K_WHITE = 3,
    GPRX_K_RATIONAL_QUADRATIC = 4,
    GPRX_K_PERIODIC = 5,
    GPRX_K_SUM = 6,
    GPRX_K_PRODUCT = 7
} gprx_kop;

#define GPRX_MAX_KNODES 32
#define GPRX_MAX_KPARAMS 48

typedef struct gprx_knode {
    int32_t op;   /* gprx_kop */
    int32_t pad;
    double p[3];  /* leaf parameters as the reference stores them (in T, widened) */
} gprx_knode;

typedef struct gprx_kernel_desc {
    int32_t n_nodes;
    int32_t pad;
    gprx_knode node[GPRX_MAX_KNODES];
} gprx_kernel_desc;

typedef struct gprx_ctx gprx_ctx;
typedef struct gprx_model gprx_model;

/* Fit diagnostics (per call). */
typedef struct gprx_fit_info {
    double logdet;       /* log det(K + sigma^2 I) = 2 sum log L_ii (exact, not clamped) */
    double datafit;      /* sum over outputs of y^T (K + sigma^2 I)^{-1} y */
    int32_t info;        /* 0, or the 1-based column of the first non-positive Cholesky pivot */
    int32_t method;      /* 0 = Cholesky (potrf/potrs), 1 = LU fallback (the Cholesky failed) */
    double ms_build;     /* device time of the covariance build (HIP events) */
    double ms_factor;    /* device time of the factorisation */
    double ms_solve;     /* device time of the regression-vector solve */
    double ms_refine;    /* fp32 models: device time of the fp64 iterative refinement */
    double refine_delta; /* fp32 models: |last correction|_inf / |alpha|_inf (0 if not refined) */
    int32_t refine_steps;/* fp32 models: refinement steps taken */
    int32_t pad;
} gprx_fit_info;

/* ---- library / context ---------------------------------------------------------- */
int gprx_abi_version(void);
gprx_status gprx_device_count(int* count);
/* One context per process per GPU. */
gprx_status gprx_ctx_create(int device, gprx_ctx** out);
/* Multi-GPU context: one process per GPU, RCCL communicator over xGMI.  `unique_id` is
 * GPRX_UNIQUE_ID_BYTES produced by gprx_dist_unique_id() on rank 0 and shared by the
 * caller (any host channel: bench.py uses gpr_amd/hostcoll.py's sockets).  The communicator is
 * initialised nonblocking and polled with a deadline (GPRX_RCCL_INIT_TIMEOUT_S, default 120 s):
 * a rank that cannot reach its peers gets GPRX_ERR_RCCL instead of blocking for ever, and the
 * caller can fall back to gprx_ctx_create_peer (every rank must then do so: bench.py agrees on
 * it over its host channel).  GPRX_RCCL_FAIL=1 fails the call on purpose (tests).  New
 * capability: the reference is single-host OpenMP only. */
#define GPRX_UNIQUE_ID_BYTES 128
gprx_status gprx_dist_unique_id(void* out);
gprx_status gprx_ctx_create_dist(int device, int rank, int world, const void* unique_id, gprx_ctx** out);
/* Multi-process context bootstrapped by the CALLER's collective instead of RCCL (e.g. over
 * torch.distributed gloo or MPI): `fn` must all-gather `bytes` bytes from every rank into recv
 * (world * bytes, rank order) and return 0.  The library calls it only for its own host-side
 * exchanges (the mailboxes' IPC handles once per problem shape, a few bytes of reductions per
 * fit); the factorisation's panel traffic goes device to device.  Ranks may share one GPU
 * (GPRX_DIST_SHARED_GPU=1: each takes 1/world of the CUs), which is how the multi-process path
 * is tested on a one-GPU box. */
typedef int (*gprx_allgather_fn)(void* user, const void* send, size_t bytes, void* recv);
gprx_status gprx_ctx_create_peer(int device, int rank, int world, gprx_allgather_fn fn, void* user, gprx_ctx** out);
void gprx_ctx_destroy(gprx_ctx* ctx);
/* Message of the last failing call on this context (ctx may be NULL: last failure of
 * any call on this thread). */
const char* gprx_last_error(const gprx_ctx* ctx);

/* Opt-in per-kernel device timing: when enabled, every launch of the library's kernel
 * classes (kbuild, potrf_diag, potrf_trsm, potrf_update, backsolve, predict, lml_grad,
 * spd_inverse) is bracketed by HIP events on the stream it runs on; gprx_ctx_get_stats
 * returns per-class launch counts, summed device milliseconds and the ALGORITHMIC flops
 * and bytes of those launches.  Enabling resets the counters. */
typedef struct gprx_kstat {
    char name[32];
    int64_t launches;
    double ms;
    double flops;
    double bytes;
} gprx_kstat;
gprx_status gprx_ctx_set_stats(gprx_ctx* ctx, int32_t enable);
gprx_status gprx_ctx_get_stats(gprx_ctx* ctx, gprx_kstat* out, int32_t max, int32_t* count);

/* Device buffers on the context's GPU, for inputs that stay resident in HBM across calls (the
 * calls documented as taking "host or device memory" read them without a PCIe transfer).
 * Upload / download are synchronous on the context's stream.
 * Runtime binding: libgprx asks for libamdhip64.so.7 and librccl.so.1 by soname (RUNPATH
 * /opt/rocm/lib), and the loader resolves a soname to an object already in the process first.
 * Loaded before any other HIP user it binds /opt/rocm's runtime and RCCL (what it is compiled
 * against; bench.py and the tests load it so).  Loaded after the PyTorch wheel it binds the
 * copies that wheel bundles instead -- one runtime in the process either way, and a pointer
 * from that runtime's allocator is then this library's too; loaded BEFORE the wheel, the wheel
 * maps a second, separate runtime whose allocations this library cannot use. */
gprx_status gprx_device_alloc(gprx_ctx* ctx, int64_t bytes, void** out);
gprx_status gprx_device_free(gprx_ctx* ctx, void* p);
gprx_status gprx_device_upload(gprx_ctx* ctx, void* dst, const void* src, int64_t bytes);
gprx_status gprx_device_download(gprx_ctx* ctx, void* dst, const void* src, int64_t bytes);

/* ---- dense GP model ------------------------------------------------------------- */
/* Replaces the GaussianProcess<T> state (include/GaussianProcess.h:267-280). */
gprx_status gprx_model_create(gprx_ctx* ctx, gprx_dtype dtype, gprx_model** out);
void gprx_model_destroy(gprx_model* model);
/* AddSample x N (lib/GaussianProcess.cpp:36-51) as one upload: X is N x d, Y is N x m. */
gprx_status gprx_model_set_data(gprx_model* model, const void* X, const void* Y, int64_t n, int32_t d, int32_t m);
/* SetKernel (include/GaussianProcess.h:118-121). */
gprx_status gprx_model_set_kernel(gprx_model* model, const gprx_kernel_desc* kernel);
/* SetSigma (include/GaussianProcess.h:140-143): noise standard deviation. */
gprx_status gprx_model_set_noise(gprx_model* model, double sigma);

#define GPRX_FIT_DEFAULT 0u
#define GPRX_FIT_NO_LU_FALLBACK 1u /* report NOT_SPD instead of refactoring with LU.  By default a
                                      fit whose Cholesky meets a non-positive pivot is redone with
                                      a partial-pivot LU in double (the reference's default
                                      FullPivotLU = dgetrf_, include/LAPACKUtils.h:38-56,85-97);
                                      gprx_fit_info.method = 1 then.  An exactly singular matrix
                                      gives GPRX_ERR_SINGULAR (the reference returns non-finite
                                      regression vectors there) */
#define GPRX_FIT_DISTRIBUTED 2u    /* multi-GPU fit on a gprx_ctx_create_dist / _peer context
                                      (implied when world > 1; forces the path at world = 1): row
                                      blocks dealt in cyclic groups over the ranks (each GPU stores
                                      and builds only the lower tiles of its own rows, ~N^2/(2 world)),
                                      one persistent tile launch per rank; the exchange is device-
                                      initiated: the task that factors a diagonal block stores its
                                      inverse into every peer's IPC-mapped mailbox, the task that
                                      finishes a panel tile stores it into the receive windows of
                                      the ranks that read it (xGMI stores + flags; RCCL / the
                                      caller's collective only for host-side agreement).  Afterwards
                                      alpha, predict, the posterior covariance (the queries' forward
                                      solve sharded the same way, no N^2 on any rank) and the LML
                                      (value and gradient, GPRX_LML_DISTRIBUTED) run on it; the core
                                      matrix gathers the dense factor onto each process (the
                                      reference returns all of C) */
#define GPRX_FIT_F32_NO_REFINE 4u  /* fp32 models: skip the fp64 iterative refinement of alpha.  By
                                      default an fp32 fit factorises in fp32 and refines alpha in
                                      fp64 until it agrees with the double solve: the reference
                                      inverts fp32 GPs in double (include/LAPACKUtils.h:85-97) */
#define GPRX_FIT_FORCE_LU 8u       /* factor with the partial-pivot LU in double directly (no
                                      Cholesky first).  The reference's JacobiSVD / BDCSVD methods
                                      (lib/GaussianProcess.cpp:564-592) form V S^{-1} U^T with every
                                      singular value inverted, i.e. the exact inverse of a
                                      nonsingular K: no SVD is built here, the LU gives the same
                                      matrix to cond(K) eps (gpr::GaussianProcess maps those two
                                      methods to this flag; SelfAdjointEigenSolver is the
                                      reference's chol_invert, :594-612, the default path) */
/* Initialize (lib/GaussianProcess.cpp:118-130) = ComputeRegressionVectors (:642-672):
 * kernel matrix (:384-402) + noise (:375-381) + factorisation (replaces the default
 * lapack::lu_invert dgetrf_+dgetri_, include/LAPACKUtils.h:38-56,85-97) + regression
 * vectors alpha = (K + sigma^2 I)^{-1} Y (:661).  Everything stays in HBM; `info` may be
 * NULL. */
gprx_status gprx_model_fit(gprx_model* model, uint32_t flags, gprx_fit_info* info);
/* m_RegressionVectors (lib/GaussianProcess.cpp:661) -> host, N x m. */
gprx_status gprx_model_get_alpha(gprx_model* model, void* alpha);
/* Install regression vectors (n x m, row-major) read back by GaussianProcess::Load
 * (lib/GaussianProcess.cpp:184-268, which restores m_RegressionVectors from file rather
 * than recomputing them).  Enables predict.  The factor needed by posterior_cov / lml /
 * core_matrix is untouched: after set_data/kernel/noise it is rebuilt by gprx_model_fit,
 * which also overwrites alpha (re-install it afterwards to keep the loaded vectors). */
gprx_status gprx_model_set_alpha(gprx_model* model, const void* alpha);
/* Predict / PredictDerivative for q queries (lib/GaussianProcess.cpp:54-81, 684-706):
 * mean is q x m; deriv (optional, may be NULL) is q x d x m with the reference's formula
 * D(:,c) = -X^T (Kx o alpha_c) (:77-79). */
gprx_status gprx_model_predict(gprx_model* model, const void* Xq, int64_t q, void* mean, void* deriv);
/* operator()(x,y) = k(x,y) - Kx^T C Ky for q pairs (lib/GaussianProcess.cpp:84-99), via
 * the Cholesky factor: k(x,y) - (L^{-1}Kx).(L^{-1}Ky).  GetCredibleInterval (:102-114) is
 * 2*sqrt(max(0, out)) of the pair (x,x).  Non-finite kernel values give NaN, as the
 * reference's (no check in ComputeKernelVectorInternal, :684-693).
 * On a SHARDED fit of a multi-process context this is a COLLECTIVE call: every process calls
 * it (q = 0 and NULL pointers allowed for a process with no pairs).  The processes agree on
 * their arguments first: identical pairs are solved once; different ones (e.g. each process
 * its own query slice) are gathered, solved together, and each process receives its own. */
gprx_status gprx_model_posterior_cov(gprx_model* model, const void* Xa, const void* Xb, int64_t q, void* out);
/* The core matrix C = (K + sigma^2 I)^{-1} (m_CoreMatrix, lib/GaussianProcess.cpp:652)
 * materialised from the factor (potri) into host memory, N x N.  On a sharded fit of a
 * multi-process context a COLLECTIVE call (the dense factor is gathered from every rank). */
gprx_status gprx_model_core_matrix(gprx_model* model, void* C);

#define GPRX_LML_GRAD 1u   /* also compute the hyper-parameter gradient */
#define GPRX_LML_COMPAT 2u /* reproduce the reference's determinant narrowing + clamps
                              (include/Likelihood.h:77-79, 240-257); otherwise exact */
#define GPRX_LML_FORCE_LU 8u /* refit with GPRX_FIT_FORCE_LU (the SVD inversion methods) */
#define GPRX_LML_DISTRIBUTED 4u /* refit with GPRX_FIT_DISTRIBUTED (implied on a multi-rank or
                              virtual context): log det = sum of the ranks' diagonal blocks,
                              C = U U^T in tiles riding along in the sharded factorisation (no
                              rank holds N^2), each rank's gradient partial over its own row
                              blocks combined by one all-reduce of the P partials (SURVEY.md
                              8(e)).  A collective call on a multi-process context */
/* GaussianLogLikelihood::operator() / GetValueAndParameterDerivatives
 * (include/Likelihood.h:166-285) for m = 1: value = -1/2 y^T C y - 1/2 log det - N/2 log 2pi,
 * grad_p = 1/2 tr((alpha alpha^T - C) dK/dp).  Refits from scratch like the reference.
 * grad may be NULL; nparams receives the kernel's parameter count. */
gprx_status gprx_model_lml(gprx_model* model, uint32_t flags, double* value, double* grad, int32_t* nparams,
                           double* logdet);

/* SparseGaussianProcess::operator()(x,y) = k(x,y) - Kx^T Kmm^{-1} Ky + Kx^T RM Ky
 * (include/SparseGaussianProcess.h:94-106) on a model whose data are the inducing points:
 * W = Kmm^{-1} - RM (M x M, row-major, from gprx_sparse_fit) becomes resident, and
 * gprx_model_posterior_cov then evaluates q pairs on the device (two cross-kernel blocks, one
 * GEMM, one row dot). */
gprx_status gprx_model_set_sparse_cov(gprx_model* model, const void* W);

/* ---- kernels with no device form ----------------------------------------------------
 * The reference dispatches every pair through the virtual Kernel<T>::operator() /
 * GetDerivative (include/Kernel.h:52-59), so a user subclass works with the GP unchanged.
 * A kernel that cannot be lowered to gprx_kernel_desc is evaluated by the CALLER and handed
 * over as matrices (row-major, model dtype); the factorisation, solves, inverse and
 * reductions stay on the device.  gpr::GaussianProcess does this automatically for kernels
 * whose Describe() throws. */
/* K(X, X) (n x n, without the noise) in place of gprx_model_set_kernel; set the data first. */
gprx_status gprx_model_set_kernel_matrix(gprx_model* model, const void* K);
/* Predict / PredictDerivative from Kx = K(Xq, X) (q x n): mean q x m; deriv (optional,
 * needs Xq, q x d) q x d x m with the reference's D(:,c) = -Xd^T (Kx o alpha_c). */
gprx_status gprx_model_predict_kx(gprx_model* model, const void* Kx, const void* Xq, int64_t q, void* mean,
                                  void* deriv);
/* operator()(a_j, b_j) = kab_j - Kxa_j^T C Kxb_j for q pairs, Kxa = K(Xa, X), Kxb = K(Xb, X)
 * (q x n), kab = k(a_j, b_j) (q). */
gprx_status gprx_model_posterior_cov_kx(gprx_model* model, const void* Kxa, const void* Kxb, const void* kab,
                                        int64_t q, void* out);
/* gprx_model_lml with the gradient from the caller's derivative matrices dK (P x n x n,
 * dK_p = d K / d p_p, the reference's GetDerivative order). */
gprx_status gprx_model_lml_dk(gprx_model* model, uint32_t flags, const void* dK, int32_t P, double* value,
                              double* grad, double* logdet);

/* ---- building blocks (host buffers; used by parity tests) --------------------------- */
/* ComputeKernelMatrixInternal (lib/GaussianProcess.cpp:384-402): K = [k(x_i,x_j)], N x N. */
gprx_status gprx_kernel_matrix(gprx_ctx* ctx, gprx_dtype dtype, const gprx_kernel_desc* kernel, const void* X,
                               int64_t n, int32_t d, void* K);
/* Cross-covariance [k(a_i, b_j)] (include/SparseGaussianProcess.h:218-235). */
gprx_status gprx_cross_matrix(gprx_ctx* ctx, gprx_dtype dtype, const gprx_kernel_desc* kernel, const void* A,
                              int64_t na, const void* B, int64_t nb, int32_t d, void* K);
/* Stacked derivative matrices [D_0;...;D_{P-1}] (lib/GaussianProcess.cpp:472-495), P*N x N. */
gprx_status gprx_deriv_matrix(gprx_ctx* ctx, gprx_dtype dtype, const gprx_kernel_desc* kernel, const void* X,
                              int64_t n, int32_t d, void* D);
/* In-place lower Cholesky of an SPD N x N matrix (replaces dpotrf_ 'L',
 * include/LAPACKUtils.h:64).  Row-major in/out; the strict upper triangle of the output is
 * zeroed.  *info as LAPACK: 0 or the 1-based column of the first non-positive pivot. */
gprx_status gprx_cholesky(gprx_ctx* ctx, gprx_dtype dtype, void* A, int64_t n, int32_t* info);
/* In-place explicit inverse of an SPD matrix via potrf + potri (replaces
 * lapack::chol_invert, include/LAPACKUtils.h:59-73,100-111). */
gprx_status gprx_spd_inverse(gprx_ctx* ctx, gprx_dtype dtype, void* A, int64_t n, int32_t* info);

/* ---- sparse GP (subset of regressors) ----------------------------------------------- */
/* SparseGaussianProcess::PreComputeRegression (include/SparseGaussianProcess.h:274-313)
 * without the N x N core matrix (:309-311, infeasible at N = 1e6): returns Kmm^{-1}
 * (M x M), the regression vectors RV (M x m) and the regression matrix RM (M x M), all
 * host, row-major.  Any pointer may be NULL. */
/* (X, Y and Xm may be host or device memory: unified addressing decides the copy's direction, so
 * samples already resident in HBM are read without a PCIe transfer.) */
gprx_status gprx_sparse_fit(gprx_ctx* ctx, gprx_dtype dtype, const gprx_kernel_desc* kernel, const void* X,
                            const void* Y, int64_t n, int32_t d, int32_t m, const void* Xm, int64_t M,
                            double sigma, double jitter, void* Kinv, void* RV, void* RM);

/* SparseGaussianLogLikelihood::operator() / GetValueAndParameterDerivatives
 * (include/SparseLikelihood.h:113-344) for m = 1, in O(N M^2) (Woodbury on the Nystrom
 * covariance sigma^2 I + Knm Kmm^{-1} Kmn; the reference's N x N C_inv and derivative stacks
 * are never formed): value = -1/2 y^T C^{-1} y - 1/2 log|C| - N/2 log 2pi, grad_p over the
 * kernel parameters (the noise is not differentiated, as in the reference).  flags:
 * GPRX_LML_GRAD, GPRX_LML_COMPAT (the reference's long-double determinant product and its
 * clamps, :132-158, 305-314; otherwise exact).  logdet receives log|C|.  On an RCCL context
 * each rank passes its share of the dense rows (as gprx_sparse_fit). */
gprx_status gprx_sparse_lml(gprx_ctx* ctx, gprx_dtype dtype, const gprx_kernel_desc* kernel, const void* X,
                            const void* Y, int64_t n, int32_t d, int32_t m, const void* Xm, int64_t M, double sigma,
                            double jitter, uint32_t flags, double* value, double* grad, int32_t* nparams,
                            double* logdet);

#ifdef __cplusplus
}
#endif
#endif /* GPRX_H */
