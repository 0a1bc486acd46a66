// gprx_api.cpp — the C ABI of libgprx (include/gprx.h): contexts, resident models and the
// host-side orchestration of the HIP kernels.  No entry point throws across the ABI.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <climits>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "gprx_dist.h"
#include "gprx_internal.h"
#include "../../include/gprx_dev.h"

namespace gprx {

// ---- extra launchers (k_predict.hip, k_lml.hip) -----------------------------------------
template <typename T>
void launch_pair_kernel(const KCanon<T>& K, const T* Xa, const T* Xb, int64_t q, int d, T* out, hipStream_t s);
template <typename T>
void launch_rowdot(const T* Va, const T* Vb, int64_t ld, int64_t q, int64_t n, const T* kab, T* out, hipStream_t s);
template <typename T>
void trsm_rows(const T* A, int64_t ldA, int64_t np, const T* Linv, T* R, int64_t ld, int64_t qp, hipStream_t s);
template <typename T>
void launch_spd_inverse_from_factor(const T* A, int64_t ldA, int64_t np, const T* Linv, T* V, T* C, hipStream_t s);
template <typename T>
void launch_lml_grad(const KCanon<T>& K, const T* X, const T* tab, int64_t n, int d, const T* alpha, const T* C,
                     int64_t ldc, double* acc /* MAX_LEAF*3 */, hipStream_t s);
template <typename T>
void launch_set_identity_pad(T* A, int64_t ld, int64_t n, int64_t np, hipStream_t s);
template <typename T>
void launch_gemm_add_lower(T* S, int64_t lds, const T* K, int64_t ldk, int64_t n, hipStream_t s);
template <typename T>
void launch_sym_fill(T* C, int64_t ldc, int64_t n, hipStream_t s);
template <typename T>
void launch_sum_partials(T* S, int64_t stride, int P, hipStream_t s);

gprx_status gprx_dev_bench_impl(gprx_dtype dtype, int32_t what, int64_t M, int64_t N, int64_t K, int32_t iters,
                                double* ms, Exec* ex);

static thread_local std::string t_last_error;
thread_local Prof* g_prof = nullptr;

// ---------------------------------------------------------------------------------------
// canonical kernel form
// ---------------------------------------------------------------------------------------
static int leaf_nparams(int op) {
    switch (op) {
        case GPRX_K_GAUSSIAN:
        case GPRX_K_GAUSSIAN_EXP:
            return 2;
        case GPRX_K_WHITE:
            return 1;
        case GPRX_K_RATIONAL_QUADRATIC:
        case GPRX_K_PERIODIC:
            return 3;
    }
    return 0;
}

template <typename T>
std::string canonicalize(const gprx_kernel_desc& desc, KCanon<T>& K) {
    std::memset(&K, 0, sizeof(K));
    if (desc.n_nodes <= 0 || desc.n_nodes > GPRX_MAX_KNODES) return "kernel descriptor: bad node count";
    std::vector<std::vector<unsigned>> st;
    int nleaf = 0, nparams = 0, nper = 0;
    bool r2 = false;
    for (int i = 0; i < desc.n_nodes; i++) {
        const gprx_knode& nd = desc.node[i];
        const int op = nd.op;
        if (op == GPRX_K_SUM || op == GPRX_K_PRODUCT) {
            if (st.size() < 2) return "kernel descriptor: malformed post-order program";
            std::vector<unsigned> b = st.back();
            st.pop_back();
            std::vector<unsigned> a = st.back();
            st.pop_back();
            std::vector<unsigned> r;
            if (op == GPRX_K_SUM) {
                r = a;
                r.insert(r.end(), b.begin(), b.end());
            } else {
                for (unsigned ta : a)
                    for (unsigned tb : b) r.push_back(ta | tb);
            }
            if ((int)r.size() > MAX_TERM) return "kernel descriptor: too many product terms for the device form";
            st.push_back(r);
            continue;
        }
        const int np = leaf_nparams(op);
        if (np == 0) return "kernel descriptor: unknown node op";
        if (nleaf >= MAX_LEAF) return "kernel descriptor: too many leaf kernels for the device form";
        KLeaf<T>& L = K.leaf[nleaf];
        const T p0 = (T)nd.p[0], p1 = (T)nd.p[1], p2 = (T)nd.p[2];
        L.p[0] = p0;
        L.p[1] = p1;
        L.p[2] = p2;
        switch (op) {
            case GPRX_K_GAUSSIAN:  // include/Kernel.h:529-537
                if (p0 == T(0)) return "GaussianKernel: sigma has to be positive";
                if (p1 == T(0)) return "GaussianKernel: scale has to be positive";
                L.type = L_GAUSS;
                L.c0 = p1 * p1;
                L.c1 = T(-0.5) / (p0 * p0);
                r2 = true;
                break;
            case GPRX_K_GAUSSIAN_EXP: {
                const T es = std::exp(p1), eg = std::exp(p0);
                L.type = L_GAUSS_EXP;
                L.c0 = es * es;
                L.c1 = T(-0.5) / (eg * eg);
                r2 = true;
                break;
            }
            case GPRX_K_WHITE:
                L.type = L_WHITE;
                L.c0 = p0 * p0;
                r2 = true;
                break;
            case GPRX_K_RATIONAL_QUADRATIC:
                L.type = L_RQ;
                L.c0 = p0 * p0;
                L.c1 = T(0.5) / (p1 * p1 * p2);
                L.c2 = p2;
                r2 = true;
                break;
            case GPRX_K_PERIODIC:  // include/Kernel.h:1003-1005
                if (p0 == T(0)) return "PeriodicKernel: scale parameter has to be positive.";
                if (p1 == T(0)) return "PeriodicKernel: period length parameter has to be positive.";
                if (p2 == T(0)) return "PeriodicKernel: sigma parameter has to be positive.";
                if (nper >= MAX_PER) return "kernel descriptor: at most 2 periodic leaves on the device";
                L.type = L_PERIODIC;
                L.pslot = nper;
                K.b[nper] = p1;
                nper++;
                L.c0 = p0 * p0;
                L.c1 = T(-0.5) / (p2 * p2);
                break;
        }
        // the folded exp constants (fexp_fold: f64 predict epilogue only)
        L.fold = 0;
        L.f1 = L.f0 = T(0);
        if (std::is_same<T, double>::value && (L.type == L_GAUSS || L.type == L_GAUSS_EXP || L.type == L_PERIODIC) &&
            L.c0 > T(0) && std::isfinite(std::log((double)L.c0))) {
            constexpr double kS = 92.33248261689366;  // 64 / ln 2
            L.f1 = (T)((double)L.c1 * kS);
            L.f0 = (T)(std::log((double)L.c0) * kS);
            L.fold = 1;
        }
        K.param_base[nleaf] = nparams;
        nparams += np;
        st.push_back(std::vector<unsigned>{1u << nleaf});
        nleaf++;
    }
    if (st.size() != 1) return "kernel descriptor: malformed post-order program";
    K.nleaf = nleaf;
    K.nterm = (int)st[0].size();
    K.sum_leaves = 1;
    for (int t = 0; t < K.nterm; t++) {
        K.term_mask[t] = st[0][t];
        if (st[0][t] != (1u << t)) K.sum_leaves = 0;
    }
    K.nper = nper;
    K.need_r2 = r2 ? 1 : 0;
    K.nparams = nparams;
    if (nparams > GPRX_MAX_KPARAMS) return "kernel descriptor: too many parameters";
    return "";
}
template std::string canonicalize<float>(const gprx_kernel_desc&, KCanon<float>&);
template std::string canonicalize<double>(const gprx_kernel_desc&, KCanon<double>&);

// ---------------------------------------------------------------------------------------
// device buffers
// ---------------------------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    void ensure(size_t b) {
        if (b <= bytes && p) return;
        release();
        if (b == 0) return;
        GPRX_HIP(hipMalloc(&p, b));
        bytes = b;
        // GPRX_POISON (debugging): fresh buffers hold finite garbage (bytes 0x41: 12.1f, 2.3e6),
        // as reused memory does, so a read of unwritten memory shows in the results
        static const bool poison = std::getenv("GPRX_POISON") != nullptr;
        if (poison) GPRX_HIP(hipMemset(p, 0x41, b));
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename T>
    T* as() const {
        return reinterpret_cast<T*>(p);
    }
    ~DevBuf() { release(); }
};

// Pinned host memory, mapped: the fit's status words come back by one kernel's stores into it
// and one stream synchronisation (three synchronous hipMemcpy calls were three copy launches
// and a host round trip each)
struct PinnedBuf {
    void* p = nullptr;
    double* dev = nullptr;  // the device's address of it (mapped, coherent)
    size_t bytes = 0;
    void ensure(size_t b) {
        if (b <= bytes && p) return;
        release();
        GPRX_HIP(hipHostMalloc(&p, b, hipHostMallocMapped | hipHostMallocCoherent));
        void* d = nullptr;
        GPRX_HIP(hipHostGetDevicePointer(&d, p, 0));
        dev = static_cast<double*>(d);
        bytes = b;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        dev = nullptr;
        bytes = 0;
    }
    ~PinnedBuf() { release(); }
};

// Device copy of a small parameter struct, uploaded only when its bytes change (a pageable
// hipMemcpyAsync blocks the host until the stream reaches it: every fit paid that wait between
// its feature kernels and the factorisation launch)
struct DevParam {
    DevBuf buf;
    std::vector<unsigned char> last;
    template <typename S>
    const S* put(const S& v, hipStream_t s) {
        const bool fresh = buf.bytes < sizeof(S) || !buf.p;
        buf.ensure(sizeof(S));
        const unsigned char* b = reinterpret_cast<const unsigned char*>(&v);
        if (fresh || last.size() != sizeof(S) || std::memcmp(last.data(), b, sizeof(S)) != 0) {
            GPRX_HIP(hipMemcpyAsync(buf.p, &v, sizeof(S), hipMemcpyHostToDevice, s));
            last.assign(b, b + sizeof(S));
        }
        return buf.as<S>();
    }
};

static int64_t round_up(int64_t x, int64_t g) { return (x + g - 1) / g * g; }

}  // namespace gprx

using namespace gprx;

// info < 0: the device scheduler of potrf_tiles timed out waiting for a dependency
static void check_sched(int hinfo) {
    if (hinfo < 0) throw Error{GPRX_ERR_HIP, "gprx: device factorisation scheduler timed out (tile dependency wait)"};
}

struct gprx_ctx {
    int device = 0;
    int rank = 0, world = 1;
    bool virt = false;          // gprx_ctx_create_virtual: world virtual ranks in this process
    ncclComm_t comm = nullptr;  // RCCL communicator (gprx_ctx_create_dist), world > 1
    HostColl* hc = nullptr;     // host collectives of a multi-process context (RCCL or the caller's)
    bool peer = false;          // gprx_ctx_create_peer: the caller's collective, no RCCL
    int cu_slot = 0, cu_slots = 1;  // GPRX_DIST_SHARED_GPU: ranks of one GPU split its CUs
    hipStream_t stream = nullptr;
    hipStream_t aux = nullptr;  // look-ahead stream of the factorisation
    hipStream_t aux2 = nullptr;  // second look-ahead stream (next panel's later columns)
    Exec ex;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
    Prof prof;
    std::shared_ptr<void> sparse_state[2];  // the sparse fit's device buffers per scalar type (sparse_state)
    std::string err;
    std::mutex mu;
};

// Per-call profiler binding: sets the thread's current profiler and resolves the
// recorded events (after draining both streams) when the call returns.
struct ProfBind {
    gprx_ctx* ctx;
    explicit ProfBind(gprx_ctx* c) : ctx(c) { g_prof = (c && c->prof.on) ? &c->prof : nullptr; }
    ~ProfBind() {
        if (ctx && ctx->prof.on) {
            (void)hipStreamSynchronize(ctx->stream);
            (void)hipStreamSynchronize(ctx->aux);
            (void)hipStreamSynchronize(ctx->aux2);
            ctx->prof.resolve();
        }
        g_prof = nullptr;
    }
};

struct gprx_model {
    gprx_ctx* ctx = nullptr;
    gprx_dtype dt = GPRX_F64;
    int64_t n = 0;
    int d = 0, m = 0;
    int64_t np = 0, mp = 0, ld = 0;
    double sigma = 0;
    bool has_data = false, has_kernel = false, fitted = false;
    bool has_alpha = false;  // regression vectors valid (fit, or gprx_model_set_alpha after Load)
    bool want_inv = false;   // the next fit also forms C = (K + s^2 I)^{-1} (identity rows in the tiles)
    bool inv_ready = false;  // C holds the inverse of the current fit
    gprx_kernel_desc desc{};
    KCanon<double> kd{};
    KCanon<float> kf{};
    DevBuf X, Y, tab, A, Linv, z, alpha, info, flag, red, V, C, scratch1, scratch2, grad, pack, featU, featV, kdev;
    // posterior covariance workspace (L^{-1} K(X, x) for a query batch: qp x np each), kept
    // across calls -- at Q = 65536, N = 16384 one buffer is 8.6 GB, whose hipMalloc + free per
    // call cost more than the solve on some boxes
    DevBuf pvRa, pvRb, pvFq;  // (+ the queries' pair features)
    // a refit, an LML call or new data frees that workspace when it is large (one
    // big variance call must not leave too little HBM for the next fit on the device)
    void trim_posterior_workspace() {
        if (pvRa.bytes + pvRb.bytes + pvFq.bytes > (size_t(1) << 30)) {
            pvRa.release();
            pvRb.release();
            pvFq.release();
        }
    }
    DevParam kfit;     // the fit's kernel tree (uploaded when it changes)
    PinnedBuf hstat;   // the fit's status words: flag, info, log det, data fit
    // fp32 models: fp64 iterative refinement state (k_refine.hip).  kd then holds the tree in
    // double with the parameters rounded to float first (the reference stores them in T).
    DevBuf Xd, Yd, ad, kxd, fud, fvd, kdev64, tabd, zd, outd, delta, nrm;
    // LU fallback state (k_getrf.hip), double for both scalar types: the factored matrix,
    // pivots, the 128-block inverses of L and U, and scratch
    int method = 0;  // factor of the current fit: 0 Cholesky (A, Linv), 1 LU (lu, ipiv, luL, luU)
    DevBuf lu, ipiv, luUt, luB, lured;
    double lu_sign = 1;  // sign of det(K + sigma^2 I) from the LU
    // distributed fit (gprx_dist.cpp): the engine (per-rank buffers, schedules) and whether
    // the current fit is one (its factor is held in tiles per rank: alpha and predict only)
    DistEngineBase* dist_engine = nullptr;
    bool dist_fitted = false;
    bool dist_dense = false;  // the tiles of a distributed fit gathered into A (ld np) and Linv
    bool dist_inv_tiles = false;  // LML-mode distributed fit: C in the ranks' tiles (dist_lml_grad)
    DistFitOut dist_stats;        // layout, window and memory of the last distributed fit
    // a kernel with no device form: the caller evaluated K (n x n, row-major, T) -- the
    // reference's virtual Kernel<T>::operator() (include/Kernel.h:52-59); see k_hostk.hip
    bool host_k = false;
    DevBuf Kext;
    // a sparse GP's variance state (gprx_model_set_sparse_cov): the model holds the inducing
    // points and W = Kmm^{-1} - RM (padded np x np, column-major) for
    // operator()(x,y) = k(x,y) - Kx^T W Ky (include/SparseGaussianProcess.h:94-106)
    bool sparse_cov = false;
    DevBuf sparseW;
    std::mutex mu;
    ~gprx_model() { dist_engine_free(dist_engine); }
};

// Every model call holds its context's mutex, then the model's (always in that order): the
// device work of a model runs on the context's streams and uses the context's scratch (the
// tile factorisation's ticket and counter words, its cached schedules, the timing events),
// so two models of one context must not interleave their launches -- a second fit's memset
// of the ticket counter landing between another fit's memset and launch leaves that launch
// with a spent ticket.  Calls on one model from several threads are serialised as well.
struct ModelLock {
    std::lock_guard<std::mutex> c, m;
    explicit ModelLock(gprx_model* M) : c(M->ctx->mu), m(M->mu) {}
};

// ---------------------------------------------------------------------------------------
// error plumbing
// ---------------------------------------------------------------------------------------
static gprx_status fail(gprx_ctx* ctx, gprx_status st, const std::string& msg) {
    t_last_error = msg;
    if (ctx) ctx->err = msg;
    return st;
}

#define API_BEGIN try {
#define API_END(ctx)                                                                   \
    }                                                                                  \
    catch (const gprx::Error& e) {                                                     \
        return fail(ctx, e.st, e.msg);                                                 \
    }                                                                                  \
    catch (const std::exception& e) {                                                  \
        return fail(ctx, GPRX_ERR_HIP, e.what());                                      \
    }                                                                                  \
    catch (...) {                                                                      \
        return fail(ctx, GPRX_ERR_HIP, "unknown exception");                           \
    }

static size_t esize(gprx_dtype dt) { return dt == GPRX_F64 ? sizeof(double) : sizeof(float); }

template <typename T>
static const KCanon<T>& kcanon(const gprx_model* m);
template <>
const KCanon<double>& kcanon<double>(const gprx_model* m) {
    return m->kd;
}
template <>
const KCanon<float>& kcanon<float>(const gprx_model* m) {
    return m->kf;
}

// ---------------------------------------------------------------------------------------
// fp64 iterative refinement of an fp32 fit (k_refine.hip): alpha_d += (L L^T)^{-1}
// (Y - (K + s2 I) alpha_d) with K evaluated in fp64 (pair statistics of the fp64-widened
// samples, the predict path with the training set as the queries) and the correction solved
// with the fp32 factor already in A (forward solve of the residual written into the label
// rows, back substitution).  Stops when the correction is below fp32 resolution of alpha.
// ---------------------------------------------------------------------------------------
static void download(void* host, const void* dev, size_t bytes, hipStream_t s);

static void refine_f32(gprx_model* M, gprx_fit_info* out) {
    gprx_ctx* ctx = M->ctx;
    hipStream_t s = ctx->stream;
    const KCanon<double>& K = M->kd;
    const int64_t n = M->n, np = M->np, mp = M->mp, ld = M->ld;
    const int d = M->d, m = M->m;
    int steps = 3;
    if (const char* e = std::getenv("GPRX_REFINE_STEPS")) steps = std::max(0, std::atoi(e));
    GPRX_HIP(hipEventRecord(ctx->ev[0], s));
    M->Xd.ensure(sizeof(double) * n * d);
    M->Yd.ensure(sizeof(double) * n * m);
    M->ad.ensure(sizeof(double) * n * m);
    M->kxd.ensure(sizeof(double) * n * m);
    M->delta.ensure(sizeof(float) * np * m);
    M->nrm.ensure(2 * sizeof(unsigned long long));
    launch_convert<float, double>(M->X.as<float>(), M->Xd.as<double>(), n * d, s);
    launch_convert<float, double>(M->Y.as<float>(), M->Yd.as<double>(), n * m, s);
    launch_convert<float, double>(M->alpha.as<float>(), M->ad.as<double>(), n * m, s);
    const bool mma = pairs_mma_supported<double>(K, 1);
    if (mma) {
        const int64_t kf = pairs_feature_cols<double>(K, d);
        M->fud.ensure(sizeof(double) * np * kf);
        M->fvd.ensure(sizeof(double) * np * kf);
        launch_pair_features<double>(K, M->Xd.as<double>(), n, d, M->Xd.as<double>(), false, M->fud.as<double>(), np, s);
        launch_pair_features<double>(K, M->Xd.as<double>(), n, d, M->Xd.as<double>(), true, M->fvd.as<double>(), np, s);
        M->kdev64.ensure(sizeof(KCanon<double>));
        GPRX_HIP(hipMemcpyAsync(M->kdev64.p, &K, sizeof(KCanon<double>), hipMemcpyHostToDevice, s));
    } else {
        if (K.nper > 0) {
            M->tabd.ensure(sizeof(double) * 2 * K.nper * n * d);
            launch_sincos_tables<double>(K, M->Xd.as<double>(), n, d, M->tabd.as<double>(), s);
        }
        M->zd.ensure(sizeof(double) * n * m);
        M->outd.ensure(sizeof(double) * n * m);
    }
    const float sf = (float)M->sigma;
    const double s2 = (double)(sf * sf);  // m_Sigma * m_Sigma in T (lib/GaussianProcess.cpp:379)
    double rel = 0;
    int taken = 0;
    for (int it = 0; it < steps; it++) {
        if (mma) {
            for (int c = 0; c < m; c++)  // one label column per launch (alpha, Kx strided by m)
                launch_predict_mma<double>(K, M->kdev64.as<KCanon<double>>(), M->fud.as<double>(), np,
                                           M->fvd.as<double>(), np, d, M->ad.as<double>() + c, n, m, n,
                                           M->kxd.as<double>() + c, s);
        } else {
            launch_predict<double>(K, M->Xd.as<double>(), M->tabd.as<double>(), n, d, m, M->ad.as<double>(),
                                   M->Xd.as<double>(), M->tabd.as<double>(), n, M->kxd.as<double>(), nullptr,
                                   M->zd.as<double>(), M->outd.as<double>(), s);
        }
        launch_residual_rows(M->Yd.as<double>(), M->kxd.as<double>(), M->ad.as<double>(), s2, n, m,
                             M->A.as<float>(), ld, np, np, (int)mp, s);
        GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)M->info.p, INT_MAX, 1, s));
        launch_forward_chain<float>(M->A.as<float>(), ld, np, m, M->Linv.as<float>(), M->info.as<int>(), ctx->ex, s);
        launch_backsolve_chain<float>(M->A.as<float>(), ld, np, m, M->Linv.as<float>(), M->delta.as<float>(),
                                      M->info.as<int>(), ctx->ex, s);
        launch_refine_accumulate(M->delta.as<float>(), M->ad.as<double>(), M->alpha.as<float>(), n * m,
                                 M->nrm.as<unsigned long long>(), s);
        unsigned long long h[2];
        int hinfo = 0;
        download(h, M->nrm.p, sizeof(h), s);
        download(&hinfo, M->info.p, sizeof(int), s);
        check_sched(hinfo);
        double dn, an;
        std::memcpy(&dn, &h[0], sizeof(double));
        std::memcpy(&an, &h[1], sizeof(double));
        rel = an > 0 ? dn / an : dn;
        taken = it + 1;
        if (!(rel > 0x1p-26)) break;  // below fp32 resolution of alpha (NaN: stop too)
    }
    GPRX_HIP(hipEventRecord(ctx->ev[1], s));
    GPRX_HIP(hipEventSynchronize(ctx->ev[1]));
    if (out) {
        float ms = 0;
        hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]);
        out->ms_refine = ms;
        out->refine_delta = rel;
        out->refine_steps = taken;
    }
}

// ---------------------------------------------------------------------------------------
// LU fallback (k_getrf.hip): K + sigma^2 I rebuilt in full, factored with partial pivoting in
// double, alpha = A^{-1} Y by the two triangular solves.  The reference's default inversion
// is exactly this LU (dgetrf_ on the matrix cast to double, include/LAPACKUtils.h:38-56,
// 85-97); it reaches here only when the Cholesky met a non-positive pivot.
// ---------------------------------------------------------------------------------------
template <typename T>
static void lu_build_matrix(gprx_model* M) {
    hipStream_t s = M->ctx->stream;
    const KCanon<T>& K = kcanon<T>(M);
    const int64_t n = M->n, np = M->np;
    const T sig = (T)M->sigma;
    const T sigma2 = sig * sig;  // in T, as the reference (lib/GaussianProcess.cpp:379)
    M->lu.ensure(sizeof(double) * np * np);
    GPRX_HIP(hipMemsetAsync(M->flag.p, 0, sizeof(int), s));
    if (M->host_k) {  // the caller's K, widened to double like lu_invert<float> (LAPACKUtils.h:85-97)
        if constexpr (std::is_same<T, double>::value) {
            launch_kext_build<double>(M->Kext.as<double>(), n, M->lu.as<double>(), np, np, sigma2, M->flag.as<int>(), s);
        } else {
            M->A.ensure(sizeof(float) * np * np);
            launch_kext_build<float>(M->Kext.as<float>(), n, M->A.as<float>(), np, np, sigma2, M->flag.as<int>(), s);
            launch_convert<float, double>(M->A.as<float>(), M->lu.as<double>(), np * np, s);
        }
        return;
    }
    if constexpr (std::is_same<T, double>::value) {
        launch_kbuild<double>(K, M->X.as<double>(), M->tab.as<double>(), n, M->X.as<double>(), M->tab.as<double>(), n,
                              M->d, M->lu.as<double>(), np, np, true, sigma2, M->flag.as<int>(), s);
    } else {  // K evaluated in float (the reference's T), then widened: lu_invert<float> casts to double
        M->A.ensure(sizeof(float) * np * np);
        launch_kbuild<float>(K, M->X.as<float>(), M->tab.as<float>(), n, M->X.as<float>(), M->tab.as<float>(), n,
                             M->d, M->A.as<float>(), np, np, true, sigma2, M->flag.as<int>(), s);
        launch_convert<float, double>(M->A.as<float>(), M->lu.as<double>(), np * np, s);
    }
    launch_sym_fill<double>(M->lu.as<double>(), np, np, s);
}

template <typename T>
static void lu_fit(gprx_model* M, gprx_fit_info* out) {
    gprx_ctx* ctx = M->ctx;
    hipStream_t s = ctx->stream;
    const int64_t n = M->n, np = M->np;
    const int m = M->m;
    GPRX_HIP(hipEventRecord(ctx->ev[0], s));
    lu_build_matrix<T>(M);
    M->ipiv.ensure(sizeof(int) * np);
    M->luUt.ensure(sizeof(double) * np * DB);
    M->luB.ensure(sizeof(double) * np * m);
    M->lured.ensure(sizeof(double) * 4);
    GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)M->info.p, INT_MAX, 1, s));
    GPRX_HIP(hipEventRecord(ctx->ev[1], s));
    lu_factor(M->lu.as<double>(), np, np, M->ipiv.as<int>(), M->info.as<int>(), M->luUt.as<double>(), s);
    GPRX_HIP(hipEventRecord(ctx->ev[2], s));
    lu_rhs_from_rows<T>(M->Y.as<T>(), n, m, M->luB.as<double>(), np, np, s);
    lu_solve(M->lu.as<double>(), np, np, M->ipiv.as<int>(), M->luB.as<double>(), np, m, s);
    M->alpha.ensure(sizeof(T) * np * m);
    lu_rows_from_rhs<T>(M->luB.as<double>(), np, n, m, M->alpha.as<T>(), s);
    lu_logdet(M->lu.as<double>(), np, n, M->ipiv.as<int>(), M->lured.as<double>(), s);
    GPRX_HIP(hipEventRecord(ctx->ev[3], s));
    int hflag = 0, hinfo = 0;
    double red[3];
    download(&hflag, M->flag.p, sizeof(int), s);
    download(&hinfo, M->info.p, sizeof(int), s);
    download(red, M->lured.p, sizeof(red), s);
    if (hflag)
        throw Error{GPRX_ERR_NONFINITE,
                    "GaussianProcess::ComputeKernelMatrixInternal: kernel matrix contains entries which are not finite."};
    if (hinfo != INT_MAX)
        throw Error{GPRX_ERR_SINGULAR, "gprx: kernel matrix is singular (LU pivot " + std::to_string(hinfo) +
                                           " is zero; the reference's dgetrf_ fails there too)"};
    // data fit y^T (K + s^2 I)^{-1} y from alpha (the host copies are small next to the factor)
    std::vector<T> ha((size_t)n * m), hy((size_t)n * m);
    download(ha.data(), M->alpha.p, sizeof(T) * n * m, s);
    download(hy.data(), M->Y.p, sizeof(T) * n * m, s);
    double df = 0;
    for (size_t e = 0; e < ha.size(); e++) df += (double)hy[e] * (double)ha[e];
    M->method = 1;
    M->lu_sign = red[1];
    M->fitted = true;
    M->has_alpha = true;
    M->inv_ready = false;
    if (out) {
        float t01 = 0, t12 = 0, t23 = 0;
        hipEventElapsedTime(&t01, ctx->ev[0], ctx->ev[1]);
        hipEventElapsedTime(&t12, ctx->ev[1], ctx->ev[2]);
        hipEventElapsedTime(&t23, ctx->ev[2], ctx->ev[3]);
        out->ms_build += t01;
        out->ms_factor += t12;
        out->ms_solve += t23;
        out->logdet = red[0];  // log |det|; the sign is the model's lu_sign
        out->datafit = df;
        out->method = 1;
    }
}

// A^{-1} B for m right-hand sides already in M->luB-shaped column-major storage (np x m)
static void lu_solve_model(gprx_model* M, double* B, int m) {
    lu_solve(M->lu.as<double>(), M->np, M->np, M->ipiv.as<int>(), B, M->np, m, M->ctx->stream);
}

// ---------------------------------------------------------------------------------------
// distributed fit (gprx_dist.cpp): row blocks dealt over the ranks, one persistent tile
// launch per rank, RCCL broadcast of each diagonal inverse and full-mesh panel exchange
// ---------------------------------------------------------------------------------------
template <typename T>
static void model_inverse(gprx_model* M);

// The LU in double on this process's full copy of the samples (np x np workspace): the
// GPRX_FIT_FORCE_LU path, and the NOT_SPD fallback of a distributed fit, where every rank
// computes the same factor from its replicated X, Y.
template <typename T>
static void lu_fit_replicated(gprx_model* M, gprx_fit_info* out) {
    hipStream_t s = M->ctx->stream;
    const KCanon<T>& K = kcanon<T>(M);
    const int64_t np0 = round_up(M->n, (int64_t)DB);
    M->np = np0;
    M->mp = round_up(M->m, GT);
    M->ld = np0;
    M->fitted = M->has_alpha = M->inv_ready = M->dist_fitted = M->dist_dense = false;
    M->info.ensure(sizeof(int));
    M->flag.ensure(sizeof(int));
    M->alpha.ensure(sizeof(T) * np0 * M->m);
    if (K.nper > 0 && !M->host_k) {
        M->tab.ensure(sizeof(T) * 2 * K.nper * M->n * M->d);
        launch_sincos_tables<T>(K, M->X.as<T>(), M->n, M->d, M->tab.as<T>(), s);
    }
    if (out) std::memset(out, 0, sizeof(*out));
    lu_fit<T>(M, out);
}

// The dense factor of a distributed fit on this process, for the calls that need the whole
// factor (the core matrix -- the reference returns all of C -- and the VALU gradient's C; the
// posterior covariance solves across the ranks instead, model_posterior_cov_dist): gathered once per
// fit from every rank's packed rows (device reads through the mappings of the mailboxes'
// storage) into A (ld np) and Linv.  The one place a sharded fit holds N^2 on a process.
template <typename T>
static void ensure_dense_factor(gprx_model* M) {
    if (!M->dist_fitted || M->dist_dense) return;
    const int64_t np = M->np;
    M->ld = np;
    M->A.ensure(sizeof(T) * np * np);
    M->Linv.ensure(sizeof(T) * np * DB);
    dist_gather_factor<T>(M->dist_engine, M->A.as<T>(), np, M->Linv.as<T>(), M->ctx->stream);
    M->dist_dense = true;
}

// fp64 iterative refinement of a SHARDED fp32 fit (the single-GPU refine_f32 restated over the
// ranks): each process evaluates the fp64 residual r = Y - (K + s2 I) alpha_d only at the rows
// its ranks own (pair statistics of those rows against all n samples), the correction
// (L L^T)^{-1} r runs as the sharded forward + back substitutions (k_dsolve.hip) and arrives on
// every rank, alpha_d += delta everywhere (identical: no reduction needed).
static void refine_f32_dist(gprx_model* M, gprx_fit_info* out) {
    gprx_ctx* ctx = M->ctx;
    hipStream_t s = ctx->stream;
    const KCanon<double>& K = M->kd;
    const int64_t n = M->n, np = M->np;
    const int d = M->d, m = M->m;
    int steps = 3;
    if (const char* e = std::getenv("GPRX_REFINE_STEPS")) steps = std::max(0, std::atoi(e));
    GPRX_HIP(hipEventRecord(ctx->ev[0], s));
    // the rows this process's ranks own
    std::vector<int64_t> idx;
    for (int b : dist_own_blocks(M->dist_engine))
        for (int64_t r = (int64_t)b * DB; r < std::min<int64_t>(n, (int64_t)(b + 1) * DB); r++) idx.push_back(r);
    const int64_t q = (int64_t)idx.size(), qp = round_up(std::max<int64_t>(q, 1), GT);
    DevBuf didx, Xo, fuo, kxo, rhs;
    didx.ensure(sizeof(int64_t) * std::max<int64_t>(q, 1));
    GPRX_HIP(hipStreamSynchronize(s));
    if (q) GPRX_HIP(hipMemcpy(didx.p, idx.data(), sizeof(int64_t) * q, hipMemcpyHostToDevice));
    M->Xd.ensure(sizeof(double) * n * d);
    M->Yd.ensure(sizeof(double) * n * m);
    M->ad.ensure(sizeof(double) * n * m);
    M->delta.ensure(sizeof(float) * np * m);
    M->nrm.ensure(2 * sizeof(unsigned long long));
    kxo.ensure(sizeof(double) * qp * m);
    rhs.ensure(sizeof(float) * np * m);
    launch_convert<float, double>(M->X.as<float>(), M->Xd.as<double>(), n * d, s);
    launch_convert<float, double>(M->Y.as<float>(), M->Yd.as<double>(), n * m, s);
    launch_convert<float, double>(M->alpha.as<float>(), M->ad.as<double>(), n * m, s);
    Xo.ensure(sizeof(double) * std::max<int64_t>(q, 1) * d);
    launch_gather_rows(M->Xd.as<double>(), didx.as<int64_t>(), q, d, Xo.as<double>(), s);
    const bool mma = pairs_mma_supported<double>(K, 1);
    if (mma) {
        const int64_t kf = pairs_feature_cols<double>(K, d);
        fuo.ensure(sizeof(double) * qp * kf);
        M->fvd.ensure(sizeof(double) * np * kf);
        launch_pair_features<double>(K, Xo.as<double>(), q, d, M->Xd.as<double>(), false, fuo.as<double>(), qp, s);
        launch_pair_features<double>(K, M->Xd.as<double>(), n, d, M->Xd.as<double>(), true, M->fvd.as<double>(), np, s);
        M->kdev64.ensure(sizeof(KCanon<double>));
        GPRX_HIP(hipMemcpyAsync(M->kdev64.p, &K, sizeof(KCanon<double>), hipMemcpyHostToDevice, s));
    } else {
        if (K.nper > 0) {
            M->tabd.ensure(sizeof(double) * 2 * K.nper * n * d);
            launch_sincos_tables<double>(K, M->Xd.as<double>(), n, d, M->tabd.as<double>(), s);
            fuo.ensure(sizeof(double) * 2 * K.nper * std::max<int64_t>(q, 1) * d);
            launch_sincos_tables<double>(K, Xo.as<double>(), q, d, fuo.as<double>(), s);
        }
        M->zd.ensure(sizeof(double) * n * m);
        M->outd.ensure(sizeof(double) * std::max<int64_t>(n, qp) * m);
    }
    const float sf = (float)M->sigma;
    const double s2 = (double)(sf * sf);  // m_Sigma * m_Sigma in T (lib/GaussianProcess.cpp:379)
    double rel = 0;
    int taken = 0;
    for (int it = 0; it < steps; it++) {
        if (mma) {
            for (int c = 0; c < m; c++)
                launch_predict_mma<double>(K, M->kdev64.as<KCanon<double>>(), fuo.as<double>(), qp, M->fvd.as<double>(),
                                           np, d, M->ad.as<double>() + c, n, m, q, kxo.as<double>() + c, s);
        } else {
            launch_predict<double>(K, M->Xd.as<double>(), M->tabd.as<double>(), n, d, m, M->ad.as<double>(),
                                   Xo.as<double>(), fuo.as<double>(), q, kxo.as<double>(), nullptr, M->zd.as<double>(),
                                   M->outd.as<double>(), s);
        }
        GPRX_HIP(hipMemsetAsync(rhs.p, 0, sizeof(float) * np * m, s));
        launch_residual_scatter(M->Yd.as<double>(), kxo.as<double>(), M->ad.as<double>(), s2, didx.as<int64_t>(), q, m,
                                rhs.as<float>(), s);
        dist_solve<float>(M->dist_engine, rhs.as<float>(), M->delta.as<float>(), s);
        launch_refine_accumulate(M->delta.as<float>(), M->ad.as<double>(), M->alpha.as<float>(), n * m,
                                 M->nrm.as<unsigned long long>(), s);
        unsigned long long h[2];
        download(h, M->nrm.p, sizeof(h), s);
        double dn, an;
        std::memcpy(&dn, &h[0], sizeof(double));
        std::memcpy(&an, &h[1], sizeof(double));
        rel = an > 0 ? dn / an : dn;
        taken = it + 1;
        if (!(rel > 0x1p-26)) break;  // below fp32 resolution of alpha (NaN: stop too)
    }
    GPRX_HIP(hipEventRecord(ctx->ev[1], s));
    GPRX_HIP(hipEventSynchronize(ctx->ev[1]));
    if (out) {
        float ms = 0;
        hipEventElapsedTime(&ms, ctx->ev[0], ctx->ev[1]);
        out->ms_refine = ms;
        out->refine_delta = rel;
        out->refine_steps = taken;
    }
}

template <typename T>
static gprx_status model_fit_dist(gprx_model* M, uint32_t flags, gprx_fit_info* out) {
    gprx_ctx* ctx = M->ctx;
    GPRX_REQUIRE(!M->host_k, GPRX_ERR_STATE, "gprx: a caller-evaluated kernel matrix needs a single-GPU fit");
    hipStream_t s = ctx->stream;
    const KCanon<T>& K = kcanon<T>(M);
    const int64_t n = M->n, np = round_up(n, DB);
    M->np = np;
    M->mp = GT;
    M->ld = 0;
    M->fitted = M->has_alpha = M->inv_ready = M->dist_fitted = M->dist_dense = false;
    M->alpha.ensure(sizeof(T) * np * M->m);
    M->flag.ensure(sizeof(int));
    GPRX_HIP(hipMemsetAsync(M->flag.p, 0, sizeof(int), s));
    if (K.nper > 0) {  // per-sample sin/cos tables: the direct predict path reads them
        M->tab.ensure(sizeof(T) * 2 * K.nper * n * M->d);
        launch_sincos_tables<T>(K, M->X.as<T>(), n, M->d, M->tab.as<T>(), s);
    }
    const T sig = (T)M->sigma;
    const T sigma2 = sig * sig;  // m_Sigma*m_Sigma in T (lib/GaussianProcess.cpp:379)
    TileBuild<T> tb;
    std::memset(&tb, 0, sizeof(tb));
    if (pairs_mma_supported<T>(K, 1)) {  // the fused MFMA build: features of all n samples on every rank
        const int64_t kf = pairs_feature_cols<T>(K, M->d);
        M->featU.ensure(sizeof(T) * np * kf);
        M->featV.ensure(sizeof(T) * np * kf);
        launch_pair_features<T>(K, M->X.as<T>(), n, M->d, M->X.as<T>(), false, M->featU.as<T>(), np, s,
                                M->flag.as<int>());
        launch_pair_features<T>(K, M->X.as<T>(), n, M->d, M->X.as<T>(), true, M->featV.as<T>(), np, s);
        M->kdev.ensure(sizeof(KCanon<T>));
        GPRX_HIP(hipMemcpyAsync(M->kdev.p, &K, sizeof(KCanon<T>), hipMemcpyHostToDevice, s));
        tb = pairs_tile_build<T>(K, M->kdev.as<KCanon<T>>(), M->featU.as<T>(), M->featV.as<T>(), np, M->d, n, sigma2,
                                 M->flag.as<int>());
    }
    GPRX_HIP(hipStreamSynchronize(s));  // the ranks' streams read the features
    int hflag = 0;
    GPRX_HIP(hipMemcpy(&hflag, M->flag.p, sizeof(int), hipMemcpyDeviceToHost));
    DistContext C;
    C.device = ctx->device;
    C.rank = ctx->rank;
    C.world = ctx->world;
    C.virt = ctx->virt;
    C.hc = ctx->hc;
    C.cu_slot = ctx->cu_slot;
    C.cu_slots = ctx->cu_slots;
    // LML mode: the inverse rides along in the sharded launch (identity rows + C tiles) when the
    // gradient pass can read C tile by tile; other trees take a dense C on every process
    const bool inv_tiles = M->want_inv && pairs_grad_supported<T>(K);
    DistFitIn<T> in{K, M->X.as<T>(), M->Y.as<T>(), n, M->d, M->m, sigma2, tb, inv_tiles};
    DistFitOut o;
    dist_fit<T>(M->dist_engine, C, in, o, M->alpha.as<T>());
    M->dist_stats = o;
    if (out) {
        std::memset(out, 0, sizeof(*out));
        out->logdet = o.logdet;
        out->datafit = o.datafit;
        out->info = (o.info == INT_MAX || o.info < 0) ? 0 : o.info;
        out->ms_factor = o.ms_kernel;  // device time of this process's persistent launch(es)
        out->ms_solve = o.ms_solve;
        out->refine_delta = 0;
    }
    if (hflag || o.flag)
        throw Error{GPRX_ERR_NONFINITE,
                    "GaussianProcess::ComputeKernelMatrixInternal: kernel matrix contains entries which are not finite."};
    check_sched(o.info);
    if (o.info != INT_MAX) {
        // the reference's default inversion is an LU (lib/GaussianProcess.cpp:545-559) and it
        // never rejects an indefinite K: every rank refactors the same K + s^2 I with the
        // partial-pivot LU in double (X and Y are replicated, the LU is deterministic, so the
        // ranks agree bit for bit).  Replicated, like the reference's own serial getrf: an
        // indefinite K is the exception path, not the sharded fit's workload.
        if (flags & GPRX_FIT_NO_LU_FALLBACK)
            throw Error{GPRX_ERR_NOT_SPD, "gprx: kernel matrix is not positive definite (Cholesky pivot " +
                                              std::to_string(o.info) + " <= 0)"};
        lu_fit_replicated<T>(M, out);
        if (out) out->info = o.info;  // the Cholesky's failing pivot, as on one GPU
        return GPRX_OK;
    }
    M->method = 0;
    M->fitted = M->has_alpha = M->dist_fitted = true;
    M->dist_inv_tiles = inv_tiles;
    if (M->want_inv) {
        if (!inv_tiles) {
            // a tree off the MFMA gradient path: its VALU gradient reads a dense C, formed on
            // every process from the gathered factor (documented N^2 per process)
            ensure_dense_factor<T>(M);
            model_inverse<T>(M);
        }
        M->inv_ready = true;
    }
    if constexpr (std::is_same<T, float>::value) {
        // the reference inverts fp32 GPs in double (include/LAPACKUtils.h:85-97): fp64
        // refinement of alpha against the sharded fp32 factor, as on one GPU
        if (!(flags & GPRX_FIT_F32_NO_REFINE) && !M->want_inv) refine_f32_dist(M, out);
    }
    return GPRX_OK;
}



// ---------------------------------------------------------------------------------------
// fit
// ---------------------------------------------------------------------------------------
template <typename T>
static gprx_status model_fit(gprx_model* M, uint32_t flags, gprx_fit_info* out) {
    gprx_ctx* ctx = M->ctx;
    GPRX_REQUIRE(M->has_data, GPRX_ERR_STATE, "GaussianProcess::Initialize: no input samples defined during initialization");
    GPRX_REQUIRE(M->has_kernel, GPRX_ERR_STATE, "gprx: no kernel set");
    GPRX_HIP(hipSetDevice(ctx->device));
    M->trim_posterior_workspace();
    hipStream_t s = ctx->stream;
    const KCanon<T>& K = kcanon<T>(M);
    // multi-GPU factorisation: an RCCL context with world > 1, a virtual-rank context, or
    // GPRX_FIT_DISTRIBUTED (the same code path on a one-rank communicator)
    GPRX_REQUIRE(!(flags & GPRX_FIT_DISTRIBUTED) || ctx->hc || ctx->virt, GPRX_ERR_STATE,
                 "gprx_model_fit: GPRX_FIT_DISTRIBUTED needs a context from gprx_ctx_create_dist / _peer");
    // the SVD inversion methods' stand-in: the LU in double directly.  On a distributed
    // context every rank runs it on its replicated X, Y (as the NOT_SPD fallback below)
    if (flags & GPRX_FIT_FORCE_LU) {
        lu_fit_replicated<T>(M, out);
        return GPRX_OK;
    }
    if ((ctx->hc && ctx->world > 1) || ctx->virt || (flags & GPRX_FIT_DISTRIBUTED))
        return model_fit_dist<T>(M, flags, out);
    M->dist_fitted = false;
    const int64_t n = M->n, np = round_up(n, (int64_t)DB), mp = round_up(M->m, GT);
    // the explicit inverse rides along in the tile factorisation as np identity rows
    const bool want_inv = M->want_inv && potrf_uses_tiles();
    const int64_t ld = np + mp + (want_inv ? np : 0);
    M->inv_ready = false;
    M->np = np;
    M->mp = mp;
    M->ld = ld;
    M->A.ensure(sizeof(T) * ld * np);
    M->Linv.ensure(sizeof(T) * np * DB);
    M->z.ensure(sizeof(T) * M->m * np);
    M->alpha.ensure(sizeof(T) * np * M->m);
    M->info.ensure(sizeof(int));
    M->flag.ensure(sizeof(int));
    M->red.ensure(sizeof(double) * (2 + 2 * (np / GT + 1)));  // results, then per-block partials
    if (K.nper > 0) {  // per-sample sin/cos tables: the direct build, predict, posterior and LML paths
        M->tab.ensure(sizeof(T) * 2 * K.nper * n * M->d);
        launch_sincos_tables<T>(K, M->X.as<T>(), n, M->d, M->tab.as<T>(), s);
    }
    launch_fit_status_init(M->info.as<int>(), M->flag.as<int>(), s);
    const T sig = (T)M->sigma;
    const T sigma2 = sig * sig;  // m_Sigma*m_Sigma in T (lib/GaussianProcess.cpp:379)
    GPRX_HIP(hipEventRecord(ctx->ev[0], s));
    static const bool direct_build = std::getenv("GPRX_KBUILD") && std::string(std::getenv("GPRX_KBUILD")) == "direct";
    // GPRX_KBUILD=separate: the MFMA build as its own kernel instead of BUILD tasks inside
    // the tile factorisation (where the tile builds fill the factorisation's start-up ramp)
    static const bool separate_build =
        std::getenv("GPRX_KBUILD") && std::string(std::getenv("GPRX_KBUILD")) == "separate";
    TileBuild<T> tb;
    std::memset(&tb, 0, sizeof(tb));
    if (M->host_k) {  // the caller's K (k_hostk.hip)
        launch_kext_build<T>(M->Kext.as<T>(), n, M->A.as<T>(), ld, np, sigma2, M->flag.as<int>(), s);
        launch_aug_rows<T>(M->Y.as<T>(), n, M->m, M->A.as<T>(), ld, np, mp, s);
    } else if (!direct_build && pairs_mma_supported<T>(K, 1)) {
        // pair statistics on the MFMA units from per-sample features (k_pairs.hip)
        const int64_t kf = pairs_feature_cols<T>(K, M->d);
        M->featU.ensure(sizeof(T) * np * kf);
        M->featV.ensure(sizeof(T) * np * kf);
        launch_pair_features<T>(K, M->X.as<T>(), n, M->d, M->X.as<T>(), false, M->featU.as<T>(), np, s,
                                M->flag.as<int>());
        launch_pair_features<T>(K, M->X.as<T>(), n, M->d, M->X.as<T>(), true, M->featV.as<T>(), np, s);
        const KCanon<T>* kdev = M->kfit.put(K, s);
        if (!separate_build && potrf_uses_tiles())
            tb = pairs_tile_build<T>(K, kdev, M->featU.as<T>(), M->featV.as<T>(), np, M->d, n, sigma2,
                                     M->flag.as<int>());
        if (!tb.mode)
            launch_kbuild_mma<T>(K, kdev, M->featU.as<T>(), M->featV.as<T>(), np, M->d, M->A.as<T>(),
                                 ld, n, sigma2, M->flag.as<int>(), s);
        launch_aug_rows<T>(M->Y.as<T>(), n, M->m, M->A.as<T>(), ld, np, mp, s);
    } else {
        launch_kbuild<T>(K, M->X.as<T>(), M->tab.as<T>(), n, M->X.as<T>(), M->tab.as<T>(), n, M->d, M->A.as<T>(), ld,
                         np, true, sigma2, M->flag.as<int>(), s);
        launch_aug_rows<T>(M->Y.as<T>(), n, M->m, M->A.as<T>(), ld, np, mp, s);
    }
    GPRX_HIP(hipEventRecord(ctx->ev[1], s));
    if (tb.mode || want_inv) {
        potrf_tiles<T>(M->A.as<T>(), ld, np, ld, M->Linv.as<T>(), M->info.as<int>(), ctx->ex, tb.mode ? &tb : nullptr,
                       want_inv ? (int)(np / GT) : 0);
    } else {
        potrf_auto<T>(M->A.as<T>(), ld, np, ld, M->Linv.as<T>(), M->info.as<int>(), ctx->ex);
    }
    GPRX_HIP(hipEventRecord(ctx->ev[2], s));
    launch_fit_reductions<T>(M->A.as<T>(), ld, n, np, M->m, M->red.as<double>(), s);
    launch_backsolve_chain<T>(M->A.as<T>(), ld, np, M->m, M->Linv.as<T>(), M->alpha.as<T>(), M->info.as<int>(), ctx->ex,
                              s);
    if (want_inv) {  // C = U U^T (lower), U = L^{-T} from the identity rows
        M->C.ensure(sizeof(T) * np * np);
        const T* U = M->A.as<T>() + np + mp;
        launch_gemm_nt_kskip<T>(M->C.as<T>(), np, U, ld, U, ld, np, np, np, s);
    }
    GPRX_HIP(hipEventRecord(ctx->ev[3], s));
    // status words: one kernel stores them into mapped pinned memory, then one synchronisation
    M->hstat.ensure(4 * sizeof(double));
    volatile double* hs = static_cast<double*>(M->hstat.p);  // [0] flag, [1] info (ints), [2..3] log det, data fit
    launch_fit_status_gather(M->flag.as<int>(), M->info.as<int>(), M->red.as<double>(), M->hstat.dev, s);
    GPRX_HIP(hipStreamSynchronize(s));
    GPRX_HIP(hipGetLastError());
    int hflag = 0, hinfo = 0;
    double hred[2] = {hs[2], hs[3]};
    hflag = reinterpret_cast<volatile int*>(hs)[0];
    hinfo = reinterpret_cast<volatile int*>(hs + 1)[0];
    M->fitted = false;
    M->has_alpha = false;
    M->inv_ready = false;
    if (out) {
        std::memset(out, 0, sizeof(*out));
        float t01 = 0, t12 = 0, t23 = 0;
        hipEventElapsedTime(&t01, ctx->ev[0], ctx->ev[1]);
        hipEventElapsedTime(&t12, ctx->ev[1], ctx->ev[2]);
        hipEventElapsedTime(&t23, ctx->ev[2], ctx->ev[3]);
        out->ms_build = t01;
        out->ms_factor = t12;
        out->ms_solve = t23;
        out->logdet = hred[0];
        out->datafit = hred[1];
        out->info = (hinfo == INT_MAX) ? 0 : hinfo;
        out->method = 0;
    }
    if (hflag)
        throw Error{GPRX_ERR_NONFINITE,
                    "GaussianProcess::ComputeKernelMatrixInternal: kernel matrix contains entries which are not finite."};
    check_sched(hinfo);
    if (hinfo != INT_MAX) {
        // the reference's default inversion is an LU (lib/GaussianProcess.cpp:545-559): refactor
        // the same matrix with partial pivoting instead of rejecting it
        if (!(flags & GPRX_FIT_NO_LU_FALLBACK)) {
            lu_fit<T>(M, out);
            return GPRX_OK;
        }
        throw Error{GPRX_ERR_NOT_SPD, "gprx: kernel matrix is not positive definite (Cholesky pivot " +
                                          std::to_string(hinfo) + " <= 0)"};
    }
    M->method = 0;
    M->fitted = true;
    M->has_alpha = true;
    M->inv_ready = want_inv;
    if constexpr (std::is_same<T, float>::value) {
        // the reference inverts fp32 GPs in double (include/LAPACKUtils.h:85-97): refine alpha
        // in fp64 against the fp32 factor.  Not for the LML's fit (its value and gradient come
        // from the factor and its inverse).
        // (a caller-evaluated kernel has no fp64 form to refine against)
        if (!(flags & GPRX_FIT_F32_NO_REFINE) && !want_inv && !M->host_k) refine_f32(M, out);
    }
    return GPRX_OK;
}

// V = L^{-T} (upper), C = V V^T (lower, ld = np) from the stored factor
template <typename T>
static void model_inverse(gprx_model* M) {
    hipStream_t s = M->ctx->stream;
    const int64_t np = M->np;
    M->V.ensure(sizeof(T) * np * np);
    M->C.ensure(sizeof(T) * np * np);
    launch_spd_inverse_from_factor<T>(M->A.as<T>(), M->ld, np, M->Linv.as<T>(), M->V.as<T>(), M->C.as<T>(), s);
}

// Host <-> device transfers use pageable caller memory: always synchronous, after the
// work stream has drained (no async copies from/to pageable memory).  An input may also be
// device memory (unified addressing decides the direction, hipMemcpyDefault): a caller whose
// samples already live in HBM passes them without a PCIe round trip.
template <typename T>
static void upload(DevBuf& b, const void* host, size_t bytes, hipStream_t s) {
    b.ensure(bytes);
    GPRX_HIP(hipStreamSynchronize(s));
    if (bytes) GPRX_HIP(hipMemcpy(b.p, host, bytes, hipMemcpyDefault));
}

// (the destination may be device memory too -- unified addressing decides the direction -- so
// a caller that keeps results in HBM gets them without a PCIe round trip)
static void download(void* host, const void* dev, size_t bytes, hipStream_t s) {
    GPRX_HIP(hipStreamSynchronize(s));
    GPRX_HIP(hipGetLastError());
    if (bytes) GPRX_HIP(hipMemcpy(host, dev, bytes, hipMemcpyDefault));
}

// An input the caller may pass as host or as device memory: device memory of this context's GPU
// is used where it is (no copy), anything else is copied into `b`.
template <typename T>
static const T* dev_input(DevBuf& b, const void* p, size_t bytes, int device, hipStream_t s) {
    hipPointerAttribute_t at;
    std::memset(&at, 0, sizeof(at));
    if (p && hipPointerGetAttributes(&at, p) == hipSuccess && at.type == hipMemoryTypeDevice && at.device == device)
        return static_cast<const T*>(p);
    (void)hipGetLastError();  // (an unregistered host pointer reports an error: not sticky)
    upload<T>(b, p, bytes, s);
    return b.as<T>();
}

template <typename T>
static gprx_status model_predict(gprx_model* M, const void* Xq, int64_t q, void* mean, void* deriv) {
    GPRX_REQUIRE(M->has_alpha, GPRX_ERR_STATE, "GaussianProcess::ComputeKernelVectorInternal: gaussian process is not initialized.");
    GPRX_REQUIRE(!M->host_k, GPRX_ERR_STATE, "gprx: a caller-evaluated kernel predicts through gprx_model_predict_kx");
    hipStream_t s = M->ctx->stream;
    const KCanon<T>& K = kcanon<T>(M);
    const int d = M->d, m = M->m;
    DevBuf dq, dtab, dmean, dder;
    upload<T>(dq, Xq, sizeof(T) * q * d, s);
    if (K.nper > 0) {
        dtab.ensure(sizeof(T) * 2 * K.nper * q * d);
        launch_sincos_tables<T>(K, dq.as<T>(), q, d, dtab.as<T>(), s);
    }
    dmean.ensure(sizeof(T) * q * m);
    static const bool direct_pred = std::getenv("GPRX_PREDICT") && std::string(std::getenv("GPRX_PREDICT")) == "direct";
    if (!deriv && !direct_pred && pairs_mma_supported<T>(K, m)) {
        // mean only: MFMA pair statistics, K(Xq, X) never materialised (k_pairs.hip)
        const int64_t kf = pairs_feature_cols<T>(K, d), qp = round_up(q, GT), npf = round_up(M->n, GT);
        DevBuf fq;
        fq.ensure(sizeof(T) * qp * kf);
        M->featV.ensure(sizeof(T) * npf * kf);
        launch_pair_features<T>(K, M->X.as<T>(), M->n, d, M->X.as<T>(), true, M->featV.as<T>(), npf, s);
        launch_pair_features<T>(K, dq.as<T>(), q, d, M->X.as<T>(), false, fq.as<T>(), qp, s);
        M->kdev.ensure(sizeof(KCanon<T>));
        GPRX_HIP(hipMemcpyAsync(M->kdev.p, &K, sizeof(KCanon<T>), hipMemcpyHostToDevice, s));
        launch_predict_mma<T>(K, M->kdev.as<KCanon<T>>(), fq.as<T>(), qp, M->featV.as<T>(), npf, d, M->alpha.as<T>(),
                              M->n, m, q, dmean.as<T>(), s);
        download(mean, dmean.p, sizeof(T) * q * m, s);
        return GPRX_OK;
    }
    if (deriv) dder.ensure(sizeof(T) * q * d * m);
    const int64_t ncz = (int64_t)m * (deriv ? (1 + d) : 1);
    M->scratch1.ensure(sizeof(T) * M->n * ncz);
    M->scratch2.ensure(sizeof(T) * q * ncz);
    launch_predict<T>(K, M->X.as<T>(), M->tab.as<T>(), M->n, d, m, M->alpha.as<T>(), dq.as<T>(), dtab.as<T>(), q,
                      dmean.as<T>(), deriv ? dder.as<T>() : nullptr, M->scratch1.as<T>(), M->scratch2.as<T>(), s);
    download(mean, dmean.p, sizeof(T) * q * m, s);
    if (deriv) download(deriv, dder.p, sizeof(T) * q * d * m, s);
    return GPRX_OK;
}

// R = K(Xq, X) (qp x np, ld qp, zero padding), then R L^{-T} in place.  K(Xq, X) as MFMA pair
// statistics (kcross_mma_kernel: the predict path's features of the queries and of the training
// set) when the tree allows it -- 23 ms -> ~4 ms of the 300 ms variance leg at Q = 65536 against
// the VALU kernel (GPRX_PREDICT=direct keeps that one).  fp64 only: the variance k(x,x) -
// |L^{-1} k_x|^2 is a cancelling difference, and in fp32 the expanded |u|^2 + |v|^2 - 2 u.v
// statistic loses ~eps (|x - c|/l)^2 per entry, which L^{-1} amplifies; fp32 models
// keep the exact-difference VALU build.  feat_ready: the training features are already in
// featV (the second side of a pair call).
template <typename T>
static void solve_rows_for(gprx_model* M, const T* dXq, const T* dtabQ, int64_t q, int64_t qp, T* R,
                           bool feat_ready = false) {
    hipStream_t s = M->ctx->stream;
    const KCanon<T>& K = kcanon<T>(M);
    static const bool direct = std::getenv("GPRX_PREDICT") && std::string(std::getenv("GPRX_PREDICT")) == "direct";
    const int64_t npf = round_up(M->n, GT);
    const bool cross_mma = std::is_same<T, double>::value && !direct && pairs_mma_supported<T>(K, 1) && npf <= M->np;
    // R must be zero outside the q x n cross block (the solves run over qp x np); the MFMA cross
    // build stores every entry of that block, so with no padding there is nothing to zero (the
    // memset was 8.6 GB, 1.3 ms, per solve at Q = 65536, N = 16384)
    if (!cross_mma || q != qp || M->n != M->np) GPRX_HIP(hipMemsetAsync(R, 0, sizeof(T) * qp * M->np, s));
    if (cross_mma) {
        const int d = M->d;
        const int64_t kf = pairs_feature_cols<T>(K, d);
        M->pvFq.ensure(sizeof(T) * qp * kf);  // (model-owned: no hipMalloc + hipFree per call)
        if (!feat_ready) {
            M->featV.ensure(sizeof(T) * npf * kf);
            launch_pair_features<T>(K, M->X.as<T>(), M->n, d, M->X.as<T>(), true, M->featV.as<T>(), npf, s);
        }
        launch_pair_features<T>(K, dXq, q, d, M->X.as<T>(), false, M->pvFq.as<T>(), qp, s);
        const KCanon<T>* kdev = M->kfit.put(K, s);
        launch_kcross_mma<T>(K, kdev, M->pvFq.as<T>(), qp, q, M->featV.as<T>(), npf, M->n, d, R, qp,
                             M->flag.as<int>(), s);
    } else {
        launch_kbuild<T>(K, dXq, dtabQ, q, M->X.as<T>(), M->tab.as<T>(), M->n, M->d, R, qp, 0, false, T(0),
                         M->flag.as<int>(), s);
    }
    trsm_rows<T>(M->A.as<T>(), M->ld, M->np, M->Linv.as<T>(), R, qp, qp, s);
}

// operator()(x, y) / GetCredibleInterval (lib/GaussianProcess.cpp:84-114) on a SHARDED fit:
// k(x, y) - (L^{-1} k_x) . (L^{-1} k_y) by the distributed forward substitution of the queries
// (dist_posterior, k_dsolve.hip dist_pvar_kernel): the ranks keep their own rows of L, the
// query columns V_k travel through the receive windows, the row sums are all-reduced.  Pairs
// (x_p, y_p) with x != y ride in the same chunk (64 + 64 columns), variances 128 per chunk.
template <typename T>
static gprx_status model_posterior_cov_dist_core(gprx_model* M, const void* Xa, const void* Xb, int64_t q, bool same,
                                                 void* out);

// FNV-1a over bytes (the processes' query agreement below)
static uint64_t fnv1a(const void* p, size_t n, uint64_t h = 1469598103934665603ull) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

// On a multi-process context the sharded solve is a collective: every process runs the same
// sequence of launches and exchanges.  The processes first agree on their arguments (q, whether
// x == y, a hash of the queries).  Identical arguments (every process asks for the same pairs)
// take the solve as they are; different ones -- e.g. each process its own query_shard slice,
// q = 0 included -- are all-gathered, the solve runs once over every process's pairs, and each
// process keeps its own.
template <typename T>
static gprx_status model_posterior_cov_dist(gprx_model* M, const void* Xa, const void* Xb, int64_t q, void* out) {
    const int d = M->d;
    const bool same = q == 0 || (Xa == Xb) || std::memcmp(Xa, Xb, sizeof(T) * q * d) == 0;
    gprx_ctx* ctx = M->ctx;
    if (!ctx->hc || ctx->world <= 1) return model_posterior_cov_dist_core<T>(M, Xa, Xb, q, same, out);
    const int g = ctx->world;
    struct Hdr {
        int64_t q;
        int64_t same;
        uint64_t hash;
    } h{q, same ? 1 : 0, fnv1a(Xa, sizeof(T) * q * d, fnv1a(same ? Xa : Xb, sizeof(T) * q * d))};
    std::vector<Hdr> all(g);
    ctx->hc->allgather(&h, sizeof(Hdr), all.data());
    bool uniform = true;
    int64_t qmax = 0, qtot = 0;
    bool all_same = true;
    for (const Hdr& x : all) {
        uniform = uniform && x.q == h.q && x.same == h.same && x.hash == h.hash;
        qmax = std::max(qmax, x.q);
        qtot += x.q;
        all_same = all_same && x.same;
    }
    if (uniform) return q ? model_posterior_cov_dist_core<T>(M, Xa, Xb, q, same, out) : GPRX_OK;
    // every process's pairs, in rank order; this process's results from offset `off`
    std::vector<T> mine((size_t)qmax * d * 2, T(0));
    if (q) {
        std::memcpy(mine.data(), Xa, sizeof(T) * q * d);
        std::memcpy(mine.data() + (size_t)qmax * d, Xb, sizeof(T) * q * d);
    }
    std::vector<T> gath((size_t)qmax * d * 2 * g);
    ctx->hc->allgather(mine.data(), sizeof(T) * mine.size(), gath.data());
    std::vector<T> xa((size_t)std::max<int64_t>(qtot, 1) * d), xb((size_t)std::max<int64_t>(qtot, 1) * d);
    int64_t off = 0, mine_off = 0;
    for (int r = 0; r < g; r++) {
        const T* src = gath.data() + (size_t)r * qmax * d * 2;
        if (r == ctx->rank) mine_off = off;
        std::memcpy(xa.data() + off * d, src, sizeof(T) * all[r].q * d);
        std::memcpy(xb.data() + off * d, src + (size_t)qmax * d, sizeof(T) * all[r].q * d);
        off += all[r].q;
    }
    if (qtot == 0) return GPRX_OK;
    std::vector<T> res((size_t)qtot);
    model_posterior_cov_dist_core<T>(M, xa.data(), all_same ? xa.data() : xb.data(), qtot, all_same, res.data());
    if (q) std::memcpy(out, res.data() + mine_off, sizeof(T) * q);
    return GPRX_OK;
}

template <typename T>
static gprx_status model_posterior_cov_dist_core(gprx_model* M, const void* Xa, const void* Xb, int64_t q, bool same,
                                                 void* out) {
    hipStream_t s = M->ctx->stream;
    const KCanon<T>& K = kcanon<T>(M);
    const int d = M->d;
    const int nchmax = dist_pvar_chunks(M->dist_engine);
    const int per = same ? DB : DB / 2;  // pairs per chunk
    const T* xa = static_cast<const T*>(Xa);
    const T* xb = static_cast<const T*>(Xb);
    DevBuf da, db, kab, dz, tz;
    upload<T>(da, Xa, sizeof(T) * q * d, s);
    upload<T>(db, Xb, sizeof(T) * q * d, s);
    kab.ensure(sizeof(T) * q);
    launch_pair_kernel<T>(K, da.as<T>(), db.as<T>(), q, d, kab.as<T>(), s);
    std::vector<T> hk((size_t)q), res((size_t)q);
    download(hk.data(), kab.p, sizeof(T) * q, s);
    std::vector<double> sum;
    for (int64_t p0 = 0; p0 < q;) {
        const int64_t cnt = std::min<int64_t>(q - p0, (int64_t)nchmax * per);
        const int nch = (int)((cnt + per - 1) / per);
        const int64_t nq = (int64_t)nch * DB;
        std::vector<T> Z((size_t)nq * d, T(0));
        for (int64_t j = 0; j < cnt; j++) {
            const int64_t c = j / per, jj = j % per;
            std::memcpy(&Z[(size_t)(c * DB + jj) * d], xa + (p0 + j) * d, sizeof(T) * d);
            if (!same) std::memcpy(&Z[(size_t)(c * DB + DB / 2 + jj) * d], xb + (p0 + j) * d, sizeof(T) * d);
        }
        upload<T>(dz, Z.data(), sizeof(T) * nq * d, s);
        if (K.nper > 0) {
            tz.ensure(sizeof(T) * 2 * K.nper * nq * d);
            launch_sincos_tables<T>(K, dz.as<T>(), nq, d, tz.as<T>(), s);
        }
        dist_posterior<T>(M->dist_engine, K, M->X.as<T>(), K.nper > 0 ? M->tab.as<T>() : nullptr, M->n, d, dz.as<T>(),
                          K.nper > 0 ? tz.as<T>() : nullptr, nch, !same, sum, s);
        for (int64_t j = 0; j < cnt; j++) res[p0 + j] = (T)((double)hk[p0 + j] - sum[(j / per) * DB + j % per]);
        p0 += cnt;
    }
    std::memcpy(out, res.data(), sizeof(T) * q);
    return GPRX_OK;
}

template <typename T>
static gprx_status model_posterior_cov(gprx_model* M, const void* Xa, const void* Xb, int64_t q, void* out) {
    GPRX_REQUIRE(M->fitted || M->sparse_cov, GPRX_ERR_STATE,
                 "GaussianProcess::ComputeKernelVectorInternal: gaussian process is not initialized.");
    GPRX_REQUIRE(!M->host_k, GPRX_ERR_STATE, "gprx: a caller-evaluated kernel uses gprx_model_posterior_cov_kx");
    // a sharded fit solves the queries across the ranks (GPRX_DIST_POSTERIOR=dense: the dense
    // factor gathered onto this process instead, as for the core matrix)
    static const bool dense_forced = std::getenv("GPRX_DIST_POSTERIOR") &&
                                     std::string(std::getenv("GPRX_DIST_POSTERIOR")) == "dense";
    if (M->dist_fitted && !M->dist_dense && M->method == 0 && !dense_forced && dist_pvar_chunks(M->dist_engine) > 0)
        return model_posterior_cov_dist<T>(M, Xa, Xb, q, out);
    ensure_dense_factor<T>(M);  // (collective on a sharded fit's first dense use)
    if (q == 0) return GPRX_OK;
    hipStream_t s = M->ctx->stream;
    const KCanon<T>& K = kcanon<T>(M);
    const int d = M->d;
    const int64_t qp = round_up(q, GT);
    DevBuf da, db, ta, tb, Ra, Rb, kab, res;
    upload<T>(da, Xa, sizeof(T) * q * d, s);
    upload<T>(db, Xb, sizeof(T) * q * d, s);
    if (K.nper > 0) {
        ta.ensure(sizeof(T) * 2 * K.nper * q * d);
        tb.ensure(sizeof(T) * 2 * K.nper * q * d);
        launch_sincos_tables<T>(K, da.as<T>(), q, d, ta.as<T>(), s);
        launch_sincos_tables<T>(K, db.as<T>(), q, d, tb.as<T>(), s);
    }
    if (M->sparse_cov) {  // k(x,y) - Kx^T W Ky over the inducing points, batched on the device
        const int64_t Mp = round_up(M->n, GT);
        DevBuf Z;
        Ra.ensure(sizeof(T) * qp * Mp);
        Rb.ensure(sizeof(T) * qp * Mp);
        Z.ensure(sizeof(T) * qp * Mp);
        GPRX_HIP(hipMemsetAsync(Ra.p, 0, sizeof(T) * qp * Mp, s));
        GPRX_HIP(hipMemsetAsync(Rb.p, 0, sizeof(T) * qp * Mp, s));
        launch_kbuild<T>(K, da.as<T>(), ta.as<T>(), q, M->X.as<T>(), M->tab.as<T>(), M->n, d, Ra.as<T>(), qp, 0, false,
                         T(0), M->flag.as<int>(), s);
        launch_kbuild<T>(K, db.as<T>(), tb.as<T>(), q, M->X.as<T>(), M->tab.as<T>(), M->n, d, Rb.as<T>(), qp, 0, false,
                         T(0), M->flag.as<int>(), s);
        launch_gemm_nt<T>(Z.as<T>(), qp, Rb.as<T>(), qp, M->sparseW.as<T>(), Mp, qp, Mp, Mp, T(1), T(0), false, s);
        kab.ensure(sizeof(T) * q);
        res.ensure(sizeof(T) * q);
        launch_pair_kernel<T>(K, da.as<T>(), db.as<T>(), q, d, kab.as<T>(), s);
        launch_rowdot<T>(Ra.as<T>(), Z.as<T>(), qp, q, Mp, kab.as<T>(), res.as<T>(), s);
        download(out, res.p, sizeof(T) * q, s);
        return GPRX_OK;
    }
    if (M->method == 1) {  // LU factors: k(x,y) - K(X,x)^T A^{-1} K(X,y), the reference's formula (:84-99)
        const int64_t np = M->np;
        DevBuf Kt, Wd, Kad;
        Wd.ensure(sizeof(double) * np * q);
        Kad.ensure(sizeof(double) * np * q);
        auto cross = [&](const T* Xq, const T* tq, double* dst) {  // K(X, Xq): np x q column-major
            T* buf;
            if constexpr (std::is_same<T, double>::value) {
                buf = dst;
            } else {
                Kt.ensure(sizeof(T) * np * q);
                buf = Kt.as<T>();
            }
            GPRX_HIP(hipMemsetAsync(buf, 0, sizeof(T) * np * q, s));
            launch_kbuild<T>(K, M->X.as<T>(), M->tab.as<T>(), M->n, Xq, tq, q, d, buf, np, 0, false, T(0),
                             M->flag.as<int>(), s);
            if constexpr (!std::is_same<T, double>::value) launch_convert<T, double>(buf, dst, np * q, s);
        };
        cross(db.as<T>(), tb.as<T>(), Wd.as<double>());
        lu_solve_model(M, Wd.as<double>(), (int)q);
        cross(da.as<T>(), ta.as<T>(), Kad.as<double>());
        kab.ensure(sizeof(T) * q);
        res.ensure(sizeof(T) * q);
        launch_pair_kernel<T>(K, da.as<T>(), db.as<T>(), q, d, kab.as<T>(), s);
        lu_coldot<T>(Kad.as<double>(), Wd.as<double>(), np, M->n, q, kab.as<T>(), res.as<T>(), s);
        download(out, res.p, sizeof(T) * q, s);
        return GPRX_OK;
    }
    // the variance (GetCredibleInterval, :102-114, pairs (x, x)): one solve, |L^{-1} k_x|^2
    const bool same = (Xa == Xb) || std::memcmp(Xa, Xb, sizeof(T) * q * d) == 0;
    kab.ensure(sizeof(T) * q);
    res.ensure(sizeof(T) * q);
    M->pvRa.ensure(sizeof(T) * qp * M->np);
    if (!same) M->pvRb.ensure(sizeof(T) * qp * M->np);
    {
        // device time of the whole solve (stats class "posterior"): K(x, X), the forward
        // solve (q np^2 flop) and the row dots
        ProfScope ps_(KC_POSTERIOR, s, (same ? 1.0 : 2.0) * (double)q * (double)M->np * (double)M->np);
        T* Ra_ = M->pvRa.as<T>();
        solve_rows_for<T>(M, da.as<T>(), ta.as<T>(), q, qp, Ra_);
        if (!same) solve_rows_for<T>(M, db.as<T>(), tb.as<T>(), q, qp, M->pvRb.as<T>(), true);
        launch_pair_kernel<T>(K, da.as<T>(), db.as<T>(), q, d, kab.as<T>(), s);
        launch_rowdot<T>(Ra_, same ? Ra_ : M->pvRb.as<T>(), qp, q, M->np, kab.as<T>(), res.as<T>(), s);
    }
    download(out, res.p, sizeof(T) * q, s);
    return GPRX_OK;
}

// the explicit inverse from the LU factors (A^{-1} I, double, np x np column-major in luC)
static void lu_inverse(gprx_model* M, DevBuf& luC) {
    const int64_t np = M->np;
    luC.ensure(sizeof(double) * np * np);
    GPRX_HIP(hipMemsetAsync(luC.p, 0, sizeof(double) * np * np, M->ctx->stream));
    launch_set_identity_pad<double>(luC.as<double>(), np, 0, np, M->ctx->stream);
    lu_solve_model(M, luC.as<double>(), (int)np);
}

template <typename T>
static gprx_status model_core_matrix(gprx_model* M, void* Cout) {
    GPRX_REQUIRE(M->fitted, GPRX_ERR_STATE, "gprx: model is not fitted");
    ensure_dense_factor<T>(M);
    hipStream_t s = M->ctx->stream;
    if (M->method == 1) {  // dgetri_'s inverse (include/LAPACKUtils.h:49) from the LU factors
        DevBuf luC;
        lu_inverse(M, luC);
        const int64_t n = M->n, np = M->np;
        std::vector<double> h((size_t)n * n);
        GPRX_HIP(hipStreamSynchronize(s));
        GPRX_HIP(hipGetLastError());
        GPRX_HIP(hipMemcpy2D(h.data(), sizeof(double) * n, luC.p, sizeof(double) * np, sizeof(double) * n, n,
                             hipMemcpyDeviceToHost));
        T* C = reinterpret_cast<T*>(Cout);
        for (int64_t j = 0; j < n; j++)
            for (int64_t i = 0; i < n; i++) C[(size_t)i * n + j] = (T)h[(size_t)j * n + i];
        return GPRX_OK;
    }
    model_inverse<T>(M);
    const int64_t n = M->n, np = M->np;
    std::vector<T> h((size_t)n * n);
    // column j of C (lower part rows >= j) -> row-major; C symmetric
    GPRX_HIP(hipStreamSynchronize(s));
    GPRX_HIP(hipGetLastError());
    GPRX_HIP(hipMemcpy2D(h.data(), sizeof(T) * n, M->C.p, sizeof(T) * np, sizeof(T) * n, n, hipMemcpyDeviceToHost));
    T* C = reinterpret_cast<T*>(Cout);
    // h[j*n + i] = C(i, j) valid for i >= j
    for (int64_t j = 0; j < n; j++)
        for (int64_t i = j; i < n; i++) {
            const T v = h[(size_t)j * n + i];
            C[(size_t)i * n + j] = v;
            C[(size_t)j * n + i] = v;
        }
    return GPRX_OK;
}

template <typename T>
static gprx_status model_lml(gprx_model* M, uint32_t flags, double* value, double* grad, int32_t* nparams,
                             double* logdet) {
    GPRX_REQUIRE(M->m == 1, GPRX_ERR_DIM,
                 "GaussianLogLikelihood: only one output dimension is supported (the reference's data-fit term is "
                 "m x m, include/Likelihood.h:175)");
    GPRX_REQUIRE(!(M->host_k && grad && (flags & GPRX_LML_GRAD)), GPRX_ERR_STATE,
                 "gprx: a caller-evaluated kernel takes its derivative matrices through gprx_model_lml_dk");
    gprx_fit_info fi;
    M->want_inv = grad && (flags & GPRX_LML_GRAD);
    gprx_status st;
    try {
        // the likelihood inverts with the GP's method too (include/Likelihood.h:77-79 ->
        // ComputeCoreMatrixWithDeterminant): a matrix the Cholesky rejects takes the LU
        // the value and gradient come from the factor (and its inverse), never from alpha:
        // an fp32 model's fp64 refinement of alpha would be thrown away (GPRX_FIT_F32_NO_REFINE)
        st = model_fit<T>(M,
                          ((flags & GPRX_LML_DISTRIBUTED) ? GPRX_FIT_DISTRIBUTED : 0u) |
                              ((flags & GPRX_LML_FORCE_LU) ? GPRX_FIT_FORCE_LU : 0u) | GPRX_FIT_F32_NO_REFINE,
                          &fi);
    } catch (...) {
        M->want_inv = false;
        throw;
    }
    M->want_inv = false;
    if (st != GPRX_OK) return st;
    const KCanon<T>& K = kcanon<T>(M);
    const double n = (double)M->n;
    const T df = (T)(-0.5 * fi.datafit);
    const T ct = (T)(-n / 2.0 * std::log(2 * M_PI));  // include/Likelihood.h:192
    double v;
    // LU fits can have det <= 0: the reference's clamp (:180-188) applies in both modes
    const double det_sign = (M->method == 1) ? M->lu_sign : 1.0;
    if ((flags & GPRX_LML_COMPAT) || det_sign <= 0) {
        // include/Likelihood.h:77-79 narrows the long-double determinant to T, :180-188 clamps
        typedef long double HP;
        const HP det_ld = (HP)det_sign * std::exp((HP)fi.logdet);
        const HP det = (HP)(T)det_ld;
        HP cp;
        if (det <= std::numeric_limits<HP>::min()) cp = -0.5L * std::log(std::numeric_limits<HP>::min());
        else if (det > std::numeric_limits<HP>::max()) cp = -0.5L * std::log(std::numeric_limits<HP>::max());
        else cp = -0.5L * std::log(det);
        v = (double)(T)(df + (T)(cp + ct));
    } else {
        v = (double)df - 0.5 * fi.logdet + (double)ct;
    }
    if (std::isinf(v))
        throw Error{GPRX_ERR_NONFINITE, "GaussianLogLikelihood::GetValueAndParameterDerivatives: likelihood is infinite."};
    if (value) *value = v;
    if (logdet) *logdet = fi.logdet;
    if (nparams) *nparams = K.nparams;
    if (grad && (flags & GPRX_LML_GRAD)) {
        hipStream_t s = M->ctx->stream;
        if (M->method == 1) {  // C from the LU factors, in the model's T (the reference casts back)
            DevBuf luC;
            lu_inverse(M, luC);
            M->C.ensure(sizeof(T) * M->np * M->np);
            if constexpr (std::is_same<T, double>::value)
                GPRX_HIP(hipMemcpyAsync(M->C.p, luC.p, sizeof(double) * M->np * M->np, hipMemcpyDeviceToDevice, s));
            else
                launch_convert<double, T>(luC.as<double>(), M->C.as<T>(), M->np * M->np, s);
            GPRX_HIP(hipStreamSynchronize(s));
        } else if (!M->inv_ready || (M->dist_fitted && !M->dist_inv_tiles && !M->dist_dense)) {
            ensure_dense_factor<T>(M);
            model_inverse<T>(M);
        }
        M->grad.ensure(sizeof(double) * MAX_LEAF * 3);
        GPRX_HIP(hipMemsetAsync(M->grad.p, 0, sizeof(double) * MAX_LEAF * 3, s));
        static const bool direct_grad =
            std::getenv("GPRX_LML_GRAD") && std::string(std::getenv("GPRX_LML_GRAD")) == "direct";
        const int64_t np = M->np, npf = round_up(M->n, GT);
        if (!direct_grad && npf == np && pairs_grad_supported<T>(K)) {
            // pair statistics (and the periodic b-derivative statistic) on the MFMA units
            const int64_t kf = pairs_feature_cols<T>(K, M->d), kg = pairs_grad_feature_cols<T>(K, M->d);
            M->featU.ensure(sizeof(T) * np * kf);
            M->featV.ensure(sizeof(T) * np * kf);
            launch_pair_features<T>(K, M->X.as<T>(), M->n, M->d, M->X.as<T>(), false, M->featU.as<T>(), np, s);
            launch_pair_features<T>(K, M->X.as<T>(), M->n, M->d, M->X.as<T>(), true, M->featV.as<T>(), np, s);
            M->kdev.ensure(sizeof(KCanon<T>));
            GPRX_HIP(hipMemcpyAsync(M->kdev.p, &K, sizeof(KCanon<T>), hipMemcpyHostToDevice, s));
            M->scratch1.ensure(sizeof(T) * np * std::max<int64_t>(kg, 1));
            M->scratch2.ensure(sizeof(T) * np * std::max<int64_t>(kg, 1));
            const int64_t nt = np / GT;
            M->pack.ensure(sizeof(double) * MAX_LEAF * 3 * nt * (nt + 1) / 2);
            if (M->dist_fitted && M->dist_inv_tiles) {
                // sharded fit in LML mode: each rank sums (alpha alpha^T - C) o dK/dp over the
                // lower tiles of its own row blocks, C straight from its packed C tiles (the
                // sharded potri riding along in the factorisation); one reduction over the ranks
                dist_lml_grad<T>(M->dist_engine, K, M->kdev.as<KCanon<T>>(), M->X.as<T>(), M->n, M->d,
                                 M->featU.as<T>(), M->featV.as<T>(), M->scratch1.as<T>(), M->scratch2.as<T>(), np,
                                 M->alpha.as<T>(), M->pack.as<double>(), M->grad.as<double>(), s);
            } else {
                launch_lml_grad_mma<T>(K, M->kdev.as<KCanon<T>>(), M->X.as<T>(), M->n, M->d, M->featU.as<T>(),
                                       M->featV.as<T>(), M->scratch1.as<T>(), M->scratch2.as<T>(), np,
                                       M->alpha.as<T>(), M->C.as<T>(), M->np, M->pack.as<double>(),
                                       M->grad.as<double>(), s);
            }
        } else {
            launch_lml_grad<T>(K, M->X.as<T>(), M->tab.as<T>(), M->n, M->d, M->alpha.as<T>(), M->C.as<T>(), M->np,
                               M->grad.as<double>(), s);
        }
        double acc[MAX_LEAF * 3];
        download(acc, M->grad.p, sizeof(acc), s);
        for (int l = 0; l < K.nleaf; l++) {
            const int t = K.leaf[l].type;
            const int np = (t == L_WHITE) ? 1 : ((t == L_GAUSS || t == L_GAUSS_EXP) ? 2 : 3);
            for (int q = 0; q < np; q++) grad[K.param_base[l] + q] = 0.5 * acc[l * 3 + q];
        }
    }
    return GPRX_OK;
}

// ---------------------------------------------------------------------------------------
// caller-evaluated kernels (k_hostk.hip): predict, posterior covariance and the LML gradient
// from the caller's kernel vectors / derivative matrices
// ---------------------------------------------------------------------------------------
template <typename T>
static gprx_status model_predict_kx(gprx_model* M, const void* Kx, const void* Xq, int64_t q, void* mean, void* deriv) {
    GPRX_REQUIRE(M->has_alpha, GPRX_ERR_STATE, "GaussianProcess::ComputeKernelVectorInternal: gaussian process is not initialized.");
    GPRX_REQUIRE(!deriv || Xq, GPRX_ERR_ARG, "gprx_model_predict_kx: the derivative needs the query points");
    hipStream_t s = M->ctx->stream;
    const int d = M->d, m = M->m;
    const int64_t n = M->n;
    DevBuf dk, dq, dmean, dder;
    upload<T>(dk, Kx, sizeof(T) * q * n, s);
    if (deriv) {
        upload<T>(dq, Xq, sizeof(T) * q * d, s);
        dder.ensure(sizeof(T) * q * d * m);
    }
    dmean.ensure(sizeof(T) * q * m);
    launch_kx_predict<T>(dk.as<T>(), deriv ? dq.as<T>() : nullptr, M->X.as<T>(), q, n, d, M->alpha.as<T>(), m,
                         dmean.as<T>(), deriv ? dder.as<T>() : nullptr, s);
    download(mean, dmean.p, sizeof(T) * q * m, s);
    if (deriv) download(deriv, dder.p, sizeof(T) * q * d * m, s);
    return GPRX_OK;
}

template <typename T>
static gprx_status model_posterior_cov_kx(gprx_model* M, const void* Kxa, const void* Kxb, const void* kab, int64_t q,
                                          void* out) {
    GPRX_REQUIRE(M->fitted, GPRX_ERR_STATE, "GaussianProcess::ComputeKernelVectorInternal: gaussian process is not initialized.");
    GPRX_REQUIRE(!M->dist_fitted, GPRX_ERR_STATE, "gprx: the posterior covariance needs a single-GPU fit");
    hipStream_t s = M->ctx->stream;
    const int64_t n = M->n, np = M->np, qp = round_up(q, GT);
    DevBuf dkab, res;
    upload<T>(dkab, kab, sizeof(T) * q, s);
    res.ensure(sizeof(T) * q);
    const T* ka = reinterpret_cast<const T*>(Kxa);
    const T* kb = reinterpret_cast<const T*>(Kxb);
    if (M->method == 1) {  // LU: k(x,y) - K(X,x)^T A^{-1} K(X,y) (lib/GaussianProcess.cpp:84-99)
        std::vector<double> ha((size_t)np * q, 0.0), hb((size_t)np * q, 0.0);  // np x q column-major
        for (int64_t j = 0; j < q; j++)
            for (int64_t i = 0; i < n; i++) {
                ha[(size_t)j * np + i] = (double)ka[j * n + i];
                hb[(size_t)j * np + i] = (double)kb[j * n + i];
            }
        DevBuf Wd, Kad;
        upload<double>(Wd, hb.data(), sizeof(double) * np * q, s);
        upload<double>(Kad, ha.data(), sizeof(double) * np * q, s);
        lu_solve_model(M, Wd.as<double>(), (int)q);
        lu_coldot<T>(Kad.as<double>(), Wd.as<double>(), np, n, q, dkab.as<T>(), res.as<T>(), s);
    } else {  // Cholesky: k(x,y) - (L^{-1} kx) . (L^{-1} ky), rows qp x np (ld qp)
        std::vector<T> ha((size_t)qp * np, T(0)), hb((size_t)qp * np, T(0));
        for (int64_t j = 0; j < q; j++)
            for (int64_t i = 0; i < n; i++) {
                ha[(size_t)i * qp + j] = ka[j * n + i];
                hb[(size_t)i * qp + j] = kb[j * n + i];
            }
        DevBuf Ra, Rb;
        upload<T>(Ra, ha.data(), sizeof(T) * qp * np, s);
        upload<T>(Rb, hb.data(), sizeof(T) * qp * np, s);
        trsm_rows<T>(M->A.as<T>(), M->ld, np, M->Linv.as<T>(), Ra.as<T>(), qp, qp, s);
        trsm_rows<T>(M->A.as<T>(), M->ld, np, M->Linv.as<T>(), Rb.as<T>(), qp, qp, s);
        launch_rowdot<T>(Ra.as<T>(), Rb.as<T>(), qp, q, np, dkab.as<T>(), res.as<T>(), s);
    }
    download(out, res.p, sizeof(T) * q, s);
    return GPRX_OK;
}

template <typename T>
static gprx_status model_lml_dk(gprx_model* M, uint32_t flags, const void* dK, int32_t P, double* value, double* grad,
                                double* logdet) {
    GPRX_REQUIRE(P >= 0 && (P == 0 || dK), GPRX_ERR_ARG, "gprx_model_lml_dk: bad derivative matrices");
    gprx_status st = model_lml<T>(M, flags & ~GPRX_LML_GRAD, value, nullptr, nullptr, logdet);
    if (st != GPRX_OK || !grad || P == 0) return st;
    hipStream_t s = M->ctx->stream;
    const int64_t n = M->n, np = M->np;
    if (M->method == 1) {  // C from the LU factors, in T (the reference casts back)
        DevBuf luC;
        lu_inverse(M, luC);
        M->C.ensure(sizeof(T) * np * np);
        if constexpr (std::is_same<T, double>::value)
            GPRX_HIP(hipMemcpyAsync(M->C.p, luC.p, sizeof(double) * np * np, hipMemcpyDeviceToDevice, s));
        else
            launch_convert<double, T>(luC.as<double>(), M->C.as<T>(), np * np, s);
        GPRX_HIP(hipStreamSynchronize(s));
    } else {
        model_inverse<T>(M);
    }
    DevBuf ddk, g;
    upload<T>(ddk, dK, sizeof(T) * (size_t)P * n * n, s);
    g.ensure(sizeof(double) * P);
    launch_dk_grad<T>(ddk.as<T>(), P, n, M->alpha.as<T>(), M->C.as<T>(), np, g.as<double>(), s);
    download(grad, g.p, sizeof(double) * P, s);
    return GPRX_OK;
}

// ---------------------------------------------------------------------------------------
// standalone building blocks
// ---------------------------------------------------------------------------------------
template <typename T>
static gprx_status kernel_matrix_impl(gprx_ctx* ctx, const gprx_kernel_desc* desc, const void* X, int64_t n, int d,
                                      void* Kout, bool deriv) {
    KCanon<T> K;
    std::string e = canonicalize<T>(*desc, K);
    GPRX_REQUIRE(e.empty(), GPRX_ERR_ARG, e);
    hipStream_t s = ctx->stream;
    DevBuf dx, tab, dk, flag;
    upload<T>(dx, X, sizeof(T) * n * d, s);
    if (K.nper > 0) {
        tab.ensure(sizeof(T) * 2 * K.nper * n * d);
        launch_sincos_tables<T>(K, dx.as<T>(), n, d, tab.as<T>(), s);
    }
    if (deriv) {
        dk.ensure(sizeof(T) * K.nparams * n * n);
        launch_deriv_matrix<T>(K, dx.as<T>(), tab.as<T>(), n, d, dk.as<T>(), s);
        download(Kout, dk.p, sizeof(T) * K.nparams * n * n, s);
        return GPRX_OK;
    }
    dk.ensure(sizeof(T) * n * n);
    flag.ensure(sizeof(int));
    GPRX_HIP(hipMemsetAsync(flag.p, 0, sizeof(int), s));
    launch_kbuild<T>(K, dx.as<T>(), tab.as<T>(), n, dx.as<T>(), tab.as<T>(), n, d, dk.as<T>(), n, n, true, T(0),
                     flag.as<int>(), s);
    std::vector<T> h((size_t)n * n);
    download(h.data(), dk.p, sizeof(T) * n * n, s);
    int hf = 0;
    download(&hf, flag.p, sizeof(int), s);
    T* out = reinterpret_cast<T*>(Kout);
    for (int64_t j = 0; j < n; j++)
        for (int64_t i = j; i < n; i++) {
            const T v = h[(size_t)j * n + i];
            out[(size_t)i * n + j] = v;
            out[(size_t)j * n + i] = v;
        }
    if (hf)
        throw Error{GPRX_ERR_NONFINITE,
                    "GaussianProcess::ComputeKernelMatrixInternal: kernel matrix contains entries which are not finite."};
    return GPRX_OK;
}

template <typename T>
static gprx_status cross_matrix_impl(gprx_ctx* ctx, const gprx_kernel_desc* desc, const void* A, int64_t na,
                                     const void* B, int64_t nb, int d, void* Kout) {
    KCanon<T> K;
    std::string e = canonicalize<T>(*desc, K);
    GPRX_REQUIRE(e.empty(), GPRX_ERR_ARG, e);
    hipStream_t s = ctx->stream;
    DevBuf da, dbb, ta, tb, dk, flag;
    upload<T>(da, A, sizeof(T) * na * d, s);
    upload<T>(dbb, B, sizeof(T) * nb * d, s);
    if (K.nper > 0) {
        ta.ensure(sizeof(T) * 2 * K.nper * na * d);
        tb.ensure(sizeof(T) * 2 * K.nper * nb * d);
        launch_sincos_tables<T>(K, da.as<T>(), na, d, ta.as<T>(), s);
        launch_sincos_tables<T>(K, dbb.as<T>(), nb, d, tb.as<T>(), s);
    }
    dk.ensure(sizeof(T) * na * nb);
    flag.ensure(sizeof(int));
    GPRX_HIP(hipMemsetAsync(flag.p, 0, sizeof(int), s));
    launch_kbuild<T>(K, da.as<T>(), ta.as<T>(), na, dbb.as<T>(), tb.as<T>(), nb, d, dk.as<T>(), na, 0, false, T(0),
                     flag.as<int>(), s);
    std::vector<T> h((size_t)na * nb);
    download(h.data(), dk.p, sizeof(T) * na * nb, s);
    T* out = reinterpret_cast<T*>(Kout);
    for (int64_t j = 0; j < nb; j++)
        for (int64_t i = 0; i < na; i++) out[(size_t)i * nb + j] = h[(size_t)j * na + i];
    return GPRX_OK;
}

template <typename T>
static gprx_status cholesky_impl(gprx_ctx* ctx, void* Ahost, int64_t n, int32_t* info, bool inverse) {
    hipStream_t s = ctx->stream;
    const int64_t np = round_up(n, DB);
    DevBuf dA, dLinv, dinfo, dV, dC;
    dA.ensure(sizeof(T) * np * np);
    dLinv.ensure(sizeof(T) * np * DB);
    dinfo.ensure(sizeof(int));
    GPRX_HIP(hipMemsetAsync(dA.p, 0, sizeof(T) * np * np, s));
    GPRX_HIP(hipStreamSynchronize(s));
    // row i of the (symmetric) host matrix = column i of the column-major device matrix
    GPRX_HIP(hipMemcpy2D(dA.p, sizeof(T) * np, Ahost, sizeof(T) * n, sizeof(T) * n, n, hipMemcpyHostToDevice));
    launch_set_identity_pad<T>(dA.as<T>(), np, n, np, s);
    GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)dinfo.p, INT_MAX, 1, s));
    potrf_auto<T>(dA.as<T>(), np, np, np, dLinv.as<T>(), dinfo.as<int>(), ctx->ex);
    int hinfo = 0;
    download(&hinfo, dinfo.p, sizeof(int), s);
    check_sched(hinfo);
    hinfo = (hinfo == INT_MAX) ? 0 : hinfo;
    if (info) *info = hinfo;
    std::vector<T> h((size_t)n * n);
    T* out = reinterpret_cast<T*>(Ahost);
    if (!inverse) {
        GPRX_HIP(hipMemcpy2D(h.data(), sizeof(T) * n, dA.p, sizeof(T) * np, sizeof(T) * n, n, hipMemcpyDeviceToHost));
        // h[j*n + i] = L(i, j) for i >= j
        for (int64_t i = 0; i < n; i++)
            for (int64_t j = 0; j < n; j++) out[(size_t)i * n + j] = (i >= j) ? h[(size_t)j * n + i] : T(0);
        return hinfo ? GPRX_ERR_NOT_SPD : GPRX_OK;
    }
    if (hinfo) return fail(ctx, GPRX_ERR_NOT_SPD, "gprx_spd_inverse: matrix is not positive definite");
    dV.ensure(sizeof(T) * np * np);
    dC.ensure(sizeof(T) * np * np);
    launch_spd_inverse_from_factor<T>(dA.as<T>(), np, np, dLinv.as<T>(), dV.as<T>(), dC.as<T>(), s);
    GPRX_HIP(hipStreamSynchronize(s));
    GPRX_HIP(hipGetLastError());
    GPRX_HIP(hipMemcpy2D(h.data(), sizeof(T) * n, dC.p, sizeof(T) * np, sizeof(T) * n, n, hipMemcpyDeviceToHost));
    for (int64_t j = 0; j < n; j++)
        for (int64_t i = j; i < n; i++) {
            const T v = h[(size_t)j * n + i];
            out[(size_t)i * n + j] = v;
            out[(size_t)j * n + i] = v;
        }
    return GPRX_OK;
}

// gprx_dev_build_matrix: the fit's covariance tiles, written alone (include/gprx_dev.h)
template <typename T>
static gprx_status dev_build_impl(gprx_ctx* ctx, const gprx_kernel_desc* desc, const void* X, int64_t n, int d,
                                  double sigma, int path, void* Kout, int iters = 0, double* ms = nullptr) {
    KCanon<T> K;
    std::string e = canonicalize<T>(*desc, K);
    GPRX_REQUIRE(e.empty(), GPRX_ERR_ARG, e);
    GPRX_REQUIRE(n > 0 && d > 0, GPRX_ERR_DIM, "gprx_dev_build_matrix: bad dimensions");
    GPRX_REQUIRE(pairs_mma_supported<T>(K, 1), GPRX_ERR_ARG,
                 "gprx_dev_build_matrix: the tree takes the direct (VALU) build, see gprx_kernel_matrix");
    hipStream_t s = ctx->stream;
    const int64_t np = round_up(n, GT), kf = pairs_feature_cols<T>(K, d);
    DevBuf dx, fu, fv, kd, A, Li, info, flag;
    upload<T>(dx, X, sizeof(T) * n * d, s);
    fu.ensure(sizeof(T) * np * kf);
    fv.ensure(sizeof(T) * np * kf);
    kd.ensure(sizeof(KCanon<T>));
    flag.ensure(sizeof(int));
    info.ensure(sizeof(int));
    A.ensure(sizeof(T) * np * np);
    Li.ensure(sizeof(T) * np * DB);
    GPRX_HIP(hipMemsetAsync(flag.p, 0, sizeof(int), s));
    GPRX_HIP(hipMemsetAsync(A.p, 0, sizeof(T) * np * np, s));
    GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)info.p, INT_MAX, 1, s));
    launch_pair_features<T>(K, dx.as<T>(), n, d, dx.as<T>(), false, fu.as<T>(), np, s, flag.as<int>());
    launch_pair_features<T>(K, dx.as<T>(), n, d, dx.as<T>(), true, fv.as<T>(), np, s);
    GPRX_HIP(hipMemcpyAsync(kd.p, &K, sizeof(KCanon<T>), hipMemcpyHostToDevice, s));
    const T sig = (T)sigma, sigma2 = sig * sig;
    TileBuild<T> tb{};
    if (path == 0) {
        tb = pairs_tile_build<T>(K, kd.as<KCanon<T>>(), fu.as<T>(), fv.as<T>(), np, d, n, sigma2, flag.as<int>());
        GPRX_REQUIRE(tb.mode != 0, GPRX_ERR_ARG,
                     "gprx_dev_build_matrix: the fused build carries sum-of-exp-leaf trees only (path 1 for others)");
    }
    auto launch = [&] {
        if (path == 0)
            potrf_tiles<T>(A.as<T>(), np, np, np, Li.as<T>(), info.as<int>(), ctx->ex, &tb, 0, true);
        else
            launch_kbuild_mma<T>(K, kd.as<KCanon<T>>(), fu.as<T>(), fv.as<T>(), np, d, A.as<T>(), np, n, sigma2,
                                 flag.as<int>(), s);
    };
    if (ms) {  // gprx_dev_build_time: device time of the build alone (features resident)
        launch();  // warm (schedule cached, code loaded)
        hipStream_t ls = path == 0 ? ctx->ex.s0 : s;
        GPRX_HIP(hipStreamSynchronize(s));
        hipEvent_t e0, e1;
        GPRX_HIP(hipEventCreate(&e0));
        GPRX_HIP(hipEventCreate(&e1));
        GPRX_HIP(hipEventRecord(e0, ls));
        for (int it = 0; it < iters; it++) launch();
        GPRX_HIP(hipEventRecord(e1, ls));
        GPRX_HIP(hipEventSynchronize(e1));
        float t = 0;
        GPRX_HIP(hipEventElapsedTime(&t, e0, e1));
        GPRX_HIP(hipEventDestroy(e0));
        GPRX_HIP(hipEventDestroy(e1));
        *ms = (double)t / std::max(1, iters);
        int hinfo = 0;
        download(&hinfo, info.p, sizeof(int), s);
        check_sched(hinfo);
        return GPRX_OK;
    }
    launch();
    std::vector<T> h((size_t)np * n);
    download(h.data(), A.p, sizeof(T) * np * n, s);
    int hf = 0, hinfo = 0;
    download(&hf, flag.p, sizeof(int), s);
    download(&hinfo, info.p, sizeof(int), s);
    check_sched(hinfo);
    T* out = reinterpret_cast<T*>(Kout);
    for (int64_t j = 0; j < n; j++)
        for (int64_t i = j; i < n; i++) {
            const T v = h[(size_t)j * np + i];  // column-major, lower triangle
            out[(size_t)i * n + j] = v;
            out[(size_t)j * n + i] = v;
        }
    if (hf)
        throw Error{GPRX_ERR_NONFINITE,
                    "GaussianProcess::ComputeKernelMatrixInternal: kernel matrix contains entries which are not finite."};
    return GPRX_OK;
}

// ---------------------------------------------------------------------------------------
// sparse GP (subset of regressors), SparseGaussianProcess::PreComputeRegression
// (include/SparseGaussianProcess.h:274-313):
//   K   = Kmm + jitter I                              (M x M)
//   S   = K + sigma^-2 Knm^T Knm,   b = sigma^-2 Knm^T Y
//   RV  = S^{-1} b          (the reference's Kinv (sigma^-2 K Sigma Knm^T Y), Kinv K = I)
//   RM  = S^{-1} = Sigma    (the reference's Kinv (K Sigma K) Kinv)
//   Kinv = K^{-1}
// Knm is streamed in chunks of dense rows: each chunk is built as the (M + labels) x Nc
// block [Kmn_c ; Y_c^T] and folded into the lower triangle of the augmented S with one
// MFMA gemm (A A^T), so b rides along as extra rows, exactly like Y in the dense fit.  With
// an RCCL context the dense rows are sharded over ranks (each rank passes its own rows) and
// the accumulated (M + labels) x M block is all-reduced -- the one exchange of the path.
// ---------------------------------------------------------------------------------------
template <typename T>
static ncclDataType_t nccl_type();
template <>
ncclDataType_t nccl_type<double>() {
    return ncclFloat64;
}
template <>
ncclDataType_t nccl_type<float>() {
    return ncclFloat32;
}

template <typename T>
static void download_sym(void* out, const DevBuf& C, int64_t ldc, int64_t n, hipStream_t s) {
    // mirrored on the device, then one strided copy: the full symmetric matrix reads the same
    // row- or column-major, so it lands in the caller's buffer as is
    launch_sym_fill<T>(C.as<T>(), ldc, n, s);
    GPRX_HIP(hipGetLastError());
    GPRX_HIP(hipMemcpy2DAsync(out, sizeof(T) * n, C.p, sizeof(T) * ldc, sizeof(T) * n, n, hipMemcpyDefault, s));
    GPRX_HIP(hipStreamSynchronize(s));
}

// Device state of the sparse GP's normal equations (shared by the fit and the likelihood).
template <typename T>
struct SparseNE {
    KCanon<T> K{};
    int64_t Mp = 0, mp = 0, ld = 0, chunk = 0, chunk128 = 0;
    bool mma = false;
    T is2 = 0;
    DevBuf dXm, dtm, dX, dtx, dY, dS, dA, dK, dLinv, dLinvK, dinfo, dflag, dz, dalpha, dV, dC, dFU, dFV, dKd;
    const T* pX = nullptr;  // the dense rows and labels in HBM: the caller's device memory, or dX / dY
    const T* pY = nullptr;
    // the streamed block dA (ld x acols): columns from dA_zero on are known to hold zeros (its
    // layout last zeroed whole for dA_p, dA_ld, dA_cols); a chunk zeroes only the columns between
    // its own end and dA_zero, instead of the whole 4.6 GB block (two memsets of it per C5 fit)
    void* dA_p = nullptr;
    int64_t dA_ld = 0, dA_cols = 0, dA_zero = 0;
};

// The sparse fit's device state lives in the context between calls (its buffers -- the
// partial normal equations, the streamed Kmn blocks, the M x M factors: hundreds of MB at C5 --
// are allocated once per shape, not per call).  One per scalar type; calls on a context are
// serialised by its mutex.
template <typename T>
static SparseNE<T>& sparse_state(gprx_ctx* ctx) {
    std::shared_ptr<void>& h = ctx->sparse_state[sizeof(T) == 8 ? 1 : 0];
    if (!h) h = std::make_shared<SparseNE<T>>();
    return *static_cast<SparseNE<T>*>(h.get());
}

// SparseGaussianProcess::PreComputeRegression (include/SparseGaussianProcess.h:274-313) up to
// the factorisation: S = Kmm + jitter I + sigma^-2 Kmn Knm with b = sigma^-2 Kmn Y riding
// along as extra rows (Kmn streamed in row chunks through the GPU, never held whole), S = L L^T
// (b becomes L^{-1} b in place), and Kmm + jitter I built (unfactored) in dK.
template <typename T>
static void sparse_normal_eq(gprx_ctx* ctx, SparseNE<T>& st, const gprx_kernel_desc* desc, const void* Xh,
                             const void* Yh, int64_t n, int d, int m, const void* Xmh, int64_t M, double sigma,
                             double jitter) {
    KCanon<T>& K = st.K;
    const std::string e = canonicalize<T>(*desc, K);
    GPRX_REQUIRE(e.empty(), GPRX_ERR_ARG, e);
    GPRX_REQUIRE(M > 0 && d > 0 && m > 0 && n >= 0, GPRX_ERR_DIM, "gprx_sparse_fit: bad dimensions");
    GPRX_REQUIRE(sigma > 0, GPRX_ERR_ARG, "SparseGaussianProcess::ComputeCoreMatrices: sigma must be positive.");
    GPRX_HIP(hipSetDevice(ctx->device));
    hipStream_t s = ctx->stream;
    const int64_t Mp = round_up(M, DB), mp = round_up(m, GT), ld = Mp + mp;
    st.Mp = Mp;
    st.mp = mp;
    st.ld = ld;
    // dense rows per streamed block (GPRX_SPARSE_CHUNK overrides, for tests): 262144 rows = four
    // split-K launches at C5 instead of 31 -- the per-launch ramp, tail and partial-sum traffic
    // amortised: syrk 0.737 -> 0.794 of the f64 peak, fit 88.1 -> 84.4 ms, same-box A/B
    // (profiles/r06d_c5_chunk_ab.txt: 131072 84.3 ms / 0.78, one launch 85.6 ms / 0.80); the
    // streamed block is ld x 262400 x 8 B = 4.6 GB of HBM
    int64_t cmax = 262144;
    if (const char* ev = std::getenv("GPRX_SPARSE_CHUNK")) cmax = std::max<int64_t>(64, round_up(std::atoll(ev), 64));
    const int64_t chunk = std::max<int64_t>(BT, std::min<int64_t>(round_up(std::max<int64_t>(n, 1), 64), cmax));
    DevBuf &dXm = st.dXm, &dtm = st.dtm, &dX = st.dX, &dtx = st.dtx, &dY = st.dY, &dS = st.dS, &dA = st.dA,
           &dK = st.dK, &dLinv = st.dLinv, &dinfo = st.dinfo, &dflag = st.dflag, &dFU = st.dFU, &dFV = st.dFV,
           &dKd = st.dKd;
    st.chunk = chunk;
    upload<T>(dXm, Xmh, sizeof(T) * M * d, s);
    st.pX = dev_input<T>(dX, Xh, sizeof(T) * std::max<int64_t>(n, 1) * d, ctx->device, s);
    st.pY = dev_input<T>(dY, Yh, sizeof(T) * std::max<int64_t>(n, 1) * m, ctx->device, s);
    // Kmn blocks as MFMA pair statistics (k_pairs.hip) when the tree allows it: features of
    // the inducing points once, of each dense chunk per chunk, both centred on Xm's first row
    const bool mma = pairs_mma_supported<T>(K, 1);
    const int64_t chunk128 = round_up(chunk, GT);
    st.mma = mma;
    st.chunk128 = chunk128;
    dflag.ensure(sizeof(int));
    GPRX_HIP(hipMemsetAsync(dflag.p, 0, sizeof(int), s));
    if (mma) {
        const int64_t fc = pairs_feature_cols<T>(K, d);
        dKd.ensure(sizeof(KCanon<T>));
        GPRX_HIP(hipMemcpyAsync(dKd.p, &K, sizeof(KCanon<T>), hipMemcpyHostToDevice, s));
        dFU.ensure(sizeof(T) * Mp * fc);
        dFV.ensure(sizeof(T) * chunk128 * fc);
        launch_pair_features<T>(K, dXm.as<T>(), M, d, dXm.as<T>(), false, dFU.as<T>(), Mp, s, dflag.as<int>());
    }
    if (K.nper > 0) {
        dtm.ensure(sizeof(T) * 2 * K.nper * M * d);  // Kmm below
        launch_sincos_tables<T>(K, dXm.as<T>(), M, d, dtm.as<T>(), s);
        if (!mma) dtx.ensure(sizeof(T) * 2 * K.nper * chunk * d);  // per-chunk tables of the dense rows
    }
    dinfo.ensure(sizeof(int));
    // ---- accumulate sigma^-2 [Kmn ; Y^T][Kmn ; Y^T]^T over the dense rows (lower part) ----
    // split-K partials: tiles x partials workgroups in whole rounds of the chip's slots (one
    // tile-mainloop workgroup per CU).  M = 2048: 152 tiles; P = 5 fills 3 rounds to 99% (an
    // earlier P = 7 on two slots per CU left the third round 4% full).
    // fused: one label column (m = 1) with the MFMA cross build -- K Y comes out of the build's
    // epilogue (kcross_mma_kernel), so the rank-k accumulation has no 128-row label tile
    const bool fused = mma && m == 1;
    const int64_t ntiles = (Mp / GT) * (Mp / GT + 1) / 2 + (fused ? 0 : (mp / GT) * (Mp / GT));
    int ncu = 0;
    GPRX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, ctx->device));
    const int64_t slots = (int64_t)std::max(1, ncu);
    const int64_t ncp_max = round_up(chunk, 16);
    int P = 1;
    double best = 0.0;
    for (int p = 1; p <= 16; p++) {
        if (p > 1 && round_up((ncp_max + p - 1) / p, 16) < 256) break;  // keep each slice >= 256 deep
        const int64_t wg = ntiles * p, rounds = (wg + slots - 1) / slots;
        const double eff = (double)wg / (double)(rounds * slots);
        if (eff > best + 1e-9) {
            best = eff;
            P = p;
        }
    }
    const int64_t sstride = ld * Mp;
    dS.ensure(sizeof(T) * sstride * P);
    GPRX_HIP(hipMemsetAsync(dS.p, 0, sizeof(T) * sstride * P, s));
    const int64_t acols = chunk + 16 * 16;  // slack: the P <= 16 split-K slices may overhang ncp (zeros)
    dA.ensure(sizeof(T) * ld * acols);
    if (dA.p != st.dA_p || st.dA_ld != ld || st.dA_cols != acols) {  // a new block layout: zero it whole
        GPRX_HIP(hipMemsetAsync(dA.p, 0, sizeof(T) * ld * acols, s));
        st.dA_p = dA.p;
        st.dA_ld = ld;
        st.dA_cols = acols;
        st.dA_zero = 0;
    }
    const T is2 = T(1) / (T(sigma) * T(sigma));  // inverse_sigma2 in T (:285)
    st.is2 = is2;
    DevBuf dKY;
    if (fused) dKY.ensure(sizeof(T) * (chunk128 / GT) * Mp);
    for (int64_t off = 0; off < n; off += chunk) {
        const int64_t nc = std::min(chunk, n - off), ncp = round_up(nc, 16);
        // columns [nc, acols) must be zero for this chunk's products (the split-K slices overhang
        // the data): zero what an earlier, longer chunk left there; this chunk dirties [0, ncp)
        if (st.dA_zero > nc) {
            GPRX_HIP(hipMemsetAsync(dA.as<T>() + nc * ld, 0, sizeof(T) * ld * (st.dA_zero - nc), s));
            st.dA_zero = nc;
        }
        st.dA_zero = std::max(st.dA_zero, ncp);
        if (mma) {
            const int64_t nc128 = round_up(nc, GT);
            launch_pair_features<T>(K, st.pX + off * d, nc, d, dXm.as<T>(), true, dFV.as<T>(), nc128, s,
                                    dflag.as<int>());
            launch_kcross_mma<T>(K, dKd.as<KCanon<T>>(), dFU.as<T>(), Mp, M, dFV.as<T>(), nc128, nc, d, dA.as<T>(), ld,
                                 dflag.as<int>(), s, fused ? st.pY + off : nullptr,
                                 fused ? dKY.as<T>() : nullptr);
            if (fused)  // label row Mp of partial 0, in chunk order
                launch_ky_reduce<T>(dKY.as<T>(), Mp, (int)(nc128 / GT), M, is2, dS.as<T>(), ld, Mp, s);
        } else {
            const T* tabc = nullptr;
            if (K.nper > 0) {
                launch_sincos_tables<T>(K, st.pX + off * d, nc, d, dtx.as<T>(), s);
                tabc = dtx.as<T>();
            }
            launch_kbuild<T>(K, dXm.as<T>(), dtm.as<T>(), M, st.pX + off * d, tabc, nc, d, dA.as<T>(), ld, 0,
                             false, T(0), dflag.as<int>(), s);
        }
        if (!fused) launch_label_rows<T>(st.pY + off * m, nc, m, dA.as<T>(), ld, Mp, ncp, mp, s);
        const int64_t kpart = round_up((ncp + P - 1) / P, 16);  // zero-padded columns make up the rest
        const int Pc = (int)((ncp + kpart - 1) / kpart);
        launch_syrk_splitk<T>(dS.as<T>(), ld, sstride, dA.as<T>(), ld, fused ? Mp : ld, Mp, kpart, Pc, is2, s);
    }
    launch_sum_partials<T>(dS.as<T>(), sstride, P, s);  // dS[0] += dS[1..P-1]
    if (ctx->comm) {  // rows sharded over the ranks: sum the partial normal equations
        rccl_settle(ctx->comm, ncclAllReduce(dS.p, dS.p, (size_t)(ld * Mp), nccl_type<T>(), ncclSum, ctx->comm, s),
                    "ncclAllReduce");
    } else if (ctx->peer && ctx->world > 1) {  // the caller's collective (host round trip)
        hostcoll_allreduce_dev<T>(ctx->hc, dS.as<T>(), (int)(ld * Mp), s);
    }
    // ---- S = K + accumulated; K separately for Kinv ----------------------------------------
    dK.ensure(sizeof(T) * Mp * Mp);
    launch_kbuild<T>(K, dXm.as<T>(), dtm.as<T>(), M, dXm.as<T>(), dtm.as<T>(), M, d, dK.as<T>(), Mp, Mp, true,
                     T(jitter), dflag.as<int>(), s);
    launch_gemm_add_lower<T>(dS.as<T>(), ld, dK.as<T>(), Mp, M, s);  // S[:M,:M] (lower) += K
    launch_set_identity_pad<T>(dS.as<T>(), ld, M, Mp, s);
    int hflag = 0;
    download(&hflag, dflag.p, sizeof(int), s);
    if (hflag)
        throw Error{GPRX_ERR_NONFINITE,
                    "GaussianProcess::ComputeKernelMatrixInternal: kernel matrix contains entries which are not finite."};
    // ---- S = L L^T with b in the extra rows -> RV; S^{-1} -> RM -----------------------------
    dLinv.ensure(sizeof(T) * Mp * DB);
    GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)dinfo.p, INT_MAX, 1, s));
    potrf_auto<T>(dS.as<T>(), ld, Mp, ld, dLinv.as<T>(), dinfo.as<int>(), ctx->ex);
    int hinfo = 0;
    download(&hinfo, dinfo.p, sizeof(int), s);
    check_sched(hinfo);
    if (hinfo != INT_MAX)
        throw Error{GPRX_ERR_NOT_SPD, "gprx_sparse_fit: K + sigma^-2 Knm^T Knm is not positive definite (pivot " +
                                          std::to_string(hinfo) + ")"};
}

// Kmm + jitter I = L L^T in place (dK, ld Mp); Linv blocks into dLinvK.
template <typename T>
static void sparse_factor_kmm(gprx_ctx* ctx, SparseNE<T>& st) {
    hipStream_t s = ctx->stream;
    const int64_t Mp = st.Mp;
    int hinfo = 0;
    st.dLinvK.ensure(sizeof(T) * Mp * DB);
    GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)st.dinfo.p, INT_MAX, 1, s));
    potrf_auto<T>(st.dK.template as<T>(), Mp, Mp, Mp, st.dLinvK.template as<T>(), st.dinfo.template as<int>(), ctx->ex);
    download(&hinfo, st.dinfo.p, sizeof(int), s);
    check_sched(hinfo);
    if (hinfo != INT_MAX)
        throw Error{GPRX_ERR_NOT_SPD,
                    "gprx_sparse_fit: Kmm + jitter I is not positive definite (pivot " + std::to_string(hinfo) + ")"};
}

template <typename T>
static gprx_status sparse_fit_impl(gprx_ctx* ctx, const gprx_kernel_desc* desc, const void* Xh, const void* Yh,
                                   int64_t n, int d, int m, const void* Xmh, int64_t M, double sigma, double jitter,
                                   void* Kinv, void* RV, void* RM) {
    SparseNE<T>& st = sparse_state<T>(ctx);
    sparse_normal_eq<T>(ctx, st, desc, Xh, Yh, n, d, m, Xmh, M, sigma, jitter);
    hipStream_t s = ctx->stream;
    const int64_t Mp = st.Mp, ld = st.ld;
    DevBuf &dS = st.dS, &dK = st.dK, &dLinv = st.dLinv, &dz = st.dz, &dalpha = st.dalpha, &dV = st.dV, &dC = st.dC;
    if (RV) {
        dz.ensure(sizeof(T) * m * Mp);
        dalpha.ensure(sizeof(T) * Mp * m);
        launch_backsolve<T>(dS.as<T>(), ld, Mp, m, dLinv.as<T>(), dz.as<T>(), dalpha.as<T>(), s);
        download(RV, dalpha.p, sizeof(T) * M * m, s);
    }
    dV.ensure(sizeof(T) * Mp * Mp);
    dC.ensure(sizeof(T) * Mp * Mp);
    if (RM) {
        launch_spd_inverse_from_factor<T>(dS.as<T>(), ld, Mp, dLinv.as<T>(), dV.as<T>(), dC.as<T>(), s);
        download_sym<T>(RM, dC, Mp, M, s);
    }
    // ---- Kinv ------------------------------------------------------------------------------
    if (Kinv) {
        sparse_factor_kmm<T>(ctx, st);
        launch_spd_inverse_from_factor<T>(dK.as<T>(), Mp, Mp, st.dLinvK.template as<T>(), dV.as<T>(), dC.as<T>(), s);
        download_sym<T>(Kinv, dC, Mp, M, s);
    }
    return GPRX_OK;
}

// SparseGaussianLogLikelihood::GetValueAndParameterDerivatives (include/SparseLikelihood.h:
// 231-344) without the reference's N x N matrices.  With B = Kmm + jitter I +
// sigma^-2 Kmn Knm (the fit's S), Sigma = B^{-1}, u = sigma^-2 Sigma Kmn y (= RV) and
// Woodbury on C = sigma^2 I + Knm Kmm^{-1} Kmn:
//   y^T C^{-1} y = sigma^-2 y^T y - |L_B^{-1} b|^2                 (b = sigma^-2 Kmn y)
//   log|C|       = N log sigma^2 + log|B| - log|Kmm + jitter I|    (EfficientDeterminant, :132-145)
// and the derivative of C, A_p = D_p W^T + W D_p^T - W E_p W^T (W = Knm Kmm^{-1}, D_p = dKnm/dp,
// E_p = dKmm/dp, :246-252), collapses to
//   grad_p = sum_{i,a} D_p,ia Omega_ia + 1/2 sum_{a,b} E_p,ab (Kmm^{-1} - Sigma - u u^T)_ab,
//   Omega  = sigma^-2 [(y - Knm u) u^T - Knm Sigma]     (the data-fit and complexity terms, :255-273)
// so the N x M part needs one GEMM Knm Sigma per row chunk (2 N M^2 flops) and a weighted
// derivative sum over the chunk's pairs; the M x M part is the dense LML's gradient pass on the
// inducing points.  Rows shard over an RCCL context like the fit (one all-reduce of the
// partials).  compat: the reference's long-double product det(Kmm^{-1}) * sigma^{2N} * det(B)
// and its clamps (:148-158, 305-314), evaluated from the three log-determinants.
template <typename T>
static gprx_status sparse_lml_impl(gprx_ctx* ctx, const gprx_kernel_desc* desc, const void* Xh, const void* Yh,
                                   int64_t n, int d, int m, const void* Xmh, int64_t M, double sigma, double jitter,
                                   uint32_t flags, double* value, double* grad, int32_t* nparams, double* logdet) {
    GPRX_REQUIRE(M > 0, GPRX_ERR_DIM,
                 "SparseLikelihood::GetValueAndParameterDerivative: there are no inducing samples specified");
    GPRX_REQUIRE(m == 1, GPRX_ERR_DIM,
                 "SparseGaussianLogLikelihood: only one output dimension is supported (the reference's data-fit term "
                 "is m x m, include/SparseLikelihood.h:303)");
    GPRX_REQUIRE(n > 0, GPRX_ERR_DIM, "SparseGaussianProcess::ComputeCoreMatrices: empty sample set.");
    SparseNE<T>& st = sparse_state<T>(ctx);
    sparse_normal_eq<T>(ctx, st, desc, Xh, Yh, n, d, m, Xmh, M, sigma, jitter);
    sparse_factor_kmm<T>(ctx, st);
    hipStream_t s = ctx->stream;
    const KCanon<T>& K = st.K;
    const int64_t Mp = st.Mp, ld = st.ld, chunk = st.chunk, c128 = st.chunk128;
    const T is2 = st.is2;
    // [0] log|B|, [1] |L_B^{-1} b|^2, [2] log|Kmm + jitter|, [4] y^T y, partials after
    DevBuf red;
    red.ensure(sizeof(double) * (8 + 2 * (Mp / 128 + 2)));
    double* dred = red.as<double>();
    launch_fit_reductions<T>(st.dS.template as<T>(), ld, M, Mp, 1, dred + 8, s);
    GPRX_HIP(hipMemcpyAsync(dred, dred + 8, 2 * sizeof(double), hipMemcpyDeviceToDevice, s));
    launch_fit_reductions<T>(st.dK.template as<T>(), Mp, M, Mp, 0, dred + 8, s);
    GPRX_HIP(hipMemcpyAsync(dred + 2, dred + 8, sizeof(double), hipMemcpyDeviceToDevice, s));
    launch_sq_sum<T>(st.pY, n, dred + 4, s);
    double h[5];
    download(h, dred, sizeof(h), s);
    double yty = h[4], nn = (double)n;
    const bool want_grad = grad && (flags & GPRX_LML_GRAD);
    double acc_x[MAX_LEAF * 3] = {0}, acc_m[MAX_LEAF * 3] = {0};
    if (want_grad) {
        // u = Sigma b (the fit's RV), Sigma (full symmetric), H = Kmm^{-1} - Sigma (lower)
        st.dz.ensure(sizeof(T) * Mp);
        st.dalpha.ensure(sizeof(T) * Mp);
        launch_backsolve<T>(st.dS.template as<T>(), ld, Mp, 1, st.dLinv.template as<T>(), st.dz.template as<T>(), st.dalpha.template as<T>(), s);
        const T* u = st.dalpha.template as<T>();
        DevBuf dSig, dH;
        st.dV.ensure(sizeof(T) * Mp * Mp);
        dSig.ensure(sizeof(T) * Mp * Mp);
        dH.ensure(sizeof(T) * Mp * Mp);
        launch_spd_inverse_from_factor<T>(st.dS.template as<T>(), ld, Mp, st.dLinv.template as<T>(), st.dV.template as<T>(), dSig.as<T>(), s);
        launch_sym_fill<T>(dSig.as<T>(), Mp, Mp, s);
        launch_spd_inverse_from_factor<T>(st.dK.template as<T>(), Mp, Mp, st.dLinvK.template as<T>(), st.dV.template as<T>(), dH.as<T>(), s);
        launch_sub<T>(dH.as<T>(), dSig.as<T>(), dH.as<T>(), Mp * Mp, s);
        // ---- N x M part, chunk by chunk: A_t = K(Xc, Xm), r = sigma^-2 (y_c - A_t u),
        // G = sigma^-2 A_t Sigma, then sum (r_i u_a - G_ia) dk(x_i, xm_a)/dp ----
        const bool gmma = st.mma && pairs_grad_supported<T>(K);
        DevBuf dAt, dG, dr, dFUc, dFVm, dGU, dGV, part, acc;
        dAt.ensure(sizeof(T) * c128 * Mp);
        dG.ensure(sizeof(T) * c128 * Mp);
        dr.ensure(sizeof(T) * c128);
        acc.ensure(sizeof(double) * MAX_LEAF * 3);
        const int64_t fc = pairs_feature_cols<T>(K, d), kg = std::max<int64_t>(1, pairs_grad_feature_cols<T>(K, d));
        if (st.mma) {
            dFUc.ensure(sizeof(T) * c128 * fc);
            dFVm.ensure(sizeof(T) * Mp * fc);
            launch_pair_features<T>(K, st.dXm.template as<T>(), M, d, st.dXm.template as<T>(), true, dFVm.as<T>(), Mp, s,
                                    st.dflag.template as<int>());
        }
        if (gmma) {
            dGU.ensure(sizeof(T) * c128 * kg);
            dGV.ensure(sizeof(T) * Mp * kg);
            part.ensure(sizeof(double) * MAX_LEAF * 3 * (c128 / GT) * (Mp / GT));
        } else {
            GPRX_HIP(hipMemsetAsync(acc.p, 0, sizeof(double) * MAX_LEAF * 3, s));
        }
        for (int64_t off = 0; off < n; off += chunk) {
            const int64_t nc = std::min(chunk, n - off), nc128 = round_up(nc, GT);
            const T* Xc = st.pX + off * d;
            if (nc < chunk || off == 0) GPRX_HIP(hipMemsetAsync(dAt.p, 0, sizeof(T) * c128 * Mp, s));
            const T* tabc = nullptr;
            if (st.mma) {
                launch_pair_features<T>(K, Xc, nc, d, st.dXm.template as<T>(), false, dFUc.as<T>(), nc128, s,
                                        st.dflag.template as<int>());
                launch_kcross_mma<T>(K, st.dKd.template as<KCanon<T>>(), dFUc.as<T>(), nc128, nc, dFVm.as<T>(), Mp, M, d,
                                     dAt.as<T>(), c128, st.dflag.template as<int>(), s, nullptr, nullptr);
            } else {
                if (K.nper > 0) {
                    launch_sincos_tables<T>(K, Xc, nc, d, st.dtx.template as<T>(), s);
                    tabc = st.dtx.template as<T>();
                }
                launch_kbuild<T>(K, Xc, tabc, nc, st.dXm.template as<T>(), st.dtm.template as<T>(), M, d, dAt.as<T>(), c128, 0, false,
                                 T(0), st.dflag.template as<int>(), s);
            }
            launch_sparse_resid<T>(dAt.as<T>(), c128, nc, M, u, st.pY + off, is2, dr.as<T>(), s);
            launch_gemm_nt<T>(dG.as<T>(), c128, dAt.as<T>(), c128, dSig.as<T>(), Mp, nc128, Mp, Mp, is2, T(0), false,
                              s);
            if (gmma) {
                launch_lml_grad_mma_cross<T>(K, st.dKd.template as<KCanon<T>>(), Xc, nc, st.dXm.template as<T>(), M, st.dXm.template as<T>(), d,
                                             dFUc.as<T>(), nc128, dFVm.as<T>(), Mp, dGU.as<T>(), dGV.as<T>(), dr.as<T>(),
                                             u, dG.as<T>(), c128, part.as<double>(), acc.as<double>(), s);
                double a[MAX_LEAF * 3];
                download(a, acc.p, sizeof(a), s);
                for (int q = 0; q < MAX_LEAF * 3; q++) acc_x[q] += a[q];  // chunk order: deterministic
            } else {
                launch_lml_grad_cross<T>(K, Xc, tabc, nc, st.dXm.template as<T>(), st.dtm.template as<T>(), M, d, dr.as<T>(), u,
                                         dG.as<T>(), c128, acc.as<double>(), s);
            }
        }
        if (!gmma) download(acc_x, acc.p, sizeof(acc_x), s);
        // ---- M x M part: sum (u_a u_b - H_ab) dKmm_ab/dp (the dense LML's pass, weights
        // alpha alpha^T - C with alpha = u, C = H) ----
        const int64_t ntm = Mp / GT;
        if (gmma) {
            DevBuf dFUm, dFVm2, dGUm, dGVm, partm;
            dFUm.ensure(sizeof(T) * Mp * fc);
            dFVm2.ensure(sizeof(T) * Mp * fc);
            dGUm.ensure(sizeof(T) * Mp * kg);
            dGVm.ensure(sizeof(T) * Mp * kg);
            partm.ensure(sizeof(double) * MAX_LEAF * 3 * ntm * (ntm + 1) / 2);
            launch_pair_features<T>(K, st.dXm.template as<T>(), M, d, st.dXm.template as<T>(), false, dFUm.as<T>(), Mp, s);
            launch_pair_features<T>(K, st.dXm.template as<T>(), M, d, st.dXm.template as<T>(), true, dFVm2.as<T>(), Mp, s);
            launch_lml_grad_mma<T>(K, st.dKd.template as<KCanon<T>>(), st.dXm.template as<T>(), M, d, dFUm.as<T>(), dFVm2.as<T>(),
                                   dGUm.as<T>(), dGVm.as<T>(), Mp, u, dH.as<T>(), Mp, partm.as<double>(),
                                   acc.as<double>(), s);
        } else {
            GPRX_HIP(hipMemsetAsync(acc.p, 0, sizeof(double) * MAX_LEAF * 3, s));
            launch_lml_grad<T>(K, st.dXm.template as<T>(), st.dtm.template as<T>(), M, d, u, dH.as<T>(), Mp, acc.as<double>(), s);
        }
        download(acc_m, acc.p, sizeof(acc_m), s);
    }
    int hflag = 0;
    download(&hflag, st.dflag.p, sizeof(int), s);
    if (hflag)
        throw Error{GPRX_ERR_NONFINITE,
                    "GaussianProcess::ComputeKernelMatrixInternal: kernel matrix contains entries which are not finite."};
    if (ctx->comm || (ctx->peer && ctx->world > 1)) {  // rows sharded over the ranks: the data terms and the N x M gradient partials
        // (the M x M part is the same on every rank: added once, after the reduction)
        double loc[MAX_LEAF * 3 + 2];
        for (int q = 0; q < MAX_LEAF * 3; q++) loc[q] = acc_x[q];
        loc[MAX_LEAF * 3] = yty;
        loc[MAX_LEAF * 3 + 1] = nn;
        DevBuf dl;
        upload<double>(dl, loc, sizeof(loc), s);
        if (ctx->comm) {
            rccl_settle(ctx->comm, ncclAllReduce(dl.p, dl.p, MAX_LEAF * 3 + 2, ncclFloat64, ncclSum, ctx->comm, s),
                        "ncclAllReduce");
        } else {
            hostcoll_allreduce_dev<double>(ctx->hc, dl.as<double>(), MAX_LEAF * 3 + 2, s);
        }
        download(loc, dl.p, sizeof(loc), s);
        for (int q = 0; q < MAX_LEAF * 3; q++) acc_x[q] = loc[q];
        yty = loc[MAX_LEAF * 3];
        nn = loc[MAX_LEAF * 3 + 1];
    }
    for (int q = 0; q < MAX_LEAF * 3; q++) acc_x[q] -= 0.5 * acc_m[q];  // replicated M x M part, once
    const double logdet_b = h[0], zz = h[1], logdet_k = h[2];
    const T s2 = T(sigma) * T(sigma);
    const double ld_c = nn * std::log((double)s2) + logdet_b - logdet_k;
    const T df = (T)(-0.5 * ((double)is2 * yty - zz));
    const T ct = (T)(-(nn / 2.0) * std::log(2 * M_PI));  // include/SparseLikelihood.h:198 (N dense samples)
    double v;
    if (flags & GPRX_LML_COMPAT) {
        typedef long double HP;
        HP det_b = std::exp(-(HP)logdet_k);  // det(Kmm^{-1}) (:138-141, inf clamped to max)
        if (std::isinf(det_b)) det_b = std::numeric_limits<HP>::max();
        const HP prod_a = std::exp((HP)nn * std::log((HP)s2));  // prod of the N noise entries
        const HP det = det_b * prod_a * std::exp((HP)logdet_b);
        HP cp;
        if (det <= std::numeric_limits<HP>::min() || std::isnan(det)) cp = -0.5L * std::log(std::numeric_limits<HP>::min());
        else if (det > std::numeric_limits<HP>::max()) cp = -0.5L * std::log(std::numeric_limits<HP>::max());
        else cp = -0.5L * std::log(det);
        v = (double)(T)(df + (T)(cp + (HP)ct));
    } else {
        v = (double)df - 0.5 * ld_c + (double)ct;
    }
    if (std::isnan(v))
        throw Error{GPRX_ERR_NONFINITE, "SparseLikelihood::GetValueAndParameterDerivative: likelihood value is not a number."};
    if (value) *value = v;
    if (logdet) *logdet = ld_c;
    if (nparams) *nparams = K.nparams;
    if (want_grad) {
        for (int l = 0; l < K.nleaf; l++) {
            const int t = K.leaf[l].type;
            const int npl = (t == L_WHITE) ? 1 : ((t == L_GAUSS || t == L_GAUSS_EXP) ? 2 : 3);
            for (int q = 0; q < npl; q++) grad[K.param_base[l] + q] = acc_x[l * 3 + q];
        }
    }
    return GPRX_OK;
}

// ---------------------------------------------------------------------------------------
// C ABI
// ---------------------------------------------------------------------------------------
extern "C" {

int gprx_abi_version(void) { return GPRX_ABI_VERSION; }

gprx_status gprx_device_count(int* count) {
    API_BEGIN
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) c = 0;
    if (count) *count = c;
    return GPRX_OK;
    API_END(nullptr)
}

static gprx_ctx* ctx_new(int device) {
    int c = 0;
    if (hipGetDeviceCount(&c) != hipSuccess || c == 0)
        throw Error{GPRX_ERR_NO_DEVICE, "gprx_ctx_create: no HIP device visible (libgprx has no CPU fallback)"};
    GPRX_REQUIRE(device >= 0 && device < c, GPRX_ERR_ARG, "gprx_ctx_create: bad device index");
    GPRX_HIP(hipSetDevice(device));
    gprx_ctx* ctx = new gprx_ctx();
    ctx->device = device;
    // The main stream carries the factorisation's critical path (panel chain): give it the
    // highest priority so its small kernels are dispatched ahead of the bulk trailing update
    // running on the aux stream.
    int prio_lo = 0, prio_hi = 0;
    GPRX_HIP(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    GPRX_HIP(hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, prio_hi));
    // The aux stream (bulk trailing updates) is kept off a few CUs so the panel chain's
    // one-workgroup diagonal kernels never queue behind a full-chip GEMM: GPRX_RESERVE_CU
    // CUs (default 0 = off: measured no gain; 8 = one per XCD when CUs are numbered XCD-major) are excluded from its mask.
    int reserve = 0;
    if (const char* e = std::getenv("GPRX_RESERVE_CU")) reserve = std::atoi(e);
    hipDeviceProp_t prop;
    GPRX_HIP(hipGetDeviceProperties(&prop, device));
    const int ncu = prop.multiProcessorCount;
    if (reserve > 0 && reserve < ncu) {
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        const int per = std::max(1, reserve / 8), stride = std::max(1, ncu / 8);
        int excluded = 0;
        for (int i = 0; i < ncu; i++) {
            const bool res = (i % stride) < per && excluded < reserve;
            if (res) excluded++;
            else mask[i / 32] |= 1u << (i % 32);
        }
        GPRX_HIP(hipExtStreamCreateWithCUMask(&ctx->aux, (uint32_t)mask.size(), mask.data()));
    } else {
        GPRX_HIP(hipStreamCreateWithPriority(&ctx->aux, hipStreamNonBlocking, prio_lo));
    }
    GPRX_HIP(hipStreamCreateWithPriority(&ctx->aux2, hipStreamNonBlocking, prio_hi));
    ctx->ex.s0 = ctx->stream;
    ctx->ex.s1 = ctx->aux;
    ctx->ex.s2 = ctx->aux2;
    for (auto& e : ctx->ev) GPRX_HIP(hipEventCreate(&e));
    return ctx;
}

gprx_status gprx_ctx_create(int device, gprx_ctx** out) {
    API_BEGIN
    GPRX_REQUIRE(out, GPRX_ERR_ARG, "gprx_ctx_create: out is NULL");
    *out = ctx_new(device);
    return GPRX_OK;
    API_END(nullptr)
}

void gprx_ctx_destroy(gprx_ctx* ctx) {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    for (auto& e : ctx->ev)
        if (e) (void)hipEventDestroy(e);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
    if (ctx->aux2) (void)hipStreamDestroy(ctx->aux2);
    delete ctx->hc;
    // abort, not destroy: local, never waits on the peers (a communicator whose collective
    // timed out, or whose peers already left, would block ncclCommDestroy); every stream of
    // this context has drained by now
    if (ctx->comm) (void)ncclCommAbort(ctx->comm);
    delete ctx;
}

const char* gprx_last_error(const gprx_ctx* ctx) { return ctx ? ctx->err.c_str() : t_last_error.c_str(); }

gprx_status gprx_model_create(gprx_ctx* ctx, gprx_dtype dtype, gprx_model** out) {
    API_BEGIN
    GPRX_REQUIRE(ctx && out, GPRX_ERR_ARG, "gprx_model_create: NULL argument");
    GPRX_REQUIRE(dtype == GPRX_F32 || dtype == GPRX_F64, GPRX_ERR_ARG, "gprx_model_create: bad dtype");
    gprx_model* m = new gprx_model();
    m->ctx = ctx;
    m->dt = dtype;
    *out = m;
    return GPRX_OK;
    API_END(ctx)
}

void gprx_model_destroy(gprx_model* model) {
    if (!model) return;
    (void)hipSetDevice(model->ctx->device);
    delete model;
}

gprx_status gprx_model_set_data(gprx_model* M, const void* X, const void* Y, int64_t n, int32_t d, int32_t m) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M && X && Y, GPRX_ERR_ARG, "gprx_model_set_data: NULL argument");
    GPRX_REQUIRE(n > 0, GPRX_ERR_STATE, "GaussianProcess::Initialize: no input samples defined during initialization");
    GPRX_REQUIRE(d > 0 && m > 0, GPRX_ERR_DIM, "gprx_model_set_data: input and output dimensions must be positive");
    ModelLock lk(M);
    GPRX_HIP(hipSetDevice(ctx->device));
    const size_t es = esize(M->dt);
    M->X.ensure(es * n * d);
    M->Y.ensure(es * n * m);
    M->trim_posterior_workspace();
    // host or device memory (include/gprx.h conventions: a gprx_device_alloc pointer too)
    GPRX_HIP(hipMemcpy(M->X.p, X, es * n * d, hipMemcpyDefault));
    GPRX_HIP(hipMemcpy(M->Y.p, Y, es * n * m, hipMemcpyDefault));
    M->n = n;
    M->d = d;
    M->m = m;
    M->has_data = true;
    M->sparse_cov = false;
    M->fitted = false;
    M->has_alpha = false;
    M->inv_ready = false;
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_model_set_kernel(gprx_model* M, const gprx_kernel_desc* k) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M && k, GPRX_ERR_ARG, "gprx_model_set_kernel: NULL argument");
    ModelLock lk(M);
    std::string e = (M->dt == GPRX_F64) ? canonicalize<double>(*k, M->kd) : canonicalize<float>(*k, M->kf);
    GPRX_REQUIRE(e.empty(), GPRX_ERR_ARG, e);
    if (M->dt == GPRX_F32) {  // the fp64 form of the fp32 tree (its parameters rounded to float)
        gprx_kernel_desc k32 = *k;
        for (int i = 0; i < k32.n_nodes && i < GPRX_MAX_KNODES; i++)
            for (int q = 0; q < 3; q++) k32.node[i].p[q] = (double)(float)k32.node[i].p[q];
        e = canonicalize<double>(k32, M->kd);
        GPRX_REQUIRE(e.empty(), GPRX_ERR_ARG, e);
    }
    M->desc = *k;
    M->has_kernel = true;
    M->host_k = false;
    M->fitted = false;
    M->has_alpha = false;
    M->inv_ready = false;
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_model_set_noise(gprx_model* M, double sigma) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M, GPRX_ERR_ARG, "gprx_model_set_noise: NULL model");
    ModelLock lk(M);
    M->sigma = sigma;
    M->fitted = false;
    M->has_alpha = false;
    M->inv_ready = false;
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_model_fit(gprx_model* M, uint32_t flags, gprx_fit_info* info) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M, GPRX_ERR_ARG, "gprx_model_fit: NULL model");
    ModelLock lk(M);
    ProfBind pb_(ctx);  // after the lock: resolved (streams drained) before it is released
    return M->dt == GPRX_F64 ? model_fit<double>(M, flags, info) : model_fit<float>(M, flags, info);
    API_END(ctx)
}

gprx_status gprx_model_get_alpha(gprx_model* M, void* alpha) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M && alpha, GPRX_ERR_ARG, "gprx_model_get_alpha: NULL argument");
    ModelLock lk(M);
    GPRX_REQUIRE(M->has_alpha, GPRX_ERR_STATE, "gprx: model is not fitted");
    GPRX_HIP(hipSetDevice(ctx->device));
    GPRX_HIP(hipMemcpy(alpha, M->alpha.p, esize(M->dt) * M->n * M->m, hipMemcpyDeviceToHost));
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_model_set_alpha(gprx_model* M, const void* alpha) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M && alpha, GPRX_ERR_ARG, "gprx_model_set_alpha: NULL argument");
    ModelLock lk(M);
    GPRX_REQUIRE(M->has_data && M->has_kernel, GPRX_ERR_STATE, "gprx_model_set_alpha: set data and kernel first");
    GPRX_HIP(hipSetDevice(ctx->device));
    const size_t es = esize(M->dt);
    M->alpha.ensure(es * M->n * M->m);
    GPRX_HIP(hipStreamSynchronize(ctx->stream));
    GPRX_HIP(hipMemcpy(M->alpha.p, alpha, es * M->n * M->m, hipMemcpyHostToDevice));
    if (M->dt == GPRX_F64 ? M->kd.nper > 0 : M->kf.nper > 0) {
        const int nper = M->dt == GPRX_F64 ? M->kd.nper : M->kf.nper;
        M->tab.ensure(es * 2 * nper * M->n * M->d);
        if (M->dt == GPRX_F64)
            launch_sincos_tables<double>(M->kd, M->X.as<double>(), M->n, M->d, M->tab.as<double>(), ctx->stream);
        else
            launch_sincos_tables<float>(M->kf, M->X.as<float>(), M->n, M->d, M->tab.as<float>(), ctx->stream);
        GPRX_HIP(hipStreamSynchronize(ctx->stream));
    }
    M->has_alpha = true;  // the factor (if any) is left as it is
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_model_predict(gprx_model* M, const void* Xq, int64_t q, void* mean, void* deriv) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M && Xq && mean, GPRX_ERR_ARG, "gprx_model_predict: NULL argument");
    if (q == 0) return GPRX_OK;
    ModelLock lk(M);
    ProfBind pb_(ctx);  // after the lock: resolved (streams drained) before it is released
    GPRX_HIP(hipSetDevice(ctx->device));
    return M->dt == GPRX_F64 ? model_predict<double>(M, Xq, q, mean, deriv)
                             : model_predict<float>(M, Xq, q, mean, deriv);
    API_END(ctx)
}

gprx_status gprx_model_posterior_cov(gprx_model* M, const void* Xa, const void* Xb, int64_t q, void* out) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M && q >= 0, GPRX_ERR_ARG, "gprx_model_posterior_cov: NULL model or negative q");
    // on a sharded fit of a multi-process context this is a collective call (gprx.h): a process
    // with no pairs of its own still takes part
    const bool collective = M->dist_fitted && ctx->hc && ctx->world > 1;
    if (q == 0 && !collective) return GPRX_OK;
    GPRX_REQUIRE(q == 0 || (Xa && Xb && out), GPRX_ERR_ARG, "gprx_model_posterior_cov: NULL argument");
    ModelLock lk(M);
    ProfBind pb_(ctx);  // after the lock: resolved (streams drained) before it is released
    GPRX_HIP(hipSetDevice(ctx->device));
    return M->dt == GPRX_F64 ? model_posterior_cov<double>(M, Xa, Xb, q, out)
                             : model_posterior_cov<float>(M, Xa, Xb, q, out);
    API_END(ctx)
}

gprx_status gprx_model_core_matrix(gprx_model* M, void* C) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M && C, GPRX_ERR_ARG, "gprx_model_core_matrix: NULL argument");
    ModelLock lk(M);
    ProfBind pb_(ctx);  // after the lock: resolved (streams drained) before it is released
    GPRX_HIP(hipSetDevice(ctx->device));
    return M->dt == GPRX_F64 ? model_core_matrix<double>(M, C) : model_core_matrix<float>(M, C);
    API_END(ctx)
}

gprx_status gprx_model_lml(gprx_model* M, uint32_t flags, double* value, double* grad, int32_t* nparams,
                           double* logdet) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M, GPRX_ERR_ARG, "gprx_model_lml: NULL model");
    ModelLock lk(M);
    ProfBind pb_(ctx);  // after the lock: resolved (streams drained) before it is released
    GPRX_HIP(hipSetDevice(ctx->device));
    return M->dt == GPRX_F64 ? model_lml<double>(M, flags, value, grad, nparams, logdet)
                             : model_lml<float>(M, flags, value, grad, nparams, logdet);
    API_END(ctx)
}

gprx_status gprx_model_set_sparse_cov(gprx_model* M, const void* W) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M && W, GPRX_ERR_ARG, "gprx_model_set_sparse_cov: NULL argument");
    ModelLock lk(M);
    GPRX_REQUIRE(M->has_data && M->has_kernel && !M->host_k, GPRX_ERR_STATE,
                 "gprx_model_set_sparse_cov: set the inducing points and the kernel first");
    GPRX_HIP(hipSetDevice(ctx->device));
    const int64_t n = M->n, Mp = round_up(n, GT);
    const size_t es = esize(M->dt);
    std::vector<unsigned char> h(es * Mp * Mp, 0);  // padded, column-major
    for (int64_t i = 0; i < n; i++)
        for (int64_t j = 0; j < n; j++)
            std::memcpy(&h[es * (i + j * Mp)], static_cast<const unsigned char*>(W) + es * (i * n + j), es);
    M->sparseW.ensure(h.size());
    GPRX_HIP(hipStreamSynchronize(ctx->stream));
    GPRX_HIP(hipMemcpy(M->sparseW.p, h.data(), h.size(), hipMemcpyHostToDevice));
    const int nper = M->dt == GPRX_F64 ? M->kd.nper : M->kf.nper;
    if (nper > 0) {  // the inducing points' sin/cos tables
        M->tab.ensure(es * 2 * nper * n * M->d);
        if (M->dt == GPRX_F64)
            launch_sincos_tables<double>(M->kd, M->X.as<double>(), n, M->d, M->tab.as<double>(), ctx->stream);
        else
            launch_sincos_tables<float>(M->kf, M->X.as<float>(), n, M->d, M->tab.as<float>(), ctx->stream);
    }
    M->flag.ensure(sizeof(int));
    GPRX_HIP(hipMemsetAsync(M->flag.p, 0, sizeof(int), ctx->stream));
    GPRX_HIP(hipStreamSynchronize(ctx->stream));
    M->sparse_cov = true;
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_model_set_kernel_matrix(gprx_model* M, const void* K) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M && K, GPRX_ERR_ARG, "gprx_model_set_kernel_matrix: NULL argument");
    ModelLock lk(M);
    GPRX_REQUIRE(M->has_data, GPRX_ERR_STATE, "gprx_model_set_kernel_matrix: set the data first");
    GPRX_HIP(hipSetDevice(ctx->device));
    const size_t es = esize(M->dt);
    M->Kext.ensure(es * M->n * M->n);
    GPRX_HIP(hipStreamSynchronize(ctx->stream));
    GPRX_HIP(hipMemcpy(M->Kext.p, K, es * M->n * M->n, hipMemcpyHostToDevice));
    std::memset(&M->kd, 0, sizeof(M->kd));  // no device form: nothing else reads the tree
    std::memset(&M->kf, 0, sizeof(M->kf));
    std::memset(&M->desc, 0, sizeof(M->desc));
    M->host_k = true;
    M->has_kernel = true;
    M->fitted = false;
    M->has_alpha = false;
    M->inv_ready = false;
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_model_predict_kx(gprx_model* M, const void* Kx, const void* Xq, int64_t q, void* mean, void* deriv) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M && Kx && mean, GPRX_ERR_ARG, "gprx_model_predict_kx: NULL argument");
    if (q == 0) return GPRX_OK;
    ModelLock lk(M);
    GPRX_HIP(hipSetDevice(ctx->device));
    return M->dt == GPRX_F64 ? model_predict_kx<double>(M, Kx, Xq, q, mean, deriv)
                             : model_predict_kx<float>(M, Kx, Xq, q, mean, deriv);
    API_END(ctx)
}

gprx_status gprx_model_posterior_cov_kx(gprx_model* M, const void* Kxa, const void* Kxb, const void* kab, int64_t q,
                                        void* out) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M && Kxa && Kxb && kab && out, GPRX_ERR_ARG, "gprx_model_posterior_cov_kx: NULL argument");
    if (q == 0) return GPRX_OK;
    ModelLock lk(M);
    GPRX_HIP(hipSetDevice(ctx->device));
    return M->dt == GPRX_F64 ? model_posterior_cov_kx<double>(M, Kxa, Kxb, kab, q, out)
                             : model_posterior_cov_kx<float>(M, Kxa, Kxb, kab, q, out);
    API_END(ctx)
}

gprx_status gprx_model_lml_dk(gprx_model* M, uint32_t flags, const void* dK, int32_t P, double* value, double* grad,
                              double* logdet) {
    gprx_ctx* ctx = M ? M->ctx : nullptr;
    API_BEGIN
    GPRX_REQUIRE(M, GPRX_ERR_ARG, "gprx_model_lml_dk: NULL model");
    ModelLock lk(M);
    ProfBind pb_(ctx);
    GPRX_HIP(hipSetDevice(ctx->device));
    return M->dt == GPRX_F64 ? model_lml_dk<double>(M, flags, dK, P, value, grad, logdet)
                             : model_lml_dk<float>(M, flags, dK, P, value, grad, logdet);
    API_END(ctx)
}

gprx_status gprx_kernel_matrix(gprx_ctx* ctx, gprx_dtype dt, const gprx_kernel_desc* k, const void* X, int64_t n,
                               int32_t d, void* K) {
    API_BEGIN
    GPRX_REQUIRE(ctx && k && X && K, GPRX_ERR_ARG, "gprx_kernel_matrix: NULL argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ProfBind pb_(ctx);  // after the lock: resolved (streams drained) before it is released
    GPRX_HIP(hipSetDevice(ctx->device));
    return dt == GPRX_F64 ? kernel_matrix_impl<double>(ctx, k, X, n, d, K, false)
                          : kernel_matrix_impl<float>(ctx, k, X, n, d, K, false);
    API_END(ctx)
}

gprx_status gprx_deriv_matrix(gprx_ctx* ctx, gprx_dtype dt, const gprx_kernel_desc* k, const void* X, int64_t n,
                              int32_t d, void* D) {
    API_BEGIN
    GPRX_REQUIRE(ctx && k && X && D, GPRX_ERR_ARG, "gprx_deriv_matrix: NULL argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ProfBind pb_(ctx);  // after the lock: resolved (streams drained) before it is released
    GPRX_HIP(hipSetDevice(ctx->device));
    return dt == GPRX_F64 ? kernel_matrix_impl<double>(ctx, k, X, n, d, D, true)
                          : kernel_matrix_impl<float>(ctx, k, X, n, d, D, true);
    API_END(ctx)
}

gprx_status gprx_cross_matrix(gprx_ctx* ctx, gprx_dtype dt, const gprx_kernel_desc* k, const void* A, int64_t na,
                              const void* B, int64_t nb, int32_t d, void* K) {
    API_BEGIN
    GPRX_REQUIRE(ctx && k && A && B && K, GPRX_ERR_ARG, "gprx_cross_matrix: NULL argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ProfBind pb_(ctx);  // after the lock: resolved (streams drained) before it is released
    GPRX_HIP(hipSetDevice(ctx->device));
    return dt == GPRX_F64 ? cross_matrix_impl<double>(ctx, k, A, na, B, nb, d, K)
                          : cross_matrix_impl<float>(ctx, k, A, na, B, nb, d, K);
    API_END(ctx)
}

gprx_status gprx_cholesky(gprx_ctx* ctx, gprx_dtype dt, void* A, int64_t n, int32_t* info) {
    API_BEGIN
    GPRX_REQUIRE(ctx && A && n > 0, GPRX_ERR_ARG, "gprx_cholesky: bad argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ProfBind pb_(ctx);  // after the lock: resolved (streams drained) before it is released
    GPRX_HIP(hipSetDevice(ctx->device));
    gprx_status st = dt == GPRX_F64 ? cholesky_impl<double>(ctx, A, n, info, false)
                                    : cholesky_impl<float>(ctx, A, n, info, false);
    if (st == GPRX_ERR_NOT_SPD) return fail(ctx, st, "gprx_cholesky: matrix is not positive definite");
    return st;
    API_END(ctx)
}

gprx_status gprx_spd_inverse(gprx_ctx* ctx, gprx_dtype dt, void* A, int64_t n, int32_t* info) {
    API_BEGIN
    GPRX_REQUIRE(ctx && A && n > 0, GPRX_ERR_ARG, "gprx_spd_inverse: bad argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ProfBind pb_(ctx);  // after the lock: resolved (streams drained) before it is released
    GPRX_HIP(hipSetDevice(ctx->device));
    return dt == GPRX_F64 ? cholesky_impl<double>(ctx, A, n, info, true) : cholesky_impl<float>(ctx, A, n, info, true);
    API_END(ctx)
}

static const char* kclass_name(int c) {
    static const char* names[KC_COUNT] = {"kbuild", "potrf_diag", "potrf_trsm", "potrf_update", "backsolve",
                                          "predict", "lml_grad", "spd_inverse", "other_gemm", "potrf_tiles",
                                          "posterior"};
    return names[c];
}

gprx_status gprx_ctx_set_stats(gprx_ctx* ctx, int32_t enable) {
    API_BEGIN
    GPRX_REQUIRE(ctx, GPRX_ERR_ARG, "gprx_ctx_set_stats: NULL ctx");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ctx->prof.on = enable != 0;
    ctx->prof.reset();
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_device_alloc(gprx_ctx* ctx, int64_t bytes, void** out) {
    API_BEGIN
    GPRX_REQUIRE(ctx && out && bytes >= 0, GPRX_ERR_ARG, "gprx_device_alloc: NULL argument or negative size");
    *out = nullptr;
    if (bytes == 0) return GPRX_OK;
    void* p = nullptr;
    GPRX_HIP(hipSetDevice(ctx->device));
    const hipError_t e = hipMalloc(&p, (size_t)bytes);
    if (e != hipSuccess)
        throw Error{GPRX_ERR_OOM, std::string("gprx_device_alloc: hipMalloc: ") + hipGetErrorString(e)};
    *out = p;
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_device_free(gprx_ctx* ctx, void* p) {
    API_BEGIN
    GPRX_REQUIRE(ctx, GPRX_ERR_ARG, "gprx_device_free: NULL ctx");
    if (p) {
        GPRX_HIP(hipStreamSynchronize(ctx->stream));  // (no launch may still read it)
        GPRX_HIP(hipFree(p));
    }
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_device_upload(gprx_ctx* ctx, void* dst, const void* src, int64_t bytes) {
    API_BEGIN
    GPRX_REQUIRE(ctx && (bytes == 0 || (dst && src)) && bytes >= 0, GPRX_ERR_ARG, "gprx_device_upload: bad argument");
    if (bytes > 0) {
        GPRX_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyHostToDevice, ctx->stream));
        GPRX_HIP(hipStreamSynchronize(ctx->stream));
    }
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_device_download(gprx_ctx* ctx, void* dst, const void* src, int64_t bytes) {
    API_BEGIN
    GPRX_REQUIRE(ctx && (bytes == 0 || (dst && src)) && bytes >= 0, GPRX_ERR_ARG, "gprx_device_download: bad argument");
    if (bytes > 0) {
        GPRX_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, hipMemcpyDeviceToHost, ctx->stream));
        GPRX_HIP(hipStreamSynchronize(ctx->stream));
    }
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_ctx_get_stats(gprx_ctx* ctx, gprx_kstat* out, int32_t max, int32_t* count) {
    API_BEGIN
    GPRX_REQUIRE(ctx, GPRX_ERR_ARG, "gprx_ctx_get_stats: NULL ctx");
    std::lock_guard<std::mutex> lk(ctx->mu);
    int k = 0;
    for (int c = 0; c < KC_COUNT; c++) {
        const Prof::Acc& a = ctx->prof.acc[c];
        if (a.launches == 0) continue;
        if (out && k < max) {
            std::memset(&out[k], 0, sizeof(gprx_kstat));
            std::strncpy(out[k].name, kclass_name(c), sizeof(out[k].name) - 1);
            out[k].launches = a.launches;
            out[k].ms = a.ms;
            out[k].flops = a.flops;
            out[k].bytes = a.bytes;
        }
        k++;
    }
    if (count) *count = k;
    return GPRX_OK;
    API_END(ctx)
}


gprx_status gprx_dev_bench(gprx_ctx* ctx, gprx_dtype dtype, int32_t what, int64_t M, int64_t N, int64_t K,
                           int32_t iters, double* ms) {
    API_BEGIN
    GPRX_REQUIRE(ctx && ms && iters > 0, GPRX_ERR_ARG, "gprx_dev_bench: bad argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    GPRX_HIP(hipSetDevice(ctx->device));
    gprx_status st = gprx_dev_bench_impl(dtype, what, M, N, K, iters, ms, &ctx->ex);
    if (st != GPRX_OK) return fail(ctx, st, "gprx_dev_bench failed");
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_dev_build_matrix(gprx_ctx* ctx, gprx_dtype dt, const gprx_kernel_desc* k, const void* X, int64_t n,
                                  int32_t d, double sigma, int32_t path, void* K) {
    API_BEGIN
    GPRX_REQUIRE(ctx && k && X && K, GPRX_ERR_ARG, "gprx_dev_build_matrix: NULL argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ProfBind pb_(ctx);
    GPRX_HIP(hipSetDevice(ctx->device));
    return dt == GPRX_F64 ? dev_build_impl<double>(ctx, k, X, n, d, sigma, path, K)
                          : dev_build_impl<float>(ctx, k, X, n, d, sigma, path, K);
    API_END(ctx)
}

gprx_status gprx_dev_build_time(gprx_ctx* ctx, gprx_dtype dt, const gprx_kernel_desc* k, const void* X, int64_t n,
                                int32_t d, double sigma, int32_t path, int32_t iters, double* ms) {
    API_BEGIN
    GPRX_REQUIRE(ctx && k && X && ms && iters > 0, GPRX_ERR_ARG, "gprx_dev_build_time: bad argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ProfBind pb_(ctx);
    GPRX_HIP(hipSetDevice(ctx->device));
    return dt == GPRX_F64 ? dev_build_impl<double>(ctx, k, X, n, d, sigma, path, nullptr, iters, ms)
                          : dev_build_impl<float>(ctx, k, X, n, d, sigma, path, nullptr, iters, ms);
    API_END(ctx)
}

gprx_status gprx_dev_dist_info(gprx_model* M, int64_t* out, int32_t nout) {
    API_BEGIN
    GPRX_REQUIRE(M && out, GPRX_ERR_ARG, "gprx_dev_dist_info: NULL argument");
    GPRX_REQUIRE(M->dist_fitted || M->dist_stats.bytes_rank > 0, GPRX_ERR_STATE,
                 "gprx_dev_dist_info: no distributed fit on this model");
    const DistFitOut& o = M->dist_stats;
    const int64_t v[15] = {o.bytes_rank, o.bytes_storage, o.gb, o.ww, o.chunk_w, o.P, (int64_t)o.est_us,
                           M->ctx->world, M->dist_dense ? 1 : 0,
                           M->dist_engine ? dist_pvar_chunks(M->dist_engine) : 0,
                           M->dist_engine ? dist_pvar_bytes(M->dist_engine) : 0,
                           o.push_linv, o.push_tiles, o.push_bytes, o.push_rank};
    for (int i = 0; i < std::min<int32_t>(nout, 15); i++) out[i] = v[i];
    return GPRX_OK;
    API_END(M ? M->ctx : nullptr)
}

gprx_status gprx_dev_ctx_info(gprx_ctx* ctx, int64_t* out, int32_t nout) {
    API_BEGIN
    GPRX_REQUIRE(ctx && out, GPRX_ERR_ARG, "gprx_dev_ctx_info: NULL argument");
    int count = -1, urank = -1;
    if (ctx->comm) {
        if (ncclCommCount(ctx->comm, &count) != ncclSuccess) count = -1;
        if (ncclCommUserRank(ctx->comm, &urank) != ncclSuccess) urank = -1;
    }
    int dom = -1, bus = -1, dev = -1;
    (void)hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, ctx->device);
    (void)hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, ctx->device);
    (void)hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, ctx->device);
    const int64_t transport = ctx->virt ? 3 : (ctx->comm ? 1 : (ctx->peer ? 2 : 0));
    const int64_t v[10] = {ctx->rank, ctx->world, ctx->device, transport, count, urank, dom, bus, dev, ctx->cu_slot};
    for (int i = 0; i < std::min<int32_t>(nout, 10); i++) out[i] = v[i];
    return GPRX_OK;
    API_END(ctx)
}

gprx_status gprx_dist_unique_id(void* out) {
    API_BEGIN
    GPRX_REQUIRE(out, GPRX_ERR_ARG, "gprx_dist_unique_id: out is NULL");
    static_assert(sizeof(ncclUniqueId) == GPRX_UNIQUE_ID_BYTES, "unique id size");
    ncclUniqueId id;
    const ncclResult_t r = ncclGetUniqueId(&id);
    if (r != ncclSuccess) throw Error{GPRX_ERR_RCCL, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r)};
    std::memcpy(out, &id, sizeof(id));
    return GPRX_OK;
    API_END(nullptr)
}

gprx_status gprx_ctx_create_virtual(int device, int world, gprx_ctx** out) {
    API_BEGIN
    GPRX_REQUIRE(out, GPRX_ERR_ARG, "gprx_ctx_create_virtual: NULL argument");
    GPRX_REQUIRE(world >= 1 && world <= 8, GPRX_ERR_ARG, "gprx_ctx_create_virtual: world must be 1..8");
    gprx_ctx* ctx = ctx_new(device);
    ctx->virt = true;
    ctx->world = world;
    *out = ctx;
    return GPRX_OK;
    API_END(nullptr)
}

gprx_status gprx_ctx_create_dist(int device, int rank, int world, const void* unique_id, gprx_ctx** out) {
    API_BEGIN
    GPRX_REQUIRE(out && unique_id, GPRX_ERR_ARG, "gprx_ctx_create_dist: NULL argument");
    GPRX_REQUIRE(world >= 1 && rank >= 0 && rank < world, GPRX_ERR_ARG, "gprx_ctx_create_dist: bad rank/world");
    gprx_ctx* ctx = ctx_new(device);
    ctx->rank = rank;
    ctx->world = world;
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    // GPRX_RCCL_FAIL=1 (testing): fail as an initialisation that never completes would, so the
    // caller's fallback (a peer context over its own all-gather) can be exercised
    if (const char* e = std::getenv("GPRX_RCCL_FAIL"); e && std::atoi(e) != 0) {
        gprx_ctx_destroy(ctx);
        throw Error{GPRX_ERR_RCCL, "ncclCommInitRankConfig: forced failure (GPRX_RCCL_FAIL)"};
    }
    // nonblocking initialisation, polled with a deadline (GPRX_RCCL_INIT_TIMEOUT_S, default
    // 120 s): a rank that cannot reach its peers returns GPRX_ERR_RCCL instead of blocking
    // the process for ever inside ncclCommInitRank
    double tmo = 120.0;
    if (const char* e = std::getenv("GPRX_RCCL_INIT_TIMEOUT_S"); e && std::atof(e) > 0) tmo = std::atof(e);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t comm = nullptr;
    ncclResult_t r = ncclCommInitRankConfig(&comm, world, id, rank, &cfg);
    try {
        if (r != ncclSuccess && r != ncclInProgress)
            throw Error{GPRX_ERR_RCCL, std::string("ncclCommInitRankConfig: ") + ncclGetErrorString(r)};
        rccl_settle(comm, r, "ncclCommInitRankConfig", tmo);
    } catch (...) {
        if (comm) (void)ncclCommAbort(comm);
        gprx_ctx_destroy(ctx);
        throw;
    }
    ctx->comm = comm;
    ctx->hc = make_rccl_coll(ctx->comm, world, device);
    *out = ctx;
    return GPRX_OK;
    API_END(nullptr)
}

gprx_status gprx_ctx_create_peer(int device, int rank, int world, gprx_allgather_fn fn, void* user, gprx_ctx** out) {
    API_BEGIN
    GPRX_REQUIRE(out && fn, GPRX_ERR_ARG, "gprx_ctx_create_peer: NULL argument");
    GPRX_REQUIRE(world >= 1 && world <= 32 && rank >= 0 && rank < world, GPRX_ERR_ARG,
                 "gprx_ctx_create_peer: bad rank/world");
    gprx_ctx* ctx = ctx_new(device);
    ctx->rank = rank;
    ctx->world = world;
    ctx->peer = true;
    ctx->hc = make_callback_coll(fn, user, world);
    if (const char* e = std::getenv("GPRX_DIST_SHARED_GPU"); e && std::atoi(e) != 0) {
        ctx->cu_slot = rank;
        ctx->cu_slots = world;
    }
    *out = ctx;
    return GPRX_OK;
    API_END(nullptr)
}

gprx_status gprx_sparse_fit(gprx_ctx* ctx, gprx_dtype dtype, const gprx_kernel_desc* kernel, const void* X,
                            const void* Y, int64_t n, int32_t d, int32_t m, const void* Xm, int64_t M, double sigma,
                            double jitter, void* Kinv, void* RV, void* RM) {
    API_BEGIN
    GPRX_REQUIRE(ctx && kernel && Xm && (X || n == 0) && (Y || n == 0), GPRX_ERR_ARG, "gprx_sparse_fit: NULL argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ProfBind pb_(ctx);  // after the lock: resolved (streams drained) before it is released
    return dtype == GPRX_F64 ? sparse_fit_impl<double>(ctx, kernel, X, Y, n, d, m, Xm, M, sigma, jitter, Kinv, RV, RM)
                             : sparse_fit_impl<float>(ctx, kernel, X, Y, n, d, m, Xm, M, sigma, jitter, Kinv, RV, RM);
    API_END(ctx)
}

gprx_status gprx_sparse_lml(gprx_ctx* ctx, gprx_dtype dtype, const gprx_kernel_desc* kernel, const void* X,
                            const void* Y, int64_t n, int32_t d, int32_t m, const void* Xm, int64_t M, double sigma,
                            double jitter, uint32_t flags, double* value, double* grad, int32_t* nparams,
                            double* logdet) {
    API_BEGIN
    GPRX_REQUIRE(M > 0, GPRX_ERR_DIM,
                 "SparseLikelihood::GetValueAndParameterDerivative: there are no inducing samples specified");
    GPRX_REQUIRE(ctx && kernel && Xm && X && Y, GPRX_ERR_ARG, "gprx_sparse_lml: NULL argument");
    std::lock_guard<std::mutex> lk(ctx->mu);
    ProfBind pb_(ctx);
    return dtype == GPRX_F64 ? sparse_lml_impl<double>(ctx, kernel, X, Y, n, d, m, Xm, M, sigma, jitter, flags, value,
                                                       grad, nparams, logdet)
                             : sparse_lml_impl<float>(ctx, kernel, X, Y, n, d, m, Xm, M, sigma, jitter, flags, value,
                                                      grad, nparams, logdet);
    API_END(ctx)
}

}  // extern "C"
