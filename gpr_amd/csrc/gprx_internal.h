// gprx_internal.h — shared declarations of libgprx (MI355X / gfx950).
//
// Kernel representation on the device
// -----------------------------------
// The reference evaluates a covariance pair through a virtual call per node
// (include/Kernel.h:52, Sum :165, Product :314).  On the GPU the tree is canonicalised on
// the host into a SUM OF PRODUCTS OF LEAVES: k = sum_t prod_{l in t} leaf_l.  Every leaf
// depends on the pair only through a few streaming statistics that are accumulated over
// the d input dimensions in one pass:
//     r2        = sum_k (x_k - y_k)^2                 (Gaussian, GaussianExp, RQ, White)
//     S_p       = sum_k sin^2(b_p (x_k - y_k))         (Periodic leaf p)
//     F_p       = sum_k 2 (x_k-y_k) sin cos(b_p(...))  (Periodic d/db, gradient only)
// sin(b(x-y)) is formed from per-sample sin/cos tables (sin(bx)cos(by) - cos(bx)sin(by)),
// so the pair loop is pure FMA work.  Leaf and term loops have compile-time trip counts
// (MAX_LEAF / MAX_TERM), so all per-pair state lives in registers.
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <cstdint>
#include <cstdio>
#include <string>
#include <vector>

#include "../../include/gprx.h"

namespace gprx {

constexpr int MAX_LEAF = 8;
constexpr int MAX_TERM = 16;
constexpr int MAX_PER = 2;  // periodic leaves with distinct tables

enum LeafType { L_GAUSS = 1, L_GAUSS_EXP = 2, L_WHITE = 3, L_RQ = 4, L_PERIODIC = 5 };

template <typename T>
struct KLeaf {
    int type;
    int pslot;   // periodic table slot
    T c0, c1, c2;  // value constants (see leaf_value)
    T p[3];        // raw reference parameters (gradient formulas)
    // exp leaves c0 exp(c1 x) with the scale folded into the exponent (f64 predict epilogue,
    // fexp_fold): y = f1 x + f0 = (c1 x + ln c0) 64 / ln 2; fold = 0 when c0 <= 0 or not an exp leaf
    T f1, f0;
    int fold;
};

template <typename T>
struct KCanon {
    int nleaf;
    int nterm;
    int nper;
    int need_r2;
    int nparams;
    int sum_leaves;  // every term is a single leaf: k = sum_l leaf_l
    unsigned term_mask[MAX_TERM];
    int param_base[MAX_LEAF];
    KLeaf<T> leaf[MAX_LEAF];
    T b[MAX_PER];
};

// Build the canonical form from the ABI post-order program.  Returns "" on success or an
// error message.  Parameters are narrowed to T first (the reference stores them in T).
template <typename T>
std::string canonicalize(const gprx_kernel_desc& desc, KCanon<T>& out);

// ---------------------------------------------------------------------------------
// Leaf evaluation (device + host).  Formulas follow include/Kernel.h:
//   Gaussian       s^2 exp(-0.5 r2 / sigma^2)                      :465-468
//   GaussianExp    exp(scale)^2 exp(-0.5 r2 / exp(sigma)^2)         :580-585
//   White          r2 == 0 ? s^2 : 0 (exact equality)               :695-702
//   RQ             s^2 (1 + 0.5 r2 / (sigma^2 alpha))^(-alpha)      :794-797
//   Periodic       s^2 exp(-0.5 S / sigma^2)                        :912-920
// ---------------------------------------------------------------------------------
template <typename T>
__host__ __device__ inline T leaf_value(const KLeaf<T>& L, T r2, T s0, T s1) {
    switch (L.type) {
        case L_GAUSS:
        case L_GAUSS_EXP:
            return L.c0 * exp(L.c1 * r2);
        case L_WHITE:
            return (r2 == T(0)) ? L.c0 : T(0);
        case L_RQ:  // alpha = 1: std::pow(b, -1) = 1 / b
            return (L.c2 == T(1)) ? L.c0 / (T(1) + L.c1 * r2) : L.c0 * exp(-L.c2 * log1p(L.c1 * r2));
        case L_PERIODIC:
            return L.c0 * exp(L.c1 * (L.pslot == 0 ? s0 : s1));
    }
    return T(0);
}

// d leaf / d params (up to 3), the reference's GetDerivative formulas
// (Gaussian :471-479, GaussianExp :588-598, White :704-713, RQ :799-808, Periodic :922-948).
template <typename T>
__host__ __device__ inline void leaf_grad(const KLeaf<T>& L, T r2, T s0, T s1, T f0, T f1, T* g) {
    switch (L.type) {
        case L_GAUSS: {  // p = (sigma, scale)
            T sig = L.p[0], sc = L.p[1];
            T f = exp(L.c1 * r2);
            g[0] = sc * sc * r2 / (sig * sig * sig) * f;
            g[1] = T(2) * sc * f;
            g[2] = 0;
            return;
        }
        case L_GAUSS_EXP: {  // p = (sigma, scale) in log space
            T sig = L.p[0], sc = L.p[1];
            T e2 = exp(T(-2) * sig);
            g[0] = r2 * exp(T(2) * sc - T(2) * sig - T(0.5) * r2 * e2);
            g[1] = T(2) * exp(T(2) * sc - T(0.5) * r2 * e2);
            g[2] = 0;
            return;
        }
        case L_WHITE: {
            g[0] = (r2 == T(0)) ? T(2) * L.p[0] : T(0);
            g[1] = 0;
            g[2] = 0;
            return;
        }
        case L_RQ: {  // p = (scale, sigma, alpha)
            T sc = L.p[0], sig = L.p[1], al = L.p[2];
            T f = T(0.5) * r2 / (sig * sig * al) + T(1);
            T lf = log(f);
            T pw = exp(-al * lf);
            g[0] = T(2) * sc * pw;
            g[1] = sc * sc * r2 * pw / f / (sig * sig * sig);
            g[2] = sc * sc * (r2 / (T(2) * sig * sig * f * al) - lf) * pw;
            return;
        }
        case L_PERIODIC: {  // p = (scale, b, sigma)
            T sc = L.p[0], sig = L.p[2];
            T s = (L.pslot == 0) ? s0 : s1, fb = (L.pslot == 0) ? f0 : f1;
            T e = exp(L.c1 * s);
            g[0] = T(2) * sc * e;
            g[1] = T(-0.5) * sc * sc * e * fb / (sig * sig);
            g[2] = sc * sc * e * s / (sig * sig * sig);
            return;
        }
    }
    g[0] = g[1] = g[2] = 0;
}

// Value of the whole kernel from the pair statistics.
template <typename T>
__host__ __device__ inline T kernel_value(const KCanon<T>& K, T r2, T s0, T s1) {
    T lv[MAX_LEAF];
#pragma unroll
    for (int l = 0; l < MAX_LEAF; l++) lv[l] = (l < K.nleaf) ? leaf_value(K.leaf[l], r2, s0, s1) : T(0);
    if (K.sum_leaves) {
        T v = lv[0];
#pragma unroll
        for (int l = 1; l < MAX_LEAF; l++)
            if (l < K.nleaf) v += lv[l];
        return v;
    }
    T v = 0;
#pragma unroll
    for (int t = 0; t < MAX_TERM; t++) {
        if (t < K.nterm) {
            unsigned m = K.term_mask[t];
            T p = 1;
#pragma unroll
            for (int l = 0; l < MAX_LEAF; l++)
                if (m & (1u << l)) p *= lv[l];
            v += p;
        }
    }
    return v;
}

// exp for f64 in the pair-statistics epilogues (k_pairs.h leaf_into): x = (64 k + j) ln2/64 + r,
// |r| <= ln2/128, exp(x) = 2^k 2^{j/64} (1 + expm1(r)) with a 64-entry table of 2^{j/64}
// (correctly rounded) and a degree-5 polynomial for expm1 (truncation r^6/720 < 4e-17): 11 f64
// operations against the 17 of the library's degree-11 sequence -- the epilogue's f64 VALU work
// is serial with the tile's f64 MFMAs.  Error < 1 ulp + the final rounding;
// x < -745 gives 0 (the library's underflow), NaN stays NaN.
__device__ __constant__ const double kExp2Tab64[64] = {
    1.0, 1.0108892860517005, 1.0218971486541166, 1.0330248790212284,
    1.0442737824274138, 1.0556451783605572, 1.0671404006768237, 1.0787607977571199,
    1.0905077326652577, 1.102382583307841, 1.1143867425958924, 1.1265216186082418,
    1.1387886347566916, 1.1511892299529827, 1.1637248587775775, 1.1763969916502812,
    1.189207115002721, 1.202156731452703, 1.215247359980469, 1.22848053610687,
    1.241857812073484, 1.255380757024691, 1.2690509571917332, 1.2828700160787783,
    1.2968395546510096, 1.3109612115247644, 1.3252366431597413, 1.339667524053303,
    1.3542555469368927, 1.3690024229745905, 1.383909881963832, 1.3989796725383112,
    1.4142135623730951, 1.42961333839197, 1.4451808069770467, 1.460917794180647,
    1.4768261459394993, 1.4929077282912648, 1.5091644275934228, 1.5255981507445384,
    1.5422108254079407, 1.559004400237837, 1.5759808451078865, 1.593142151342267,
    1.6104903319492543, 1.6280274218573478, 1.645755478153965, 1.6636765803267364,
    1.681792830507429, 1.7001063537185235, 1.718619298122478, 1.7373338352737062,
    1.7562521603732995, 1.7753764925265212, 1.7947090750031072, 1.8142521755003989,
    1.8340080864093424, 1.8539791250833855, 1.8741676341103, 1.8945759815869656,
    1.9152065613971474, 1.9360617934922943, 1.9571441241754002, 1.978456026387951,
};
__device__ __forceinline__ double fexp(double x) {
    const double kd = __builtin_rint(x * 92.33248261689366);  // 64 / ln2
    double r = fma(-kd, 0.01083042469326756, x);             // ln2/64, high part (exact product)
    r = fma(-kd, 2.9815858269852933e-12, r);                   // low part
    const int n = (int)kd;
    const double t = kExp2Tab64[n & 63];
    const double p = fma(r * r, fma(r, fma(r, fma(r, 1.0 / 120.0, 1.0 / 24.0), 1.0 / 6.0), 0.5), r);
    const double v = __builtin_ldexp(fma(t, p, t), n >> 6);
    return x < -745.5 ? 0.0 : v;
}
__device__ __forceinline__ float fexp(float x) { return expf(x); }
// c0 exp(c1 x) for an exp leaf from y = f1 x + f0 = (c1 x + ln c0) 64 / ln2 (KLeaf::f1, f0; one
// FMA in place of fexp's two multiplications before the reduction and the scale's multiplication
// after it).  kd = rint(y), y - kd is exact (Sterbenz), r = (y - kd) ln2 / 64, |r| <= ln2/128,
// then fexp's table and polynomial.  The rounding of y (|y| ulp / 2, ln2/64 of that in the
// argument) matches the rounding of c1 x in the unfolded form within a factor of 2: ~1e-14
// relative on the C3 tree's Gaussian leaf (x ~ 110).  y below -745.5 * 64/ln2 gives 0 as fexp.
__device__ __forceinline__ double fexp_fold(double y) {
    const double kd = __builtin_rint(y);
    const double r = (y - kd) * (0.6931471805599453094 / 64.0);
    const int n = (int)kd;
    const double t = kExp2Tab64[n & 63];
    const double p = fma(r * r, fma(r, fma(r, fma(r, 1.0 / 120.0, 1.0 / 24.0), 1.0 / 6.0), 0.5), r);
    const double v = __builtin_ldexp(fma(t, p, t), n >> 6);
    return y < -68834.5 ? 0.0 : v;
}

// sincos for both scalar types
__device__ inline void gsincos(double x, double* s, double* c) { sincos(x, s, c); }
__device__ inline void gsincos(float x, float* s, float* c) { sincosf(x, s, c); }

// ---------------------------------------------------------------------------------
// Error helpers (host)
// ---------------------------------------------------------------------------------
struct Error {
    gprx_status st;
    std::string msg;
};

#define GPRX_HIP(call)                                                                             \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess)                                                                      \
            throw ::gprx::Error{e_ == hipErrorOutOfMemory ? GPRX_ERR_OOM : GPRX_ERR_HIP,           \
                                std::string(#call) + ": " + hipGetErrorString(e_)};                \
    } while (0)

#define GPRX_REQUIRE(cond, status, msg)                                                            \
    do {                                                                                           \
        if (!(cond)) throw ::gprx::Error{status, msg};                                             \
    } while (0)


// ---------------------------------------------------------------------------------
// Opt-in per-kernel device timing (gprx_ctx_set_stats): HIP events around every launch
// of the classes below, on the stream the kernel is launched on.
// ---------------------------------------------------------------------------------
enum KClass { KC_BUILD = 0, KC_DIAG, KC_TRSM, KC_UPDATE, KC_BACKSOLVE, KC_PREDICT, KC_LML_GRAD, KC_INVERSE, KC_OTHER,
              KC_TILES, KC_POSTERIOR, KC_COUNT };
struct Prof {
    bool on = false;
    struct Rec {
        int cls;
        hipEvent_t a, b;
        double flops, bytes;
    };
    struct Acc {
        int64_t launches = 0;
        double ms = 0, flops = 0, bytes = 0;
    };
    std::vector<hipEvent_t> pool;
    size_t used = 0;
    std::vector<Rec> recs;
    Acc acc[KC_COUNT];
    hipEvent_t next() {
        if (used == pool.size()) {
            hipEvent_t e;
            (void)hipEventCreate(&e);
            pool.push_back(e);
        }
        return pool[used++];
    }
    void resolve() {  // caller has synchronised the streams
        for (auto& r : recs) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, r.a, r.b);
            acc[r.cls].launches++;
            acc[r.cls].ms += ms;
            acc[r.cls].flops += r.flops;
            acc[r.cls].bytes += r.bytes;
        }
        recs.clear();
        used = 0;
    }
    void reset() {
        recs.clear();
        used = 0;
        for (auto& a : acc) a = Acc();
    }
    ~Prof() {
        for (auto e : pool) (void)hipEventDestroy(e);
    }
};
extern thread_local Prof* g_prof;

struct ProfScope {
    Prof* p;
    int cls;
    hipStream_t s;
    double flops, bytes;
    hipEvent_t a = nullptr;
    ProfScope(int c, hipStream_t st, double f = 0, double b = 0) : p(g_prof), cls(c), s(st), flops(f), bytes(b) {
        if (p && p->on) {
            a = p->next();
            (void)hipEventRecord(a, s);
        }
    }
    ~ProfScope() {
        if (p && p->on) {
            hipEvent_t b = p->next();
            (void)hipEventRecord(b, s);
            p->recs.push_back(Prof::Rec{cls, a, b, flops, bytes});
        }
    }
};

// ---------------------------------------------------------------------------------
// Launchers implemented in the .hip files.  All device matrices are column-major.
// ---------------------------------------------------------------------------------
constexpr int BT = 64;     // build tile edge
constexpr int DB = 128;    // Cholesky diagonal block edge (also the padding granule)
constexpr int GT = 128;    // GEMM output tile edge

// per-sample sin/cos tables for the periodic leaves: tab[(slot*2 + {0:sin,1:cos})][i*d + k]
template <typename T>
void launch_sincos_tables(const KCanon<T>& K, const T* X, int64_t n, int d, T* tab, hipStream_t s);

// Covariance tiles.  lower=true: square lower-triangle build of K(X,X) into A (column-major,
// ld), rows/cols >= n padded with the identity, sigma2 added to the diagonal (for i < n).
// lower=false: rectangular cross matrix K(Xa, Xb) (na x nb) into A.
template <typename T>
void launch_kbuild(const KCanon<T>& K, const T* Xa, const T* tabA, int64_t na, const T* Xb, const T* tabB,
                   int64_t nb, int d, T* A, int64_t ld, int64_t npad, bool lower, T sigma2, int* flag,
                   hipStream_t s);

// Kernels with no device form, evaluated by the caller (k_hostk.hip)
template <typename T>
void launch_kext_build(const T* Kx, int64_t n, T* A, int64_t ld, int64_t np, T sigma2, int* flag, hipStream_t s);
template <typename T>
void launch_kx_predict(const T* Kx, const T* Xq, const T* X, int64_t q, int64_t n, int d, const T* alpha, int m,
                       T* mean, T* D, hipStream_t s);
template <typename T>
void launch_dk_grad(const T* dK, int P, int64_t n, const T* alpha, const T* C, int64_t ldc, double* out, hipStream_t s);

// MFMA pair statistics (k_pairs.hip): kernels without White leaves and with at most one
// periodic frequency build their covariance / predict their mean from per-sample feature
// matrices (np rows x pairs_feature_cols columns, column-major) and 128x128 MFMA tiles.
template <typename T>
bool pairs_mma_supported(const KCanon<T>& K, int m);
template <typename T>
int64_t pairs_feature_cols(const KCanon<T>& K, int d);
// flag (optional): set when an input sample has a non-finite coordinate (the fit's check)
template <typename T>
void launch_pair_features(const KCanon<T>& K, const T* X, int64_t n, int d, const T* center, bool right, T* F,
                          int64_t np, hipStream_t s, int* flag = nullptr);
// Kd: a device copy of K (the kernels read the tree from memory)
template <typename T>
void launch_kbuild_mma(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, const T* FV, int64_t nf, int d, T* A,
                       int64_t ld, int64_t n, T sigma2, int* flag, hipStream_t s);
// Cross matrix K(Xa, Xb) (na x nb, column-major, ld) from the features FU of Xa (nfu rows)
// and FV of Xb (nfv rows, right = true), both centred on the same point; only valid entries
// are stored.
template <typename T>
void launch_kcross_mma(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, int64_t nfu, int64_t na, const T* FV,
                       int64_t nfv, int64_t nb, int d, T* A, int64_t ld, int* flag, hipStream_t s,
                       const T* Y = nullptr, T* kyp = nullptr);
// With Y (one label column of the nb samples of Xb): kyp[c * nfu + i] = the column tile c's
// part of sum_j K(a_i, b_j) Y[j]; launch_ky_reduce adds alpha times their ordered sum into
// row row0 of S (column i at S[row0 + i * lds]).
template <typename T>
void launch_ky_reduce(const T* kyp, int64_t nfu, int nct, int64_t na, T alpha, T* S, int64_t lds, int64_t row0,
                      hipStream_t s);
template <typename T>
void launch_predict_mma(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, int64_t nfu, const T* FV, int64_t nfv,
                        int d, const T* alpha, int64_t n, int m, int64_t q, T* mean, hipStream_t s);

// Stacked derivative matrices (tests): D[p] (n x n, column-major, ld = n).
template <typename T>
void launch_deriv_matrix(const KCanon<T>& K, const T* X, const T* tab, int64_t n, int d, T* D, hipStream_t s);

// Augmented label rows: A[np + r, j] = Y[j, r] (j < n, r < m), zero elsewhere in the block.
template <typename T>
void launch_aug_rows(const T* Y, int64_t n, int m, T* A, int64_t ld, int64_t np, int64_t mp, hipStream_t s);
// General form: A[row0 + r, j] = Y[j, r] for j < n, r < m; zero for the other of the mp rows
// and for n <= j < ncols.
template <typename T>
void launch_diag_fix(T* A, int64_t ld, int64_t c0, int64_t w, int64_t n, T sigma2, hipStream_t s);
// a fit's status words (k_build.hip): info = INT_MAX, flag = 0; and back into mapped pinned
// host memory (out[0] flag, out[1] info as ints, out[2..3] = red[0..1])
void launch_fit_status_init(int* info, int* flag, hipStream_t s);
void launch_fit_status_gather(const int* flag, const int* info, const double* red, double* out_mapped, hipStream_t s);
template <typename T>
void launch_label_rows(const T* Y, int64_t n, int m, T* A, int64_t ld, int64_t row0, int64_t ncols, int64_t mp,
                       hipStream_t s);

// Blocked right-looking Cholesky of the leading np x np block of A (ld rows; rows np..ld
// are extra rows solved along: they end up holding (L^{-1} B)^T).  Linv receives the
// inverses of the np/DB diagonal blocks (DB x DB each, column-major).  info: device int,
// first failing column (1-based) via atomicMin semantics (initialised to INT_MAX).
struct PtState;             // tile-dataflow potrf: cached schedules + counters (k_ptiles.hip)
void pt_state_free(PtState* p);
struct Exec {
    hipStream_t s0 = nullptr;  // main stream (panel chain)
    hipStream_t s1 = nullptr;  // look-ahead stream (bulk trailing updates); may be null
    hipStream_t s2 = nullptr;  // second look-ahead stream (next panel's later columns); may be null
    std::vector<hipEvent_t> ev;
    PtState* pt = nullptr;
    int* scratch = nullptr;  // device ints for in-launch counters/flags (grown on demand)
    size_t scratch_n = 0;
    int* scratch_ints(size_t n);
    hipEvent_t event(size_t i);
    ~Exec();
};
int outer_block();
template <typename T>
void potrf_blocked(T* A, int64_t ld, int64_t np, int64_t nrows, T* Linv, int* info, Exec& ex);
// The covariance build fused into the tile factorisation: each lower tile of the leading
// np x np block is built from the pair-statistics features (k_pairs.h) by a BUILD task of
// the same persistent launch, ahead of its first consumer, instead of by a separate kernel.
// mode: 1 = periodic + r2 statistics, 2 = r2 only, 3 = periodic only.  Rows >= np (the
// label rows) must already be in A.  A non-finite value sets *flag.
template <typename T>
struct TileBuild {
    const KCanon<T>* Kd;
    const T* FU;
    const T* FV;
    int64_t nf;
    int Kr, Kp;
    T hd, sigma2;
    int64_t n;
    int* flag;
    int mode;
};
// Per diagonal block k, TP_STRIDE state words of the split diagonal step (k_ptiles.hip): [0..7]
// TPART(k, p)'s phase, [TP_DPAN] DIAGX(k)'s published panels (the progressive TPART(k + 1, .)
// follow it)
constexpr int TP_STRIDE = 16, TP_DPAN = 8;  // (up to eight parts: k_ptiles.hip tp_parts)

// Distributed tile factorisation (k_ptiles.hip, potrf_tiles_kernel<T, true>; gprx_dist.cpp):
// this rank's view of a factorisation whose row blocks are dealt over g ranks in groups of gb
// (row block i on rank (i / gb) mod g).  Device copy, read per task.
//
// Storage: a rank keeps only the LOWER part of its own row blocks, packed -- row block i's
// tiles (i, j), j = 0..i (the label row block nc: j < nc), contiguous 128 x 128 column-major
// tiles (ld DB) from element roff[loc[i]]; the identity row blocks of the inverse (LML mode,
// E_a = nc + 1 + a) keep their tiles (E_a, b), b = a..nc-1, then the C tiles (E_a, E_c), c <= a.
//
// Exchange: no host in the loop.  Every rank has a MAILBOX (one device allocation, the same
// byte offsets on every rank, mapped into every peer: the same process for virtual ranks,
// hipIpcOpenMemHandle across processes) and a receive WINDOW (pieces below 2 GiB, mapped the
// same way).  A producing task pushes its final tile straight into the window slot of each rank
// that consumes the row -- slot (b mod ww, row j) -- and raises that rank's per-tile flag; a diagonal task pushes Linv_k into every rank's Linv array.  Flags hold
// the fit's epoch (no reset between fits).  A window slot is reused for panel b + ww only after
// every consumer released panel b: a rank counts its completed window-reading updates per panel
// (ucnt) and, at the last one, stores its release flag into every peer's mailbox.
template <typename T>
struct PtDist {
    int g, r, nc, nr, ww;      // ranks, this rank, column blocks, row blocks, window panels
    int nci;                   // column blocks of the counter array (nc, or 2 nc with C tiles)
    unsigned ep;               // this fit's epoch (flag value)
    const int* loc;            // [nr] local index of row block i, -1 if owned elsewhere
    const int64_t* roff;       // [nloc] element offset of local row block li in the storage
    const int* own;            // [nr] owner rank of row block i
    const uint64_t* tptr;      // [nr * nc] window address (this rank) of remote tile (j, b)
    const unsigned char* cons; // [g * nr] rank q consumes the tiles of row block j
    const int* need;           // [g * nc] window-reading update chunks of rank q covering panel p
    int* ucnt;                 // [nc] this rank's completed window-reading chunks per panel (local)
    const uint64_t* mb;        // [g] mailbox base of every rank (as mapped in this process)
    // the receive windows: slot (b mod ww, row j) is tile t = (b mod ww) nr + j of rank q's window,
    // in its piece t / tpp (allocations below 2 GiB: IPC-mappable) at tile t mod tpp
    const uint64_t* wpc;       // [g * npc] window piece bases of every rank (as mapped here)
    int64_t tpp;               // tiles per window piece
    int npc;                   // window pieces per rank
    // mailbox byte offsets (the same on every rank)
    int64_t o_linv, o_z, o_flags;
    int64_t o_tags;            // GPRX_DIST_CHECK: per window slot (panel, row) the tag of its occupant
    int check;                 // GPRX_DIST_CHECK: verify every window read against the slot's tag
    int wt;                    // pushes cross devices: written-through (sc0 sc1) stores, no L2 write-back fence
    int acq_agent;             // ranks of one device: agent-scope acquire before reading pushed data
    int* check_err;            // [2] window reads of a stale slot / of a slot overwritten during the read
    // flag words in the mailbox (unsigned, from o_flags): tile (j, b) received at
    // [F_TILE + j * nc + b], Linv_k at [F_LINV(nr, nc) + k], panel p released by rank q at
    // [F_REL(nr, nc) + q * nc + p]
};
constexpr int64_t dist_f_tile() { return 0; }
constexpr int64_t dist_f_linv(int nr, int nc) { return (int64_t)nr * nc; }
constexpr int64_t dist_f_rel(int nr, int nc) { return (int64_t)nr * nc + nc; }

// One rank's launch of the distributed tile factorisation (k_ptiles.hip).  ctr: C_NCTL +
// nr + nr * nci ints, zeroed (ver = -1 for the tiles the launch builds; the identity rows'
// counters start at their first column) by the caller.
template <typename T>
struct DistLaunch {
    T* A;              // packed storage of this rank's row blocks (ld DB)
    T* Linv;           // nc diagonal-block inverses (this rank's mailbox)
    int* info;
    const int4* list;
    int ntasks, nc, nr, nci;
    int* ctr;
    const TileBuild<T>* tb_dev;
    const PtDist<T>* dist_dev;
    long long tlimit;  // wall-clock ticks (100 MHz) a single wait may take
    int P;             // workgroups (one per CU)
    hipStream_t s;
    int* dbg;          // optional: per-workgroup {ticket, phase, i, j} in coherent host memory
    long long* trace;  // optional: 4 * (ntasks + 2 nc) words, as GPRX_PT_TRACE (k_ptiles.hip)
    int split;         // the split diagonal step (f64): TPART tasks in the list
    T* pbuf;           // [4][DB x DB] the TPART products
    int* tflag;        // [nc][TP_STRIDE] split-step states (zeroed per fit with the counters)
};
// The simulated schedule of a distributed factorisation: per-rank ticket lists (in start
// order of one list-schedule simulation of all ranks, window flow control included), the
// window-reading chunks per (rank, panel), and the predicted makespan.  ni > 0: nc identity
// row blocks ride along (U = L^{-T}) plus the lower C = U U^T tiles (LML mode).
struct DistSched {
    std::vector<std::vector<int4>> lists;
    std::vector<int> need;            // [g * nc]
    std::vector<unsigned char> cons;  // [g * nr]: rank q reads row block j through its window
    double est_us = 0;
    int W = 0;              // update chunk width used
};
DistSched potrf_dist_schedule(int nc, int g, int gb, int ww, int P, bool build, bool inv, int ratio = 0, bool f64 = true,
                              int tail = 0);
bool potrf_split_for(bool f64, int P);  // the split diagonal step is on (this precision, P workgroups)
// GPRX_PT_DEBUG: the per-workgroup status words gprx_dev_pt_debug reads (k_ptiles.hip);
// n = 0 unregisters dbg (if registered)
void pt_debug_register(int* dbg, int n);
template <typename T>
void potrf_tiles_dist_launch(const DistLaunch<T>& L);

// LML gradient on the MFMA units (k_pairs.hip): trees it covers, the extra feature columns
// it needs per sample set, and the launch (partials of ntiles * 3 MAX_LEAF doubles, reduced
// in a fixed order into acc[3 l + q]).
template <typename T>
bool pairs_grad_supported(const KCanon<T>& K);
template <typename T>
int64_t pairs_grad_feature_cols(const KCanon<T>& K, int d);
template <typename T>
void launch_lml_grad_mma(const KCanon<T>& K, const KCanon<T>* Kd, const T* X, int64_t n, int d, const T* FU,
                         const T* FV, T* GU, T* GV, int64_t nf, const T* alpha, const T* C, int64_t ldc, double* part,
                         double* acc, hipStream_t s,
                         const uint64_t* ctab = nullptr);  // ctab: C tile (i, j) pointers of a sharded fit (gprx_dist.cpp)
// Rectangular form for the sparse likelihood (k_pairs.hip): acc[3 l + q] = sum over the
// na x nb pairs (xa_i, xb_j) of (a_i b_j - C_ij) d leaf_l / d p_q.
template <typename T>
void launch_lml_grad_mma_cross(const KCanon<T>& K, const KCanon<T>* Kd, const T* Xa, int64_t na, const T* Xb,
                               int64_t nb, const T* center, int d, const T* FU, int64_t nfu, const T* FV, int64_t nfv,
                               T* GU, T* GV, const T* a, const T* b, const T* C, int64_t ldc, double* part, double* acc,
                               hipStream_t s);
// VALU form of the same sum for every tree (k_lml.hip); acc is accumulated into (atomics).
template <typename T>
void launch_lml_grad_cross(const KCanon<T>& K, const T* Xa, const T* tabA, int64_t na, const T* Xb, const T* tabB,
                           int64_t nb, int d, const T* a, const T* b, const T* C, int64_t ldc, double* acc,
                           hipStream_t s);
// Sparse likelihood helpers (k_sparse.hip).
// out[i] = alpha (y[i] - sum_j A[i + j lda] u[j]) for i < n (rows of K(Xc, Xm) u)
template <typename T>
void launch_sparse_resid(const T* A, int64_t lda, int64_t n, int64_t M, const T* u, const T* y, T alpha, T* out,
                         hipStream_t s);
// out[0] = sum_i y[i]^2 (fixed order, double)
template <typename T>
void launch_sq_sum(const T* y, int64_t n, double* out, hipStream_t s);
// Z = X - Y elementwise (e entries)
template <typename T>
void launch_sub(const T* X, const T* Y, T* Z, int64_t e, hipStream_t s);
// The BUILD description of K(X, X) + sigma2 I from the features of launch_pair_features
// (k_pairs.hip; the same trees as launch_kbuild_mma).
template <typename T>
TileBuild<T> pairs_tile_build(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, const T* FV, int64_t nf, int d,
                              int64_t n, T sigma2, int* flag);
// Same contract, one persistent launch: 128x128 tile tasks scheduled on the device by
// dependency counters (k_ptiles.hip).  A timed-out dependency wait sets *info = -1.
// ni > 0: the last ni row blocks of the nrows are the identity, set up here, and leave as
// L^{-T} (upper triangular, ni = np / 128): the inverse factor riding along as extra rows,
// each identity block updated only from its own column block on.
// build_only: run the BUILD tasks alone (the covariance tiles, no factorisation; parity hook).
template <typename T>
void potrf_tiles(T* A, int64_t ld, int64_t np, int64_t nrows, T* Linv, int* info, Exec& ex,
                 const TileBuild<T>* build = nullptr, int ni = 0, bool build_only = false);
// C (lower) = A B^T where both operands vanish left of their row (LAUUM shape), k_potrf.hip
template <typename T>
void launch_gemm_nt_kskip(T* C, int64_t ldc, const T* A, int64_t lda, const T* B, int64_t ldb, int64_t M, int64_t N,
                          int64_t K, hipStream_t s);
// Factorisation used by the fit paths: potrf_tiles unless GPRX_POTRF=streams.
template <typename T>
void potrf_auto(T* A, int64_t ld, int64_t np, int64_t nrows, T* Linv, int* info, Exec& ex);
bool potrf_uses_tiles();
int64_t potrf_tiles_schedule_stats(int nc, int nr, int P, bool build, double* est_us, int ni = 0, int ratio = -1,
                                   int32_t* list_out = nullptr, int64_t list_max = 0, int pair = -1);
// Generic C = beta C + alpha A B^T on GT-multiples (column-major).  lower: only tiles
// with col-tile <= row-tile are computed, and inside diagonal tiles only row >= col.
template <typename T>
void launch_gemm_nt(T* C, int64_t ldc, const T* A, int64_t lda, const T* B, int64_t ldb, int64_t M, int64_t N,
                    int64_t K, T alpha, T beta, bool lower, hipStream_t s);
// Split-K accumulation: partial p (of P) += alpha A[:, pK:(p+1)K] B[:, pK:(p+1)K]^T into
// C + p*cstride; K is the per-partial depth (multiple of 16).
template <typename T>
void launch_gemm_nt_splitk(T* C, int64_t ldc, int64_t cstride, const T* A, int64_t lda, const T* B, int64_t ldb,
                           int64_t M, int64_t N, int64_t K, int P, T alpha, bool lower, hipStream_t s);

// Split-K rank-k accumulation on the tile mainloop (k_syrk.hip): partial p (of P) +=
// alpha A[:, pK:(p+1)K] A[:, pK:(p+1)K]^T into C + p*cstride, lower triangle of the leading
// N x N block plus the M - N rows below it.
template <typename T>
void launch_syrk_splitk(T* C, int64_t ldc, int64_t cstride, const T* A, int64_t lda, int64_t M, int64_t N, int64_t K,
                        int P, T alpha, hipStream_t s);
// C = alpha A B^T + beta C (no triangle) on 256 x 128 tiles (k_syrk.hip) when the shape allows:
// returns false otherwise (launch_gemm_nt then takes its own kernel)
template <typename T>
bool launch_gemm_tall(T* C, int64_t ldc, const T* A, int64_t lda, const T* B, int64_t ldb, int64_t M, int64_t N,
                      int64_t K, T alpha, T beta, hipStream_t s);

// Back substitution L^T alpha = z with z given as the m augmented rows (row-major output
// alpha: np x m, ld m).  Uses the diagonal-block inverses.
template <typename T>
void launch_backsolve(const T* A, int64_t ld, int64_t np, int m, const T* Linv, T* z, T* alpha, hipStream_t s);

// Same solve in one launch: one workgroup per 128-block, chained by flags (k_bsolve.hip).
// z is read from the label rows np..np+m-1 of A (ld).  A timed-out wait sets *info = -1.
// tiles/tld (optional, the distributed factor): tile (j, k) at tiles[j * (np/128) + k] with
// leading dimension tld[j], the label rows as row block np/128; A and ld unused then.
template <typename T>
void launch_backsolve_chain(const T* A, int64_t ld, int64_t np, int m, const T* Linv, T* alpha, int* info, Exec& ex,
                            hipStream_t s, const uint64_t* tiles = nullptr, const int64_t* tld = nullptr);
// Forward substitution z = L^{-1} r in place in the label rows (A + np, ld), one chained launch
template <typename T>
void launch_forward_chain(T* A, int64_t ld, int64_t np, int m, const T* Linv, int* info, Exec& ex, hipStream_t s);

// logdet partial = 2 sum log L_ii over i < n, datafit = sum of squares of the augmented
// rows; results accumulated in double on the device (out[0], out[1]).
template <typename T>
void launch_fit_reductions(const T* A, int64_t ld, int64_t n, int64_t np, int m, double* out,
                           hipStream_t s);  // out: 2 + 2 * (np / 128) doubles

// Fused prediction: mean (q x m row-major) and optional derivative (q x d x m).
template <typename T>
void launch_predict(const KCanon<T>& K, const T* X, const T* tabX, int64_t n, int d, int m, const T* alpha,
                    const T* Xq, const T* tabQ, int64_t q, T* mean, T* deriv, T* Z, T* out, hipStream_t s);

// LU with partial pivoting, always in double (k_getrf.hip): the fallback when the Cholesky
// reports a non-positive pivot, as the reference's default LU inverse (include/LAPACKUtils.h
// :38-56, 85-97).  A: np x np column-major (np a multiple of 128, identity padding); Ut: np x
// 128 scratch.
void lu_factor(double* A, int64_t ld, int64_t np, int* ipiv, int* info, double* Ut, hipStream_t s);
// B (np x m, column-major, ldb) <- A^{-1} B
void lu_solve(const double* A, int64_t ld, int64_t np, const int* ipiv, double* B, int64_t ldb, int m, hipStream_t s);
template <typename T>
void lu_rhs_from_rows(const T* Y, int64_t n, int m, double* B, int64_t ldb, int64_t np, hipStream_t s);
template <typename T>
void lu_rows_from_rhs(const double* B, int64_t ldb, int64_t n, int m, T* X, hipStream_t s);
// out[0] = sum log|U_ii| (i < n), out[1] = sign of det, out[2] = 1 if a U_ii is zero
void lu_logdet(const double* A, int64_t ld, int64_t n, const int* ipiv, double* out, hipStream_t s);
// out[c] = kab[c] - sum_{j<n} Ka[j, c] W[j, c]
template <typename T>
void lu_coldot(const double* Ka, const double* W, int64_t ld, int64_t n, int64_t q, const T* kab, T* out,
               hipStream_t s);

// fp64 iterative refinement of an fp32 fit (k_refine.hip)
template <typename S, typename D>
void launch_convert(const S* in, D* out, int64_t n, hipStream_t s);
void launch_residual_rows(const double* Y, const double* Kx, const double* a, double s2, int64_t n, int m, float* A,
                          int64_t ld, int64_t row0, int64_t ncols, int mp, hipStream_t s);
void launch_refine_accumulate(const float* delta, double* a, float* alpha, int64_t e, unsigned long long* nrm,
                              hipStream_t s);
// the sharded refinement: the rows this process's ranks own (idx, q of them)
void launch_gather_rows(const double* X, const int64_t* idx, int64_t q, int d, double* out, hipStream_t s);
void launch_residual_scatter(const double* Y, const double* Kx, const double* a, double s2, const int64_t* idx,
                             int64_t q, int m, float* rhs, hipStream_t s);

}  // namespace gprx
