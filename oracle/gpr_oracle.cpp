// =====================================================================================
//  gpr_oracle.cpp — TEST INFRASTRUCTURE, NOT PRODUCT CODE.
//
//  A CPU restatement of the agiger/GPR (reference) GP hot path, used ONLY as the parity
//  checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  The
//  product (libgprx, gpr_amd/) never links, loads or calls this file.
//
//  Every function below cites the reference line(s) it restates (paths are relative
//  to the reference repo root).  The reference itself cannot be compiled in this image
//  (Eigen3 and Boost are absent; see DESIGN.md "Oracle"), so this is a line-by-line
//  restatement of its arithmetic with the same scalar types and promotion rules:
//    * kernels + derivatives ............ include/Kernel.h:465-1036
//    * kernel-string factory ............ include/KernelFactory.h:83-178
//    * kernel / derivative matrices ..... lib/GaussianProcess.cpp:375-402, 472-495
//    * inversion dispatch ............... lib/GaussianProcess.cpp:531-618
//    * LAPACK LU / Cholesky inverse ..... include/LAPACKUtils.h:29-111 (runtime-resolved
//                                          LAPACK: MKL libmkl_rt, else system liblapack,
//                                          else the Eigen-style partial-pivot fallback)
//    * regression vectors ............... lib/GaussianProcess.cpp:642-672
//    * predict / derivative / variance .. lib/GaussianProcess.cpp:54-114, 684-706
//    * long-double determinant .......... lib/GaussianProcess.cpp:513-528
//    * Gaussian log likelihood .......... include/Likelihood.h:77-79, 166-344
//    * sparse PreComputeRegression ...... include/SparseGaussianProcess.h:174-313
//                                          (without the N x N core matrix, :309-311)
//    * sparse log likelihood ............ include/SparseLikelihood.h:129-145, 231-344
//  Parity pinning: see tests/test_oracle_kats.py (the reference's own deterministic
//  known-answer tests) and tests/test_oracle_numpy.py (independent numpy/scipy check).
// =====================================================================================
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <dlfcn.h>
#include <limits>
#include <memory>
#include <sstream>
#include <string>
#include <vector>
#include <omp.h>

namespace orc {

// ----------------------------------------------------------------------------------
// Error plumbing: the reference throws std::string; the oracle's C entry points turn
// that into a return code plus a retrievable message.
// ----------------------------------------------------------------------------------
static thread_local std::string g_err;

// ----------------------------------------------------------------------------------
// Runtime LAPACK (include/LAPACKUtils.h:13-27 declares the Fortran symbols).
// ----------------------------------------------------------------------------------
typedef void (*getrf_t)(int*, int*, double*, int*, int*, int*);
typedef void (*getri_t)(int*, double*, int*, int*, double*, int*, int*);
typedef void (*potrf_t)(char*, int*, double*, int*, int*);
typedef void (*potri_t)(char*, int*, double*, int*, int*);
typedef int (*ilaenv_t)(int*, char*, char*, int*, int*, int*, int*);
typedef void (*dgemm_t)(const char*, const char*, const int*, const int*, const int*, const double*, const double*,
                        const int*, const double*, const int*, const double*, double*, const int*);
typedef void (*sgemm_t)(const char*, const char*, const int*, const int*, const int*, const float*, const float*,
                        const int*, const float*, const int*, const float*, float*, const int*);

struct Lapack {
    getrf_t getrf = nullptr;
    getri_t getri = nullptr;
    potrf_t potrf = nullptr;
    potri_t potri = nullptr;
    ilaenv_t ilaenv = nullptr;
    dgemm_t dgemm = nullptr;  // BLAS GEMM for the oracle's Eigen products (optional)
    sgemm_t sgemm = nullptr;
    std::string name = "none (partial-pivot fallback)";
    bool ok() const { return getrf && getri && potrf && potri && ilaenv; }
};

static Lapack load_lapack() {
    Lapack L;
    if (const char* off = std::getenv("ORACLE_NO_LAPACK")) {
        if (off[0] == '1') return L;
    }
    // MKL + libgomp spin forever without the GNU threading layer.
    setenv("MKL_THREADING_LAYER", "GNU", 0);
    const char* cands[] = {"/opt/conda/lib/libmkl_rt.so.1", "libmkl_rt.so.1", "libmkl_rt.so",
                           "liblapack.so.3", "liblapack.so", "libopenblas.so.0"};
    for (const char* c : cands) {
        void* h = dlopen(c, RTLD_NOW | RTLD_LOCAL);
        if (!h) continue;
        Lapack T;
        T.getrf = (getrf_t)dlsym(h, "dgetrf_");
        T.getri = (getri_t)dlsym(h, "dgetri_");
        T.potrf = (potrf_t)dlsym(h, "dpotrf_");
        T.potri = (potri_t)dlsym(h, "dpotri_");
        T.ilaenv = (ilaenv_t)dlsym(h, "ilaenv_");
        T.dgemm = (dgemm_t)dlsym(h, "dgemm_");
        T.sgemm = (sgemm_t)dlsym(h, "sgemm_");
        if (T.ok()) {
            typedef int (*setlayer_t)(int);
            if (auto f = (setlayer_t)dlsym(h, "MKL_Set_Threading_Layer")) f(3 /* MKL_THREADING_GNU */);
            T.name = c;
            return T;
        }
        dlclose(h);
    }
    return L;
}

static Lapack& lapack() {
    static Lapack L = load_lapack();
    return L;
}

struct LapackFailure {};  // stands in for lapack::LAPACKException (include/LAPACKUtils.h:76-82)

// include/LAPACKUtils.h:29-56 — LU inverse in place, LWORK = N * ilaenv(1,"DGETRI")
static int lu_inversion(double* A, int N) {
    Lapack& L = lapack();
    int ispec = 1, m1 = -1;
    char name[] = "DGETRI";
    char opts[] = " ";
    int nb = L.ilaenv(&ispec, name, opts, &N, &m1, &m1, &m1);
    int lwork = N * std::max(nb, 1);
    std::vector<int> ipiv(N);
    std::vector<double> work((size_t)lwork);
    int info = 0;
    L.getrf(&N, &N, A, &N, ipiv.data(), &info);
    if (info != 0) return info;
    L.getri(&N, A, &N, ipiv.data(), work.data(), &lwork, &info);
    return info;
}

// include/LAPACKUtils.h:59-73 — Cholesky inverse ('L' on the row-major buffer), INFO ignored,
// then the row-major upper triangle is mirrored into the lower one.
static void chol_inversion(double* A, int N) {
    Lapack& L = lapack();
    int info = 0;
    char uplo = 'L';
    L.potrf(&uplo, &N, A, &N, &info);
    L.potri(&uplo, &N, A, &N, &info);
    for (int i = 0; i < N; i++)
        for (int j = i; j < N; j++) A[(size_t)j * N + i] = A[(size_t)i * N + j];
}

// Eigen's dense inverse() for dynamic matrices (used by lib/GaussianProcess.cpp:549,557):
// partial-pivot LU in T, then solve against the identity.
template <class T>
static std::vector<T> pp_lu_inverse(const std::vector<T>& K, int n) {
    std::vector<T> A(K);
    std::vector<int> perm(n);
    for (int i = 0; i < n; i++) perm[i] = i;
    for (int k = 0; k < n; k++) {
        int p = k;
        T best = std::fabs(A[(size_t)k * n + k]);
        for (int i = k + 1; i < n; i++) {
            T v = std::fabs(A[(size_t)i * n + k]);
            if (v > best) { best = v; p = i; }
        }
        if (p != k) {
            for (int j = 0; j < n; j++) std::swap(A[(size_t)k * n + j], A[(size_t)p * n + j]);
            std::swap(perm[k], perm[p]);
        }
        T piv = A[(size_t)k * n + k];
        if (piv == T(0)) continue;  // Eigen leaves inf/nan in this case
        for (int i = k + 1; i < n; i++) {
            T l = A[(size_t)i * n + k] / piv;
            A[(size_t)i * n + k] = l;
            for (int j = k + 1; j < n; j++) A[(size_t)i * n + j] -= l * A[(size_t)k * n + j];
        }
    }
    std::vector<T> inv((size_t)n * n, T(0));
#pragma omp parallel for schedule(static)
    for (int c = 0; c < n; c++) {
        std::vector<T> x(n);
        for (int i = 0; i < n; i++) x[i] = (perm[i] == c) ? T(1) : T(0);
        for (int i = 0; i < n; i++) {
            T s = x[i];
            for (int j = 0; j < i; j++) s -= A[(size_t)i * n + j] * x[j];
            x[i] = s;
        }
        for (int i = n - 1; i >= 0; i--) {
            T s = x[i];
            for (int j = i + 1; j < n; j++) s -= A[(size_t)i * n + j] * x[j];
            x[i] = s / A[(size_t)i * n + i];
        }
        for (int i = 0; i < n; i++) inv[(size_t)i * n + c] = x[i];
    }
    return inv;
}

// include/LAPACKUtils.h:85-97 — lu_invert<T>: cast to double, LAPACK LU inverse, cast back.
template <class T>
static std::vector<T> lu_invert(const std::vector<T>& K, int n) {
    if (!lapack().ok()) throw LapackFailure();
    std::vector<double> A(K.begin(), K.end());
    int info = lu_inversion(A.data(), n);
    if (info != 0) throw LapackFailure();
    return std::vector<T>(A.begin(), A.end());
}

// include/LAPACKUtils.h:100-111 — chol_invert<T>
template <class T>
static std::vector<T> chol_invert(const std::vector<T>& K, int n) {
    if (!lapack().ok()) throw LapackFailure();
    std::vector<double> A(K.begin(), K.end());
    chol_inversion(A.data(), n);
    return std::vector<T>(A.begin(), A.end());
}

enum InvMethod { FullPivotLU = 0, JacobiSVD = 1, BDCSVD = 2, SelfAdjointEigenSolver = 3 };

// lib/GaussianProcess.cpp:531-618 — InvertKernelMatrix (LU and Cholesky branches; the SVD
// branches are out of scope for this path).
template <class T>
static std::vector<T> invert(const std::vector<T>& K, int n, int method, bool stable) {
    if (method == FullPivotLU) {
        try {
            if (stable) return pp_lu_inverse<T>(K, n);
            return lu_invert<T>(K, n);
        } catch (LapackFailure&) {
            return pp_lu_inverse<T>(K, n);
        }
    }
    if (method == SelfAdjointEigenSolver) {
        try {
            return chol_invert<T>(K, n);
        } catch (LapackFailure&) {
            throw std::string("oracle: eigen-solver fallback of SelfAdjointEigenSolver needs LAPACK");
        }
    }
    throw std::string("oracle: SVD inversion methods are out of scope");
}

// ----------------------------------------------------------------------------------
// Kernel tree (include/Kernel.h).  Parameters are stored as T, exactly like the reference
// members; derived members (sigma2, sigma3, scale2) are computed as in the SetParameters
// helpers (:523-542, :642-659, :754-762, :855-874, :996-1018).
// ----------------------------------------------------------------------------------
enum Kind { GAUSS = 1, GAUSS_EXP = 2, WHITE = 3, RQ = 4, PERIODIC = 5, SUM = 6, PRODUCT = 7 };

template <class T>
struct Node {
    int kind = 0;
    T p[3] = {0, 0, 0};
    T sigma2 = 0, sigma3 = 0, scale2 = 0;
    std::unique_ptr<Node> a, b;
    int nparams() const {
        switch (kind) {
            case GAUSS: case GAUSS_EXP: return 2;
            case WHITE: return 1;
            case RQ: case PERIODIC: return 3;
            default: return a->nparams() + b->nparams();
        }
    }
};

template <class T>
static T s2p(const std::string& s) {  // Kernel::S2P (include/Kernel.h:135-141)
    T p;
    std::stringstream ss;
    ss << s;
    ss >> p;
    return p;
}

template <class T>
static std::unique_ptr<Node<T>> make_leaf(const std::string& type, const std::vector<std::string>& ps) {
    std::unique_ptr<Node<T>> n(new Node<T>());
    auto need = [&](size_t k) {
        if (ps.size() != k) throw std::string(type + "::Load: wrong number of kernel parameters.");
    };
    if (type == "GaussianKernel") {  // :453-559 ; params (sigma, scale)
        need(2);
        n->kind = GAUSS;
        n->p[0] = s2p<T>(ps[0]);
        n->p[1] = s2p<T>(ps[1]);
        if (n->p[0] == 0) throw std::string("GaussianKernel: sigma has to be positive");
        if (n->p[1] == 0) throw std::string("GaussianKernel: scale has to be positive");
        n->sigma2 = n->p[0] * n->p[0];
        n->sigma3 = n->p[0] * n->p[0] * n->p[0];
        n->scale2 = n->p[1] * n->p[1];
    } else if (type == "GaussianExpKernel") {  // :568-676 ; params (sigma, scale), no validation
        need(2);
        n->kind = GAUSS_EXP;
        n->p[0] = s2p<T>(ps[0]);
        n->p[1] = s2p<T>(ps[1]);
    } else if (type == "WhiteKernel") {  // :684-773 ; params (scale)
        need(1);
        n->kind = WHITE;
        n->p[0] = s2p<T>(ps[0]);
        n->scale2 = n->p[0] * n->p[0];
    } else if (type == "RationalQuadraticKernel") {  // :783-891 ; params (scale, sigma, alpha)
        need(3);
        n->kind = RQ;
        for (int i = 0; i < 3; i++) n->p[i] = s2p<T>(ps[i]);
        n->scale2 = n->p[0] * n->p[0];
        n->sigma2 = n->p[1] * n->p[1];
        n->sigma3 = n->p[1] * n->p[1] * n->p[1];
    } else if (type == "PeriodicKernel") {  // :901-1036 ; params (scale, b, sigma)
        need(3);
        n->kind = PERIODIC;
        for (int i = 0; i < 3; i++) n->p[i] = s2p<T>(ps[i]);
        if (n->p[0] == 0) throw std::string("PeriodicKernel: scale parameter has to be positive.");
        if (n->p[1] == 0) throw std::string("PeriodicKernel: period length parameter has to be positive.");
        if (n->p[2] == 0) throw std::string("PeriodicKernel: sigma parameter has to be positive.");
        n->scale2 = n->p[0] * n->p[0];
        n->sigma2 = n->p[2] * n->p[2];
        n->sigma3 = n->p[2] * n->p[2] * n->p[2];
    } else {
        throw std::string("KernelFactory::GetKernel: failed to load kernel.");
    }
    return n;
}

// include/KernelFactory.h:83-178 — recursive parse; `ks` is consumed by reference exactly
// like the reference's kernel_string argument.
template <class T>
static std::unique_ptr<Node<T>> parse(std::string& ks) {
    std::stringstream line(ks);
    std::string type;
    if (!std::getline(line, type, '('))
        throw std::string("KernelFactory::GetKernel: failed to tokanize kernel name string");
    if (type == "SumKernel" || type == "ProductKernel") {
        ks = ks.substr(type.size() + 1);
        std::unique_ptr<Node<T>> k1 = parse<T>(ks);
        size_t pos = ks.find("),");
        if (pos == std::string::npos)
            throw std::string("KernelFactory::GetKernel: failed to tokanize  composite kernel name string");
        ks = ks.substr(pos + 2);
        std::unique_ptr<Node<T>> k2 = parse<T>(ks);
        std::unique_ptr<Node<T>> n(new Node<T>());
        n->kind = (type == "SumKernel") ? SUM : PRODUCT;
        n->a = std::move(k1);
        n->b = std::move(k2);
        return n;
    }
    std::vector<std::string> ps;
    for (;;) {
        std::string p;
        if (!std::getline(line, p, ',')) break;
        if (p.find(")") != std::string::npos) break;
        ps.push_back(p);
    }
    return make_leaf<T>(type, ps);
}

template <class T>
static T norm_diff(const T* x, const T* y, int d) {  // Eigen (x-y).norm()
    T s = 0;
    for (int k = 0; k < d; k++) {
        T t = x[k] - y[k];
        s += t * t;
    }
    return std::sqrt(s);
}

// operator() of every kernel class
template <class T>
static T keval(const Node<T>& n, const T* x, const T* y, int d) {
    switch (n.kind) {
        case GAUSS: {  // include/Kernel.h:465-468
            T r = norm_diff(x, y, d);
            return n.scale2 * std::exp(-0.5 * (r * r) / (n.sigma2));
        }
        case GAUSS_EXP: {  // :580-585
            T r = norm_diff(x, y, d);
            T es = std::exp(n.p[1]);
            T eg = std::exp(n.p[0]);
            return es * es * std::exp(-0.5 * (r * r) / (eg * eg));
        }
        case WHITE: {  // :695-702 (exact equality)
            if (norm_diff(x, y, d) == 0) return n.scale2;
            return 0;
        }
        case RQ: {  // :794-797
            T r = norm_diff(x, y, d);
            return n.scale2 * std::pow(1 + 0.5 * (r * r) / (n.sigma2 * n.p[2]), -n.p[2]);
        }
        case PERIODIC: {  // :912-920
            T sum = 0;
            for (int i = 0; i < d; i++) {
                double f = std::sin(n.p[1] * (x[i] - y[i]));
                sum += f * f;
            }
            return n.scale2 * std::exp(-0.5 * sum / n.sigma2);
        }
        case SUM:  // :165-167
            return keval(*n.a, x, y, d) + keval(*n.b, x, y, d);
        case PRODUCT:  // :314-316
            return keval(*n.a, x, y, d) * keval(*n.b, x, y, d);
    }
    return 0;
}

// GetDerivative() of every kernel class; appends n.nparams() entries to out
template <class T>
static void kgrad(const Node<T>& n, const T* x, const T* y, int d, std::vector<T>& out) {
    switch (n.kind) {
        case GAUSS: {  // :471-479
            T r = norm_diff(x, y, d);
            T f = std::exp(-0.5 * (r * r) / (n.sigma2));
            out.push_back(n.scale2 * (r * r) / (n.sigma3) * f);
            out.push_back(2 * n.p[1] * f);
            return;
        }
        case GAUSS_EXP: {  // :588-598
            T sigma = n.p[0], scale = n.p[1];
            T r = norm_diff(x, y, d);
            T r2 = r * r;
            T f1 = std::exp(-2 * sigma);
            T f2 = std::exp(2 * sigma);
            out.push_back(r2 * std::exp(-0.5 * f1 * ((4 * sigma - 4 * scale) * f2 + r2)));
            out.push_back(2 * std::exp(0.5 * f1 * (4 * f2 * scale - r2)));
            return;
        }
        case WHITE: {  // :704-713
            if (norm_diff(x, y, d) == 0) out.push_back(2 * n.p[0]);
            else out.push_back(0);
            return;
        }
        case RQ: {  // :799-808
            T scale = n.p[0], alpha = n.p[2];
            T r = norm_diff(x, y, d);
            T f = 0.5 * r * r / (n.sigma2 * alpha) + 1;
            out.push_back(2 * scale * std::pow(f, -alpha));
            out.push_back(n.scale2 * (r * r) * std::pow(f, -alpha - 1) / n.sigma3);
            out.push_back(n.scale2 * ((r * r / (2 * n.sigma2 * f * alpha)) - std::log(f)) * std::pow(f, -alpha));
            return;
        }
        case PERIODIC: {  // :922-948
            T b = n.p[1];
            T f1 = 0;
            for (int i = 0; i < d; i++) {
                double r = std::sin(b * (x[i] - y[i]));
                f1 += r * r;
            }
            T f2 = 0;
            for (int i = 0; i < d; i++) {
                double r = (x[i] - y[i]);
                f2 += 2 * r * std::cos(b * r) * std::sin(b * r);
            }
            T f3 = 0;
            for (int i = 0; i < d; i++) {
                double r = (x[i] - y[i]);
                double v = std::sin(b * r);
                f3 += (v * v);
            }
            out.push_back(2 * n.p[0] * std::exp(-0.5 * f1 / n.sigma2));
            out.push_back(-0.5 * n.scale2 * std::exp(-0.5 * f1 / n.sigma2) * f2 / n.sigma2);
            out.push_back(n.scale2 * std::exp(-0.5 * f1 / n.sigma2) * f3 / n.sigma3);
            return;
        }
        case SUM: {  // :169-178
            kgrad(*n.a, x, y, d, out);
            kgrad(*n.b, x, y, d, out);
            return;
        }
        case PRODUCT: {  // :318-327
            size_t s0 = out.size();
            kgrad(*n.a, x, y, d, out);
            size_t s1 = out.size();
            kgrad(*n.b, x, y, d, out);
            T k2 = keval(*n.b, x, y, d);
            T k1 = keval(*n.a, x, y, d);
            for (size_t i = s0; i < s1; i++) out[i] = out[i] * k2;
            for (size_t i = s1; i < out.size(); i++) out[i] = out[i] * k1;
            return;
        }
    }
}

// Kernel<T>::SetParameters for every leaf in GetParameters() order (include/Kernel.h:239-245,
// 514-520, 633-639, 745-751, 846-852, 987-993) with the constructor-time validation.
template <class T>
static void set_params(Node<T>& n, const T* p, int& idx) {
    switch (n.kind) {
        case SUM:
        case PRODUCT:
            set_params(*n.a, p, idx);
            set_params(*n.b, p, idx);
            return;
        case GAUSS:
            n.p[0] = p[idx++];
            n.p[1] = p[idx++];
            if (n.p[0] == 0) throw std::string("GaussianKernel: sigma has to be positive");
            if (n.p[1] == 0) throw std::string("GaussianKernel: scale has to be positive");
            n.sigma2 = n.p[0] * n.p[0];
            n.sigma3 = n.p[0] * n.p[0] * n.p[0];
            n.scale2 = n.p[1] * n.p[1];
            return;
        case GAUSS_EXP:
            n.p[0] = p[idx++];
            n.p[1] = p[idx++];
            return;
        case WHITE:
            n.p[0] = p[idx++];
            n.scale2 = n.p[0] * n.p[0];
            return;
        case RQ:
            for (int i = 0; i < 3; i++) n.p[i] = p[idx++];
            n.scale2 = n.p[0] * n.p[0];
            n.sigma2 = n.p[1] * n.p[1];
            n.sigma3 = n.p[1] * n.p[1] * n.p[1];
            return;
        case PERIODIC:
            for (int i = 0; i < 3; i++) n.p[i] = p[idx++];
            if (n.p[0] == 0) throw std::string("PeriodicKernel: scale parameter has to be positive.");
            if (n.p[1] == 0) throw std::string("PeriodicKernel: period length parameter has to be positive.");
            if (n.p[2] == 0) throw std::string("PeriodicKernel: sigma parameter has to be positive.");
            n.scale2 = n.p[0] * n.p[0];
            n.sigma2 = n.p[2] * n.p[2];
            n.sigma3 = n.p[2] * n.p[2] * n.p[2];
            return;
    }
}

template <class T>
static std::unique_ptr<Node<T>> kernel_from(const char* kstr) {
    std::string s(kstr);
    return parse<T>(s);
}

// lib/GaussianProcess.cpp:384-402 — full symmetric matrix from the upper loop, non-finite check
template <class T>
static void kernel_matrix(const Node<T>& k, const T* X, int n, int d, T* M) {
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; i++)
        for (int j = i; j < n; j++) {
            T v = keval(k, X + (size_t)i * d, X + (size_t)j * d, d);
            M[(size_t)i * n + j] = v;
            M[(size_t)j * n + i] = v;
        }
    for (size_t e = 0; e < (size_t)n * n; e++) {
        T z = M[e] - M[e];
        if (!(z == z))
            throw std::string("GaussianProcess::ComputeKernelMatrixInternal: kernel matrix contains entries which are not finite.");
    }
}

// lib/GaussianProcess.cpp:472-495 — stacked derivative matrices [D_0; ...; D_{P-1}]
template <class T>
static void deriv_matrix(const Node<T>& k, const T* X, int n, int d, T* M) {
    const int P = k.nparams();
#pragma omp parallel for schedule(dynamic, 16)
    for (int i = 0; i < n; i++) {
        std::vector<T> v;
        for (int j = i; j < n; j++) {
            v.clear();
            kgrad(k, X + (size_t)i * d, X + (size_t)j * d, d, v);
            for (int p = 0; p < P; p++) {
                M[((size_t)i + (size_t)p * n) * n + j] = v[p];
                M[((size_t)j + (size_t)p * n) * n + i] = v[p];
            }
        }
    }
}

// Column-major BLAS GEMM in T (C = alpha op(A) op(B) + beta C); false when the runtime
// library has none (the callers then loop).  Eigen's products (the reference's) are blocked
// GEMMs in T with an unspecified summation order, as BLAS's are.
static bool blas_gemm(char ta, char tb, int m, int n, int k, double alpha, const double* A, int lda, const double* B,
                      int ldb, double beta, double* C, int ldc) {
    if (!lapack().dgemm) return false;
    lapack().dgemm(&ta, &tb, &m, &n, &k, &alpha, A, &lda, B, &ldb, &beta, C, &ldc);
    return true;
}
static bool blas_gemm(char ta, char tb, int m, int n, int k, float alpha, const float* A, int lda, const float* B,
                      int ldb, float beta, float* C, int ldc) {
    if (!lapack().sgemm) return false;
    lapack().sgemm(&ta, &tb, &m, &n, &k, &alpha, A, &lda, B, &ldb, &beta, C, &ldc);
    return true;
}

// Eigen-style row-major GEMM in T: C(r x c) = A(r x k) * B(k x c)
template <class T>
static void gemm(const T* A, const T* B, T* C, int r, int kk, int c) {
    // row-major C = A B is column-major C^T = B^T A^T
    if (blas_gemm('N', 'N', c, r, kk, T(1), B, c, A, kk, T(0), C, c)) return;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < r; i++) {
        for (int j = 0; j < c; j++) C[(size_t)i * c + j] = 0;
        for (int l = 0; l < kk; l++) {
            T a = A[(size_t)i * kk + l];
            const T* b = B + (size_t)l * c;
            T* cr = C + (size_t)i * c;
            for (int j = 0; j < c; j++) cr[j] += a * b[j];
        }
    }
}

// lib/GaussianProcess.cpp:513-528 — det of (K + sigma^2 I) cast to long double
// (Eigen's determinant() = partial-pivot LU in the cast scalar type).
template <class T>
static long double det_long_double(const std::vector<T>& K, int n) {
    std::vector<long double> A(K.begin(), K.end());
    long double det = 1;
    for (int k = 0; k < n; k++) {
        int p = k;
        long double best = std::fabs(A[(size_t)k * n + k]);
        for (int i = k + 1; i < n; i++) {
            long double v = std::fabs(A[(size_t)i * n + k]);
            if (v > best) { best = v; p = i; }
        }
        if (p != k) {
            for (int j = 0; j < n; j++) std::swap(A[(size_t)k * n + j], A[(size_t)p * n + j]);
            det = -det;
        }
        long double piv = A[(size_t)k * n + k];
        det *= piv;
        if (piv == 0) continue;
#pragma omp parallel for schedule(static) if (n - k > 256)
        for (int i = k + 1; i < n; i++) {
            long double l = A[(size_t)i * n + k] / piv;
            for (int j = k + 1; j < n; j++) A[(size_t)i * n + j] -= l * A[(size_t)k * n + j];
        }
    }
    return det;
}

// Core matrix C = inv(K + sigma^2 I)  (lib/GaussianProcess.cpp:498-510, 375-381)
template <class T>
static std::vector<T> core_matrix(const Node<T>& k, const T* X, int n, int d, T sigma, int method,
                                  std::vector<T>* Kout) {
    std::vector<T> K((size_t)n * n);
    kernel_matrix(k, X, n, d, K.data());
    for (int i = 0; i < n; i++) K[(size_t)i * n + i] += sigma * sigma;
    std::vector<T> C = invert<T>(K, n, method, false);
    if (Kout) *Kout = std::move(K);
    return C;
}

// SparseGaussianLogLikelihood::GetValueAndParameterDerivatives, include/SparseLikelihood.h:
// 231-344, with its N x N matrices (small n only): ComputeCoreMatrices
// (include/SparseGaussianProcess.h:323-350), EfficientInversion (SparseLikelihood.h:129-135),
// the derivative stacks (SparseGaussianProcess.h:237-264, 380+), A_p (:246-252), the data-fit
// and complexity gradients (:255-273), EfficientDeterminant (:138-145) with the clamps
// (:305-314) and the constant term (:325).  Y is n x 1.  det_out: the long-double
// determinant; logdet_out: log of its three factors summed (exact).
// The sparse likelihood's core quantities: SparseGaussianProcess::ComputeCoreMatrices
// (include/SparseGaussianProcess.h:323-350: K = Kmm + jitter I, K_inv, Knm, I_sigma),
// SparseGaussianLogLikelihood::EfficientInversion (include/SparseLikelihood.h:129-135, called
// with B = K_inv, B_inv = K: C_inv = inv(sigma^2 I + Knm K_inv Knm^T) by Woodbury) and the
// "inner" matrix B_inv + X^T A_inv X = K + Knm^T Knm / sigma^2 whose determinant enters
// EfficientDeterminant (:138-145).
template <class T>
struct SparseCore {
    std::vector<T> K, Kinv, Knm, inner, Cinv;
    T s2, ainv;
};
template <class T>
static SparseCore<T> sparse_core(const Node<T>& k, const T* X, int n, int d, const T* Xm, int M, T sigma, T jitter) {
    if (M == 0)
        throw std::string("SparseLikelihood::GetValueAndParameterDerivative: there are no inducing samples specified");
    SparseCore<T> c;
    const bool stable = (jitter < std::numeric_limits<T>::min()) ? true : false;
    // ComputeKernelMatrixWithJitter (SparseGaussianProcess.h:174-180), InvertKernelMatrix
    c.K.resize((size_t)M * M);
    kernel_matrix(k, Xm, M, d, c.K.data());
    for (int i = 0; i < M; i++) c.K[(size_t)i * M + i] += jitter;
    c.Kinv = invert<T>(c.K, M, FullPivotLU, stable);
    if (!(M <= n))
        throw std::string("SparseGaussianProcess::ComputeKernelVectorMatrix: number of dense samples must be higher than the number of sparse samples");
    c.Knm.resize((size_t)n * M);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++)
        for (int j = 0; j < M; j++) c.Knm[(size_t)i * M + j] = keval(k, X + (size_t)i * d, Xm + (size_t)j * d, d);
    if (sigma <= 0) throw std::string("SparseGaussianProcess::ComputeCoreMatrices: sigma must be positive.");
    if (n == 0) throw std::string("SparseGaussianProcess::ComputeCoreMatrices: empty sample set.");
    c.s2 = sigma * sigma;     // I_sigma diagonal (GetSigmaSquared)
    c.ainv = T(1.0) / c.s2;  // A_inv = 1 / A.diagonal()
    const T ainv = c.ainv;
    const std::vector<T>& Knm = c.Knm;
    // EfficientInversion: inner = B_inv + X^T A_inv X = K + Knm^T A_inv Knm; C_inv = A_inv - A_inv X inner^-1 X^T A_inv
    c.inner.assign((size_t)M * M, T(0));
#pragma omp parallel for schedule(static)
    for (int a = 0; a < M; a++)
        for (int b = 0; b < M; b++) {
            T acc = 0;
            for (int i = 0; i < n; i++) acc += Knm[(size_t)i * M + a] * ainv * Knm[(size_t)i * M + b];
            c.inner[(size_t)a * M + b] = c.K[(size_t)a * M + b] + acc;
        }
    std::vector<T> inner_inv = invert<T>(c.inner, M, FullPivotLU, false);  // GetInverseMatrix (SparseLikelihood.h:100-102)
    std::vector<T> Z((size_t)n * M);  // X inner^-1
    gemm(Knm.data(), inner_inv.data(), Z.data(), n, M, M);
    c.Cinv.resize((size_t)n * n);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) {
            T acc = 0;
            for (int a = 0; a < M; a++) acc += Z[(size_t)i * M + a] * Knm[(size_t)j * M + a];
            c.Cinv[(size_t)i * n + j] = (i == j ? ainv : T(0)) - ainv * acc * ainv;
        }
    return c;
}

template <class T>
static void sparse_lml(const Node<T>& k, const T* X, const T* Y, int n, int d, const T* Xm, int M, T sigma, T jitter,
                       T* value, T* grad, double* det_out, double* logdet_out) {
    typedef long double HP;
    SparseCore<T> core = sparse_core(k, X, n, d, Xm, M, sigma, jitter);
    const std::vector<T>&Kinv = core.Kinv, &Knm = core.Knm, &inner = core.inner, &Cinv = core.Cinv;
    const T s2 = core.s2;
    // data fit (:301-302): -0.5 Y^T C_inv Y
    std::vector<T> v(n);  // C_inv Y
    for (int i = 0; i < n; i++) {
        T acc = 0;
        for (int j = 0; j < n; j++) acc += Cinv[(size_t)i * n + j] * Y[j];
        v[i] = acc;
    }
    T df = 0;
    for (int i = 0; i < n; i++) df += Y[i] * v[i];
    df = -0.5 * df;
    // EfficientDeterminant: |A + X B X'| = |B| |A| |inv(B) + X' inv(A) X|, B = K_inv
    HP det_B = det_long_double(Kinv, M);
    if (std::isinf(det_B)) det_B = std::numeric_limits<HP>::max();
    HP prodA = 1;
    for (int i = 0; i < n; i++) prodA *= (HP)s2;
    const HP det_inner = det_long_double(inner, M);
    const HP determinant = det_B * prodA * det_inner;
    if (det_out) *det_out = (double)determinant;
    if (logdet_out)
        *logdet_out = (double)(std::log(std::fabs(det_long_double(Kinv, M))) + (HP)n * std::log((HP)s2) +
                               std::log(std::fabs(det_inner)));
    HP cp;
    if (determinant <= std::numeric_limits<HP>::min() || std::isnan(determinant))
        cp = -0.5 * std::log(std::numeric_limits<HP>::min());
    else if (determinant > std::numeric_limits<HP>::max())
        cp = -0.5 * std::log(std::numeric_limits<HP>::max());
    else
        cp = -0.5 * std::log(determinant);
    const T ct = -(n / 2.0) * std::log(2 * M_PI);
    const T val = df + (T)(cp + ct);
    if (std::isnan(val))
        throw std::string("SparseLikelihood::GetValueAndParameterDerivative: likelihood value is not a number.");
    *value = val;
    if (!grad) return;
    // Kmm_d (P stacked M x M, no jitter) and Knm_d (P stacked n x M)
    const int P = k.nparams();
    std::vector<T> Kmm_d((size_t)P * M * M), Knm_d((size_t)P * n * M);
    deriv_matrix(k, Xm, M, d, Kmm_d.data());
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++) {
        std::vector<T> g;
        for (int j = 0; j < M; j++) {
            g.clear();
            kgrad(k, X + (size_t)i * d, Xm + (size_t)j * d, d, g);
            for (int p = 0; p < P; p++) Knm_d[((size_t)p * n + i) * M + j] = g[p];
        }
    }
    std::vector<T> W((size_t)n * M);  // Knm K_inv
    gemm(Knm.data(), Kinv.data(), W.data(), n, M, M);
    std::vector<T> Ap((size_t)n * n), T1((size_t)n * M), T2((size_t)M * M), Q((size_t)n * M);
    for (int p = 0; p < P; p++) {
        const T* Dp = Knm_d.data() + (size_t)p * n * M;
        const T* Ep = Kmm_d.data() + (size_t)p * M * M;
        gemm(Dp, Kinv.data(), T1.data(), n, M, M);  // Knm_d K_inv
        gemm(Ep, Kinv.data(), T2.data(), M, M, M);  // Kmm_d K_inv
        gemm(W.data(), T2.data(), Q.data(), n, M, M);  // Knm K_inv Kmm_d K_inv
#pragma omp parallel for schedule(static)
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++) {
                T a = 0, b = 0, c = 0;
                for (int l = 0; l < M; l++) {
                    a += T1[(size_t)i * M + l] * Knm[(size_t)j * M + l];  // Knm_d K_inv Knm^T
                    b += Q[(size_t)i * M + l] * Knm[(size_t)j * M + l];   // Knm K_inv Kmm_d K_inv Knm^T
                    c += W[(size_t)i * M + l] * Dp[(size_t)j * M + l];    // Knm K_inv Knm_d^T
                }
                Ap[(size_t)i * n + j] = a - b + c;
            }
        // 0.5 Y^T C_inv A_p C_inv Y (C_inv symmetric: v^T A_p v) and -0.5 tr(C_inv A_p)
        T dt = 0, tr = 0;
        for (int i = 0; i < n; i++) {
            T r = 0, q = 0;
            for (int j = 0; j < n; j++) {
                r += Ap[(size_t)i * n + j] * v[j];
                q += Cinv[(size_t)i * n + j] * Ap[(size_t)j * n + i];
            }
            dt += v[i] * r;
            tr += q;
        }
        grad[p] = 0.5 * dt - 0.5 * tr;
    }
}

}  // namespace orc

using namespace orc;

// =====================================================================================
// C entry points (ctypes from tests/ and bench.py).  Return 0 on success, nonzero with
// orc_last_error() set otherwise.  All matrices are row-major, like the reference.
// =====================================================================================
#define ORC_TRY try {
#define ORC_CATCH                           \
    }                                       \
    catch (std::string & e) {               \
        orc::g_err = e;                     \
        return 1;                           \
    }                                       \
    catch (std::exception & e) {            \
        orc::g_err = e.what();              \
        return 2;                           \
    }                                       \
    return 0;

extern "C" {

const char* orc_last_error() { return orc::g_err.c_str(); }
const char* orc_lapack_name() { return orc::lapack().name.c_str(); }
int orc_num_threads() { return omp_get_max_threads(); }

#define ORC_DEFINE(SUF, T)                                                                         \
    int orc_kernel_nparams_##SUF(const char* ks, int* np) {                                        \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        *np = k->nparams();                                                                        \
        ORC_CATCH                                                                                  \
    }                                                                                              \
    int orc_kernel_eval_##SUF(const char* ks, const T* x, const T* y, int d, T* val, T* grad) {    \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        *val = keval(*k, x, y, d);                                                                 \
        if (grad) {                                                                                \
            std::vector<T> g;                                                                      \
            kgrad(*k, x, y, d, g);                                                                 \
            std::copy(g.begin(), g.end(), grad);                                                   \
        }                                                                                          \
        ORC_CATCH                                                                                  \
    }                                                                                              \
    /* B parameter vectors (B x P, GetParameters order) on one (x, y) pair: val (B), grad (B x P) */ \
    int orc_kernel_eval_params_##SUF(const char* ks, const T* params, int B, const T* x, const T* y, int d,  \
                                     T* val, T* grad) {                                            \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        const int P = k->nparams();                                                                \
        for (int b = 0; b < B; b++) {                                                              \
            int idx = 0;                                                                           \
            set_params(*k, params + (size_t)b * P, idx);                                           \
            val[b] = keval(*k, x, y, d);                                                           \
            if (grad) {                                                                            \
                std::vector<T> g;                                                                  \
                kgrad(*k, x, y, d, g);                                                             \
                std::copy(g.begin(), g.end(), grad + (size_t)b * P);                               \
            }                                                                                      \
        }                                                                                          \
        ORC_CATCH                                                                                  \
    }                                                                                              \
    int orc_kernel_matrix_##SUF(const char* ks, const T* X, int n, int d, T* K) {                  \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        kernel_matrix(*k, X, n, d, K);                                                             \
        ORC_CATCH                                                                                  \
    }                                                                                              \
    int orc_cross_matrix_##SUF(const char* ks, const T* A, int na, const T* B, int nb, int d,      \
                               T* K) { /* include/SparseGaussianProcess.h:218-235 */               \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        _Pragma("omp parallel for schedule(static)") for (int i = 0; i < na; i++) for (int j = 0;  \
                                                                                     j < nb; j++)  \
            K[(size_t)i * nb + j] = keval(*k, A + (size_t)i * d, B + (size_t)j * d, d);            \
        ORC_CATCH                                                                                  \
    }                                                                                              \
    int orc_deriv_matrix_##SUF(const char* ks, const T* X, int n, int d, T* D) {                   \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        deriv_matrix(*k, X, n, d, D);                                                              \
        ORC_CATCH                                                                                  \
    }                                                                                              \
    int orc_invert_##SUF(const T* K, int n, int method, int stable, T* C) {                        \
        ORC_TRY std::vector<T> k(K, K + (size_t)n * n);                                            \
        std::vector<T> c = invert<T>(k, n, method, stable != 0);                                   \
        std::copy(c.begin(), c.end(), C);                                                          \
        ORC_CATCH                                                                                  \
    }                                                                                              \
    /* Initialize(): lib/GaussianProcess.cpp:118-130, 642-672.  C may be NULL. */                  \
    int orc_fit_##SUF(const char* ks, const T* X, const T* Y, int n, int d, int m, T sigma,        \
                      int method, T* alpha, T* C) {                                                \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        std::vector<T> c = core_matrix(*k, X, n, d, sigma, method, (std::vector<T>*)nullptr);                       \
        gemm(c.data(), Y, alpha, n, n, m);                                                         \
        if (C) std::copy(c.begin(), c.end(), C);                                                   \
        ORC_CATCH                                                                                  \
    }                                                                                              \
    /* Predict / PredictDerivative: lib/GaussianProcess.cpp:54-81, 684-706.  D may be NULL; */     \
    /* D is (q, d, m) row-major = per query the reference's d x m matrix. */                       \
    int orc_predict_##SUF(const char* ks, const T* X, int n, int d, int m, const T* alpha,         \
                          const T* Xq, int q, T* mean, T* D) {                                     \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        _Pragma("omp parallel for schedule(static)") for (int t = 0; t < q; t++) {                 \
            const T* x = Xq + (size_t)t * d;                                                       \
            std::vector<T> kx(n);                                                                  \
            for (int i = 0; i < n; i++) kx[i] = keval(*k, x, X + (size_t)i * d, d);                \
            for (int c = 0; c < m; c++) {                                                          \
                T s = 0;                                                                           \
                for (int i = 0; i < n; i++) s += kx[i] * alpha[(size_t)i * m + c];                 \
                mean[(size_t)t * m + c] = s;                                                       \
            }                                                                                      \
            if (D) {                                                                               \
                for (int c = 0; c < m; c++)                                                        \
                    for (int j = 0; j < d; j++) {                                                  \
                        T s = 0;                                                                   \
                        for (int i = 0; i < n; i++)                                                \
                            s += (x[j] - X[(size_t)i * d + j]) * (kx[i] * alpha[(size_t)i * m + c]); \
                        D[((size_t)t * d + j) * m + c] = -s;                                       \
                    }                                                                              \
            }                                                                                      \
        }                                                                                          \
        ORC_CATCH                                                                                  \
    }                                                                                              \
    /* operator()(x,y) = k(x,y) - Kx' C Ky: lib/GaussianProcess.cpp:84-99 (per query pair) */     \
    int orc_posterior_cov_##SUF(const char* ks, const T* X, int n, int d, const T* C,              \
                                const T* Xa, const T* Xb, int q, T* out) {                         \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        _Pragma("omp parallel for schedule(static)") for (int t = 0; t < q; t++) {                 \
            const T* xa = Xa + (size_t)t * d;                                                      \
            const T* xb = Xb + (size_t)t * d;                                                      \
            std::vector<T> ka(n), kb(n);                                                           \
            for (int i = 0; i < n; i++) {                                                          \
                ka[i] = keval(*k, xa, X + (size_t)i * d, d);                                       \
                kb[i] = keval(*k, xb, X + (size_t)i * d, d);                                       \
            }                                                                                      \
            T s = 0;                                                                               \
            for (int i = 0; i < n; i++) {                                                          \
                T r = 0;                                                                           \
                for (int j = 0; j < n; j++) r += C[(size_t)i * n + j] * kb[j];                     \
                s += ka[i] * r;                                                                    \
            }                                                                                      \
            out[t] = keval(*k, xa, xb, d) - s;                                                     \
        }                                                                                          \
        ORC_CATCH                                                                                  \
    }                                                                                              \
    /* GaussianLogLikelihood::GetValueAndParameterDerivatives, include/Likelihood.h:231-285. */    \
    /* m must be 1 (the reference's df is m x m assigned to a vector, :175).  grad may be */       \
    /* NULL (then only operator(), :166-202, is evaluated).  det_out receives the */               \
    /* long-double determinant BEFORE narrowing, logdet_out log|det| in long double. */            \
    int orc_lml_##SUF(const char* ks, const T* X, const T* Y, int n, int d, T sigma, int method,   \
                      T* value, T* grad, double* det_out, double* logdet_out) {                    \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        std::vector<T> K;                                                                          \
        std::vector<T> C = core_matrix(*k, X, n, d, sigma, method, &K);                            \
        long double det_ld = det_long_double(K, n);                                                \
        if (det_out) *det_out = (double)det_ld;                                                    \
        if (logdet_out) *logdet_out = (double)std::log(std::fabs(det_ld));                         \
        typedef long double HP;                                                                    \
        HP determinant = (T)det_ld; /* narrowed by Likelihood::GetCoreMatrix (:77-79) */           \
        std::vector<T> alpha(n);                                                                   \
        gemm(C.data(), Y, alpha.data(), n, n, 1);                                                  \
        T df = 0;                                                                                  \
        for (int i = 0; i < n; i++) df += Y[i] * alpha[i];                                         \
        df = -0.5 * df;                                                                            \
        HP cp;                                                                                     \
        if (determinant <= std::numeric_limits<HP>::min())                                         \
            cp = -0.5 * std::log(std::numeric_limits<HP>::min());                                  \
        else if (determinant > std::numeric_limits<HP>::max())                                     \
            cp = -0.5 * std::log(std::numeric_limits<HP>::max());                                  \
        else                                                                                       \
            cp = -0.5 * std::log(determinant);                                                     \
        T ct = -(long)n / 2.0 * std::log(2 * M_PI);                                                \
        T v = df + (T)(cp + ct);                                                                   \
        if (std::isinf(v))                                                                         \
            throw std::string("GaussianLogLikelihood::GetValueAndParameterDerivatives: likelihood is infinite."); \
        *value = v;                                                                                \
        if (grad) {                                                                                \
            const int P = k->nparams();                                                            \
            std::vector<T> D((size_t)P * n * n);                                                   \
            deriv_matrix(*k, X, n, d, D.data());                                                   \
            for (int p = 0; p < P; p++) {                                                          \
                const T* Dp = D.data() + (size_t)p * n * n;                                        \
                T tr = 0;                                                                          \
                _Pragma("omp parallel for reduction(+ : tr) schedule(static)") for (int i = 0;     \
                                                                                     i < n; i++) { \
                    T row = 0;                                                                     \
                    for (int j = 0; j < n; j++)                                                    \
                        row += (alpha[i] * alpha[j] - C[(size_t)i * n + j]) * Dp[(size_t)i * n + j]; /* D_p symmetric */ \
                    tr += row;                                                                     \
                }                                                                                  \
                grad[p] = 0.5 * tr;                                                                \
            }                                                                                      \
        }                                                                                          \
        ORC_CATCH                                                                                  \
    }                                                                                              \
    /* SparseGaussianProcess::PreComputeRegression (include/SparseGaussianProcess.h:274-313) */    \
    /* without the N x N core matrix.  Outputs: Kinv (M x M), RV (M x m), RM (M x M). */           \
    int orc_sparse_fit_##SUF(const char* ks, const T* X, const T* Y, int n, int d, int m,          \
                             const T* Xm, int M, T sigma, T jitter, T* Kinv, T* RV, T* RM) {       \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        if (!(M <= n))                                                                             \
            throw std::string("SparseGaussianProcess::ComputeKernelVectorMatrix: number of dense samples must be higher than the number of sparse samples"); \
        bool stable = (jitter < std::numeric_limits<T>::min()) ? true : false;                     \
        std::vector<T> K((size_t)M * M);                                                           \
        kernel_matrix(*k, Xm, M, d, K.data());                                                     \
        for (int i = 0; i < M; i++) K[(size_t)i * M + i] += jitter;                                \
        std::vector<T> Ki = invert<T>(K, M, FullPivotLU, stable);                                  \
        std::vector<T> Knm((size_t)n * M);                                                         \
        _Pragma("omp parallel for schedule(static)") for (int i = 0; i < n; i++) for (int j = 0;   \
                                                                                    j < M; j++)    \
            Knm[(size_t)i * M + j] = keval(*k, X + (size_t)i * d, Xm + (size_t)j * d, d);          \
        T is2 = 1.0 / (sigma * sigma);                                                             \
        /* S = K + is2 Knm^T Knm (:298-299); Knm row-major n x M is column-major Knm^T */         \
        std::vector<T> S((size_t)M * M), KtY((size_t)M * m);                                       \
        if (!blas_gemm('N', 'T', M, M, n, T(1), Knm.data(), M, Knm.data(), M, T(0), S.data(), M)) { \
            _Pragma("omp parallel for schedule(static)") for (int a = 0; a < M; a++) for (int b = 0; \
                                                                                    b < M; b++) {  \
                T s = 0;                                                                           \
                for (int i = 0; i < n; i++) s += Knm[(size_t)i * M + a] * Knm[(size_t)i * M + b];  \
                S[(size_t)a * M + b] = s;                                                          \
            }                                                                                      \
        }                                                                                          \
        for (size_t e = 0; e < S.size(); e++) S[e] = K[e] + is2 * S[e];                            \
        std::vector<T> Sig = invert<T>(S, M, FullPivotLU, stable);                                 \
        /* Knm^T Y (:303): column-major (Knm^T Y)^T = Y^T Knm */                                   \
        if (!blas_gemm('N', 'T', m, M, n, T(1), Y, m, Knm.data(), M, T(0), KtY.data(), m)) {       \
            for (int a = 0; a < M; a++)                                                            \
                for (int c = 0; c < m; c++) {                                                      \
                    T s = 0;                                                                       \
                    for (int i = 0; i < n; i++) s += Knm[(size_t)i * M + a] * Y[(size_t)i * m + c]; \
                    KtY[(size_t)a * m + c] = s;                                                    \
                }                                                                                  \
        } /* column-major m x M (ld m) is the row-major M x m layout */                             \
        std::vector<T> A((size_t)M * M), B((size_t)M * M), t1((size_t)M * m), t2((size_t)M * m);   \
        gemm(K.data(), Sig.data(), A.data(), M, M, M);                                             \
        gemm(A.data(), KtY.data(), t1.data(), M, M, m);                                            \
        for (auto& v : t1) v = is2 * v;                                                            \
        gemm(Ki.data(), t1.data(), RV, M, M, m);                                                   \
        gemm(A.data(), K.data(), B.data(), M, M, M);                                               \
        gemm(Ki.data(), B.data(), A.data(), M, M, M);                                              \
        gemm(A.data(), Ki.data(), RM, M, M, M);                                                    \
        std::copy(Ki.begin(), Ki.end(), Kinv);                                                     \
        ORC_CATCH                                                                                  \
    }

#define ORC_DEFINE_SPARSE_LML(SUF, T)                                                              \
    int orc_sparse_lml_##SUF(const char* ks, const T* X, const T* Y, int n, int d, const T* Xm, int M, \
                             T sigma, T jitter, T* value, T* grad, double* det_out, double* logdet_out) { \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        sparse_lml(*k, X, Y, n, d, Xm, M, sigma, jitter, value, grad, det_out, logdet_out);        \
        ORC_CATCH                                                                                  \
    }
ORC_DEFINE_SPARSE_LML(f64, double)
ORC_DEFINE_SPARSE_LML(f32, float)

/* SparseLikelihood::GetCoreMatrices + EfficientInversion + EfficientDeterminant (the quantities
   tests/SparseInferenceTest.cpp:37-224 checks): K = Kmm + jitter I (M x M), Kinv (M x M), Knm
   (n x M), Cinv = the Woodbury inverse of sigma^2 I + Knm Kinv Knm^T (n x n), det_eff = the
   long-double |Kinv| |sigma^2 I| |K + Knm^T Knm / sigma^2| (include/SparseLikelihood.h:138-145;
   |B| made finite as there), narrowed to double.  Any output pointer may be NULL. */
#define ORC_DEFINE_SPARSE_CORE(SUF, T)                                                             \
    int orc_sparse_core_##SUF(const char* ks, const T* X, int n, int d, const T* Xm, int M, T sigma, T jitter, \
                              T* K, T* Kinv, T* Knm, T* Cinv, double* det_eff) {                   \
        ORC_TRY auto k = kernel_from<T>(ks);                                                       \
        SparseCore<T> c = sparse_core(*k, X, n, d, Xm, M, sigma, jitter);                           \
        if (K) std::copy(c.K.begin(), c.K.end(), K);                                               \
        if (Kinv) std::copy(c.Kinv.begin(), c.Kinv.end(), Kinv);                                   \
        if (Knm) std::copy(c.Knm.begin(), c.Knm.end(), Knm);                                       \
        if (Cinv) std::copy(c.Cinv.begin(), c.Cinv.end(), Cinv);                                   \
        if (det_eff) {                                                                             \
            typedef long double HP;                                                                \
            HP det_B = det_long_double(c.Kinv, M);                                                 \
            if (std::isinf(det_B)) det_B = std::numeric_limits<HP>::max();                         \
            HP prodA = 1;                                                                          \
            for (int i = 0; i < n; i++) prodA *= (HP)c.s2;                                         \
            *det_eff = (double)(det_B * prodA * det_long_double(c.inner, M));                      \
        }                                                                                          \
        ORC_CATCH                                                                                  \
    }
ORC_DEFINE_SPARSE_CORE(f64, double)
ORC_DEFINE_SPARSE_CORE(f32, float)

ORC_DEFINE(f64, double)
ORC_DEFINE(f32, float)

}  // extern "C"
