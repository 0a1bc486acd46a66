// k_pairs.hip — pair statistics of the covariance on the MFMA units (gfx950).
//
// Replaces the same reference loops as k_build.hip / k_predict.hip -- the OpenMP pair loop of
// GaussianProcess::ComputeKernelMatrixInternal (lib/GaussianProcess.cpp:384-402) with
// AddNoiseToKernelMatrix (:375-381), and the per-query kernel vector of Predict
// (lib/GaussianProcess.cpp:54-61, 684-693) -- for kernel trees whose leaves are Gaussian,
// GaussianExp, RationalQuadratic and at most one Periodic frequency (no White leaf, which
// needs the exact test r2 == 0, include/Kernel.h:696).
//
// Every leaf depends on a pair only through r2 = sum_k (x_k - y_k)^2 and
// S = sum_k sin^2(b (x_k - y_k)) (gprx_internal.h).  Both are inner products of per-sample
// feature vectors, so a 128 x 128 block of pair statistics is a 128 x 128 x K MFMA tile
// (k_mma.h) instead of O(d) VALU work per pair:
//     r2 = [x~, |x~|^2, 1] . [-2 y~, 1, |y~|^2]                           (K = d + 2)
//     S  = [s_x^2, c_x^2, s_x c_x] . [c_y^2, s_y^2, -2 s_y c_y]            (K = 3 d)
// with x~ = x - x_0 (both sets centred on the first training sample: r2 and S are translation
// invariant, and centring keeps |x~|^2 ~ r2 so the expansion loses no significant digits),
// s = sin(b x~_k), c = cos(b x~_k).  Feature matrices are column-major (rows padded to 128,
// columns to 16) so the tile kernel streams them with LDS-DMA like any GEMM operand.
#include "gprx_internal.h"
#include "k_mma.h"

#include <type_traits>

namespace gprx {

namespace pr {

using namespace mm;

constexpr int KG = 16;  // feature-column granule (the tile kernel's k-stage)

static int64_t rup(int64_t x, int64_t g) { return (x + g - 1) / g * g; }

// F (np x (Kr + Kp), column-major, ld np): the left (U) or right (V) features of n samples.
template <typename T>
__global__ void features_kernel(const T* __restrict__ X, int64_t n, int d, const T* __restrict__ center, T b,
                                int need_r2, int nper, int right, T* __restrict__ F, int64_t np, int Kr, int Kp) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    const bool live = i < n;
    T nrm = 0;
    if (need_r2) {
        for (int k = 0; k < d; k++) {
            const T xt = live ? X[i * d + k] - center[k] : T(0);
            nrm = fma(xt, xt, nrm);
            F[i + (int64_t)k * np] = right ? T(-2) * xt : xt;
        }
        F[i + (int64_t)d * np] = right ? T(1) : nrm;
        F[i + (int64_t)(d + 1) * np] = right ? nrm : T(1);
        if (!live) {  // padding rows: all-zero statistics
            F[i + (int64_t)d * np] = 0;
            F[i + (int64_t)(d + 1) * np] = 0;
        }
        for (int k = d + 2; k < Kr; k++) F[i + (int64_t)k * np] = 0;
    }
    if (nper) {
        T* P = F + (int64_t)Kr * np;
        for (int k = 0; k < d; k++) {
            T sn = 0, cs = 0;
            if (live) gsincos(b * (X[i * d + k] - center[k]), &sn, &cs);
            P[i + (int64_t)k * np] = right ? cs * cs : sn * sn;
            P[i + (int64_t)(d + k) * np] = right ? sn * sn : cs * cs;
            P[i + (int64_t)(2 * d + k) * np] = right ? T(-2) * sn * cs : sn * cs;
        }
        for (int k = 3 * d; k < Kp; k++) P[i + (int64_t)k * np] = 0;
    }
}

// Kernel values of E pairs from their (r2, S) for the trees this file accepts (no White
// leaf, one periodic table).  Same formulas and products/sums as kernel_value/leaf_value
// (0 + x and 1 * x are exact, so the results are bit-identical), but organised leaf-outer:
// the loops over leaves and terms are wave-uniform (leaf constants come in through scalar
// loads, the type test is a uniform branch) and the per-pair work is an unrolled,
// statically indexed loop over E registers.  The generic kernel_value reached from 32
// unrolled call sites per thread was emitted as an out-of-line call per pair.
template <typename T, int E, bool MUL>
__device__ __forceinline__ void leaf_into(const KLeaf<T>* __restrict__ L, const T (&r2)[E], const T (&s)[E],
                                          T (&p)[E]) {
    const int ty = L->type;
    const T c0 = L->c0, c1 = L->c1, c2 = L->c2;
    if (ty == L_PERIODIC) {
#pragma unroll
        for (int e = 0; e < E; e++) {
            const T f = c0 * exp(c1 * s[e]);
            p[e] = MUL ? p[e] * f : p[e] + f;
        }
    } else if (ty == L_RQ) {
#pragma unroll
        for (int e = 0; e < E; e++) {
            const T f = c0 * exp(-c2 * log1p(c1 * r2[e]));
            p[e] = MUL ? p[e] * f : p[e] + f;
        }
    } else {  // L_GAUSS, L_GAUSS_EXP
#pragma unroll
        for (int e = 0; e < E; e++) {
            const T f = c0 * exp(c1 * r2[e]);
            p[e] = MUL ? p[e] * f : p[e] + f;
        }
    }
}

template <typename T, int E>
__device__ __forceinline__ void pair_values(const KCanon<T>* __restrict__ K, const T (&r2)[E], const T (&s)[E],
                                            T (&v)[E]) {
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = 0;
    const int nl = K->nleaf;
    if (K->sum_leaves) {
#pragma unroll 1
        for (int l = 0; l < nl; l++) leaf_into<T, E, false>(&K->leaf[l], r2, s, v);
        return;
    }
    const int nt = K->nterm;
#pragma unroll 1
    for (int t = 0; t < nt; t++) {
        const unsigned msk = K->term_mask[t];
        T p[E];
#pragma unroll
        for (int e = 0; e < E; e++) p[e] = 1;
#pragma unroll 1
        for (int l = 0; l < nl; l++)
            if (msk & (1u << l)) leaf_into<T, E, true>(&K->leaf[l], r2, s, p);
#pragma unroll
        for (int e = 0; e < E; e++) v[e] += p[e];
    }
}

// Statistics of the 128 x 128 pair block (rows from FU + i0, columns from FV + j0).
template <typename T, int NPER, bool R2>
__device__ __forceinline__ void block_stats(const T* FU, int64_t nu, int64_t i0, const T* FV, int64_t nv, int64_t j0,
                                            int Kr, int Kp, T* smem, int t, typename Mfma<T>::acc_t (&ar)[2][4],
                                            typename Mfma<T>::acc_t (&ap)[2][4]) {
    if (R2) tile_mma<T>(ar, FU + i0, nu, FV + j0, nv, Kr, true, smem, t);
    if (NPER) {
        __syncthreads();  // the second product reuses the staging ring
        tile_mma<T>(ap, FU + (int64_t)Kr * nu + i0, nu, FV + (int64_t)Kr * nv + j0, nv, Kp, true, smem, t);
    }
}

// Lower triangle of K(X, X) (+ sigma2 on the diagonal, identity padding) into A (column-major).
template <typename T, int NPER, bool R2>
__global__ __launch_bounds__(NT) void kbuild_mma_kernel(const KCanon<T>* __restrict__ Kd, const T* __restrict__ FU,
                                                        const T* __restrict__ FV,
                                                        int64_t nf, int Kr, int Kp, T* __restrict__ A, int64_t ld,
                                                        int64_t n, T sigma2, int* __restrict__ flag) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* smem = reinterpret_cast<T*>(smem_raw);
    typedef Mfma<T> Tr;
    // the kernel tree is read from device memory (scalar loads): as a by-value kernel
    // argument indexed per leaf/term, hipcc copied it to scratch
    int64_t ti, tj;
    {
        const int64_t b = blockIdx.x;
        int64_t i = (int64_t)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
        while ((i + 1) * (i + 2) / 2 <= b) i++;
        while (i * (i + 1) / 2 > b) i--;
        ti = i;
        tj = b - i * (i + 1) / 2;
    }
    const int64_t i0 = ti * GT, j0 = tj * GT;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w & 1, wc = w >> 1, lr = lane & 15, lk = lane >> 4;
    typename Tr::acc_t ar[2][4], ap[2][4];
    block_stats<T, NPER, R2>(FU, nf, i0, FV, nf, j0, Kr, Kp, smem, t, ar, ap);
    bool bad = false;
    // four chunks of 8 pairs per thread (column group x, registers 2h, 2h+1):
    // statistics -> values -> stores; 8 keeps the interleaved exp sequences within registers
    auto chunk = [&](auto cc) {
        constexpr int x = decltype(cc)::value >> 1, h = decltype(cc)::value & 1;
        T r2[8], sp[8], v[8];
#pragma unroll
        for (int reg = 2 * h; reg < 2 * h + 2; reg++)
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const int64_t gj = j0 + wc * 32 + x * 16 + Tr::orow(lk, reg);
                const int64_t gi = i0 + wr * 64 + y * 16 + lr;
                r2[(reg - 2 * h) * 4 + y] = R2 ? (gi == gj ? T(0) : fmax(ar[x][y][reg], T(0))) : T(0);
                sp[(reg - 2 * h) * 4 + y] = NPER ? (gi == gj ? T(0) : fmax(ap[x][y][reg], T(0))) : T(0);
            }
        pair_values<T, 8>(Kd, r2, sp, v);
#pragma unroll
        for (int reg = 2 * h; reg < 2 * h + 2; reg++) {
            const int64_t gj = j0 + wc * 32 + x * 16 + Tr::orow(lk, reg);
            T* col = A + gj * ld;
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const int64_t gi = i0 + wr * 64 + y * 16 + lr;
                T val = v[(reg - 2 * h) * 4 + y];
                if (gi >= n || gj >= n) {
                    val = (gi == gj) ? T(1) : T(0);
                } else {
                    if (!isfinite(val)) bad = true;
                    if (gi == gj) val += sigma2;
                }
                if (gi >= gj) col[gi] = val;
            }
        }
    };
    chunk(std::integral_constant<int, 0>{});
    chunk(std::integral_constant<int, 1>{});
    chunk(std::integral_constant<int, 2>{});
    chunk(std::integral_constant<int, 3>{});
    if (bad) atomicOr(flag, 1);
}

// mean[q][r] = sum_j k(xq_q, x_j) alpha[j][r], r < m <= PM, one workgroup per 128 queries
// streaming the training set in 128-point blocks; K(Xq, X) is never materialised.  (PM = 1:
// more outputs per query would spill next to the two accumulator sets; they take the direct
// kernel of k_predict.hip.)
constexpr int PM = 1;
template <typename T, int NPER, bool R2>
__global__ __launch_bounds__(NT) void predict_mma_kernel(const KCanon<T>* __restrict__ Kd, const T* __restrict__ FU,
                                                         int64_t nfu,
                                                         const T* __restrict__ FV, int64_t nfv, int Kr, int Kp,
                                                         const T* __restrict__ alpha, int64_t n, int m, int64_t q,
                                                         T* __restrict__ mean) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* smem = reinterpret_cast<T*>(smem_raw);
    typedef Mfma<T> Tr;
    const int64_t i0 = (int64_t)blockIdx.x * GT;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w & 1, wc = w >> 1, lr = lane & 15, lk = lane >> 4;
    T racc[PM][4];
#pragma unroll
    for (int r = 0; r < PM; r++)
#pragma unroll
        for (int y = 0; y < 4; y++) racc[r][y] = 0;
    for (int64_t j0 = 0; j0 < n; j0 += GT) {
        typename Tr::acc_t ar[2][4], ap[2][4];
        block_stats<T, NPER, R2>(FU, nfu, i0, FV, nfv, j0, Kr, Kp, smem, t, ar, ap);
        auto chunk = [&](auto cc) {  // 8 pairs per thread at a time, as in kbuild_mma_kernel
            constexpr int x = decltype(cc)::value >> 1, h = decltype(cc)::value & 1;
            T r2[8], sp[8], v[8];
#pragma unroll
            for (int e = 0; e < 8; e++) {
                r2[e] = R2 ? fmax(ar[x][e & 3][2 * h + (e >> 2)], T(0)) : T(0);
                sp[e] = NPER ? fmax(ap[x][e & 3][2 * h + (e >> 2)], T(0)) : T(0);
            }
            pair_values<T, 8>(Kd, r2, sp, v);
#pragma unroll
            for (int reg = 2 * h; reg < 2 * h + 2; reg++) {
                const int64_t gj = j0 + wc * 32 + x * 16 + Tr::orow(lk, reg);
                const bool okj = gj < n;
                T al[PM];
#pragma unroll
                for (int r = 0; r < PM; r++) al[r] = (okj && r < m) ? alpha[gj * m + r] : T(0);
#pragma unroll
                for (int y = 0; y < 4; y++) {
                    const T kv = okj ? v[(reg - 2 * h) * 4 + y] : T(0);
#pragma unroll
                    for (int r = 0; r < PM; r++) racc[r][y] = fma(kv, al[r], racc[r][y]);
                }
            }
        };
        chunk(std::integral_constant<int, 0>{});
        chunk(std::integral_constant<int, 1>{});
        chunk(std::integral_constant<int, 2>{});
        chunk(std::integral_constant<int, 3>{});
        __syncthreads();  // the staging ring is refilled by the next block's product
    }
    // rows 64 wr + 16 y + lr: sum over the lane groups lk, then over the 4 column waves (LDS)
    T* red = smem;  // [4 wc][128 rows][PM]
#pragma unroll
    for (int r = 0; r < PM; r++)
#pragma unroll
        for (int y = 0; y < 4; y++) {
            T v = racc[r][y];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lk == 0) red[(wc * GT + wr * 64 + y * 16 + lr) * PM + r] = v;
        }
    __syncthreads();
    if (t < GT * PM) {
        const int row = t / PM, r = t % PM;
        const int64_t gi = i0 + row;
        if (r < m && gi < q) {
            T s = 0;
#pragma unroll
            for (int c = 0; c < 4; c++) s += red[(c * GT + row) * PM + r];
            mean[gi * m + r] = s;
        }
    }
}

}  // namespace pr

template <typename T>
bool pairs_mma_supported(const KCanon<T>& K, int m) {
    if (K.nper > 1 || m > pr::PM) return false;
    for (int l = 0; l < K.nleaf; l++)
        if (K.leaf[l].type == L_WHITE) return false;
    return K.need_r2 || K.nper > 0;
}

// feature columns of one sample set (Kr + Kp), for the workspace size
template <typename T>
int64_t pairs_feature_cols(const KCanon<T>& K, int d) {
    return (K.need_r2 ? pr::rup(d + 2, pr::KG) : 0) + (K.nper ? pr::rup(3 * d, pr::KG) : 0);
}

template <typename T>
void launch_pair_features(const KCanon<T>& K, const T* X, int64_t n, int d, const T* center, bool right, T* F,
                          int64_t np, hipStream_t s) {
    const int Kr = K.need_r2 ? (int)pr::rup(d + 2, pr::KG) : 0, Kp = K.nper ? (int)pr::rup(3 * d, pr::KG) : 0;
    hipLaunchKernelGGL(pr::features_kernel<T>, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, X, n, d, center,
                       K.nper ? K.b[0] : T(0), K.need_r2 ? 1 : 0, K.nper, right ? 1 : 0, F, np, Kr, Kp);
}

template <typename T>
static size_t pairs_lds() {
    const size_t a = mm::gemm_lds<T>(), b = sizeof(T) * 4 * GT * pr::PM;
    return a > b ? a : b;
}

#define GPRX_PAIRS_DISPATCH(KERN, ...)                                                                  \
    do {                                                                                              \
        const size_t lds_ = pairs_lds<T>();                                                           \
        auto go = [&](auto kfn) {                                                                     \
            GPRX_HIP(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,     \
                                         (int)lds_));                                                \
            hipLaunchKernelGGL(kfn, grid, dim3(mm::NT), lds_, s, __VA_ARGS__);                        \
        };                                                                                            \
        if (K.nper && K.need_r2) go(pr::KERN<T, 1, true>);                                            \
        else if (K.nper) go(pr::KERN<T, 1, false>);                                                   \
        else go(pr::KERN<T, 0, true>);                                                                \
    } while (0)

// Lower triangle of K(X, X) + sigma2 I (identity beyond n) into A, from the features FU, FV
// (nf rows, nf = npad: a multiple of 128 >= n).
template <typename T>
void launch_kbuild_mma(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, const T* FV, int64_t nf, int d, T* A,
                       int64_t ld, int64_t n, T sigma2, int* flag, hipStream_t s) {
    const int Kr = K.need_r2 ? (int)pr::rup(d + 2, pr::KG) : 0, Kp = K.nper ? (int)pr::rup(3 * d, pr::KG) : 0;
    const int64_t nt = nf / GT;
    const dim3 grid((unsigned)(nt * (nt + 1) / 2));
    ProfScope ps(KC_BUILD, s, 2.0 * (double)GT * GT * (Kr + Kp) * nt * (nt + 1) / 2,
                 (double)sizeof(T) * (n * (double)d + (double)n * (n + 1) / 2));
    GPRX_PAIRS_DISPATCH(kbuild_mma_kernel, Kd, FU, FV, nf, Kr, Kp, A, ld, n, sigma2, flag);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void launch_predict_mma(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, int64_t nfu, const T* FV, int64_t nfv,
                        int d, const T* alpha, int64_t n, int m, int64_t q, T* mean, hipStream_t s) {
    const int Kr = K.need_r2 ? (int)pr::rup(d + 2, pr::KG) : 0, Kp = K.nper ? (int)pr::rup(3 * d, pr::KG) : 0;
    const dim3 grid((unsigned)(nfu / GT));
    ProfScope ps(KC_PREDICT, s, (double)q * n * (2.0 * d + 2.0 * m), (double)sizeof(T) * (double)(q + n) * d);
    GPRX_PAIRS_DISPATCH(predict_mma_kernel, Kd, FU, nfu, FV, nfv, Kr, Kp, alpha, n, m, q, mean);
    GPRX_HIP(hipGetLastError());
}

#define GPRX_PAIRS_INST(T)                                                                                    \
    template bool pairs_mma_supported<T>(const KCanon<T>&, int);                                              \
    template int64_t pairs_feature_cols<T>(const KCanon<T>&, int);                                            \
    template void launch_pair_features<T>(const KCanon<T>&, const T*, int64_t, int, const T*, bool, T*, int64_t, \
                                          hipStream_t);                                                       \
    template void launch_kbuild_mma<T>(const KCanon<T>&, const KCanon<T>*, const T*, const T*, int64_t, int, T*,    \
                                       int64_t, int64_t, T, int*, hipStream_t);                               \
    template void launch_predict_mma<T>(const KCanon<T>&, const KCanon<T>*, const T*, int64_t, const T*, int64_t, \
                                        int, const T*, int64_t, int, int64_t, T*, hipStream_t);
GPRX_PAIRS_INST(double)
GPRX_PAIRS_INST(float)
#undef GPRX_PAIRS_INST

}  // namespace gprx
