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
// feature vectors plus per-sample constants, so a 128 x 128 block of pair statistics is a
// 128 x 128 x K MFMA tile (k_mma.h) instead of O(d) VALU work per pair:
//     r2 = |x~|^2 + |y~|^2 + x~ . (-2 y~)                                   (K = d)
//     S  = d/2 - 1/2 [C_x, S_x] . [C_y, S_y]                                (K = 2 d)
// (sin^2 u = (1 - cos 2u) / 2 and cos(2b(x - y)) = C_x C_y + S_x S_y) with x~ = x - x_0
// (both sets centred on the first training sample: r2 and S are translation invariant, and
// centring keeps |x~|^2 ~ r2 so the expansion loses no significant digits), C = cos(2b x~_k),
// S = sin(2b x~_k).  Feature matrices are column-major (rows padded to 128, columns to 16) so
// the tile kernel streams them with LDS-DMA like any GEMM operand; the squared norms sit in
// one more column after the MFMA operands and are added in the epilogue.
#include "k_pairs.h"

namespace gprx {

namespace pr {

// F (np x (Kr + Kp + 1), column-major, ld np): the left (U) or right (V) features of n
// samples, then their squared norms |x~|^2.  Padding rows are all zero.
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
        for (int k = d; k < Kr; k++) F[i + (int64_t)k * np] = 0;
    }
    F[i + (int64_t)(Kr + Kp) * np] = nrm;
    if (nper) {
        T* P = F + (int64_t)Kr * np;
        const T b2 = T(2) * b;
        for (int k = 0; k < d; k++) {
            T sn = 0, cs = 0;
            if (live) gsincos(b2 * (X[i * d + k] - center[k]), &sn, &cs);
            P[i + (int64_t)k * np] = cs;
            P[i + (int64_t)(d + k) * np] = sn;
        }
        for (int k = 2 * d; k < Kp; k++) P[i + (int64_t)k * np] = 0;
    }
}

// Lower triangle of K(X, X) (+ sigma2 on the diagonal, identity padding) into A (column-major).
template <typename T, int NPER, bool R2>
__global__ __launch_bounds__(NT) void kbuild_mma_kernel(const KCanon<T>* __restrict__ Kd, const T* __restrict__ FU,
                                                        const T* __restrict__ FV,
                                                        int64_t nf, int Kr, int Kp, T hd, T* __restrict__ A,
                                                        int64_t ld, int64_t n, T sigma2, int* __restrict__ flag) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* smem = reinterpret_cast<T*>(smem_raw);
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
    const bool bad = build_tile<T, NPER, R2>(Kd, FU, FV, nf, Kr, Kp, hd, A, ld, n, sigma2, ti * GT, tj * GT, smem,
                                                    threadIdx.x);
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
                                                         const T* __restrict__ FV, int64_t nfv, int Kr, int Kp, T hd,
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
    T nu[4];
#pragma unroll
    for (int y = 0; y < 4; y++) nu[y] = R2 ? FU[(int64_t)(Kr + Kp) * nfu + i0 + wr * 64 + y * 16 + lr] : T(0);
    // column norms of the current block go through LDS (after the staging ring): held in
    // registers across the two tile products they made this kernel spill
    T* nvs = smem + gemm_lds<T>() / sizeof(T);
    T* als = nvs + GT;
    for (int64_t j0 = 0; j0 < n; j0 += GT) {
        // column norms and alpha of the current block go through LDS (after the staging ring;
        // written here, read after tile_mma's barriers): held in registers across the two
        // tile products they made this kernel spill.  alpha = 0 masks the padding columns.
        if (t < GT) {
            if (R2) nvs[t] = FV[(int64_t)(Kr + Kp) * nfv + j0 + t];
            als[t] = (j0 + t < n) ? alpha[(j0 + t) * m] : T(0);
        }
        typename Tr::acc_t ar[2][4], ap[2][4];
        // opaque thread index: the query-side operand addresses are loop-invariant, and
        // hoisted out of this loop they stayed live in registers across it (spills)
        int tid = t;
        asm volatile("" : "+v"(tid));
        block_stats<T, NPER, R2>(FU, nfu, i0, FV, nfv, j0, Kr, Kp, smem, tid, ar, ap);
        auto chunk = [&](auto cc) {  // 4 pairs per thread at a time: column (x, reg), rows y
            constexpr int x = decltype(cc)::value >> 2, reg = decltype(cc)::value & 3;
            const int jl = wc * 32 + x * 16 + Tr::orow(lk, reg);
            T r2[4], sp[4], v[4];
#pragma unroll
            for (int y = 0; y < 4; y++)
                pair_stats<T, NPER, R2>(R2 ? ar[x][y][reg] : T(0), NPER ? ap[x][y][reg] : T(0), nu[y],
                                        R2 ? nvs[jl] : T(0), hd, r2[y], sp[y]);
            pair_values<T, 4>(Kd, r2, sp, v);
            const T al = als[jl];
#pragma unroll
            for (int y = 0; y < 4; y++) racc[0][y] = fma(v[y], al, racc[0][y]);
        };
        chunk(std::integral_constant<int, 0>{});
        chunk(std::integral_constant<int, 1>{});
        chunk(std::integral_constant<int, 2>{});
        chunk(std::integral_constant<int, 3>{});
        chunk(std::integral_constant<int, 4>{});
        chunk(std::integral_constant<int, 5>{});
        chunk(std::integral_constant<int, 6>{});
        chunk(std::integral_constant<int, 7>{});
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

// feature columns of one sample set (Kr + Kp operand columns + the squared norms)
template <typename T>
int64_t pairs_feature_cols(const KCanon<T>& K, int d) {
    return pr::kr_of(K, d) + pr::kp_of(K, d) + 1;
}

template <typename T>
void launch_pair_features(const KCanon<T>& K, const T* X, int64_t n, int d, const T* center, bool right, T* F,
                          int64_t np, hipStream_t s) {
    const int Kr = pr::kr_of(K, d), Kp = pr::kp_of(K, d);
    hipLaunchKernelGGL(pr::features_kernel<T>, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, X, n, d, center,
                       K.nper ? K.b[0] : T(0), K.need_r2 ? 1 : 0, K.nper, right ? 1 : 0, F, np, Kr, Kp);
}

template <typename T>
static size_t pairs_lds() {
    const size_t a = mm::gemm_lds<T>() + sizeof(T) * 2 * GT, b = sizeof(T) * 4 * GT * pr::PM;  // + norms, alpha
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
    const int Kr = pr::kr_of(K, d), Kp = pr::kp_of(K, d);
    const int64_t nt = nf / GT;
    const dim3 grid((unsigned)(nt * (nt + 1) / 2));
    ProfScope ps(KC_BUILD, s, 2.0 * (double)GT * GT * (Kr + Kp) * nt * (nt + 1) / 2,
                 (double)sizeof(T) * (n * (double)d + (double)n * (n + 1) / 2));
    GPRX_PAIRS_DISPATCH(kbuild_mma_kernel, Kd, FU, FV, nf, Kr, Kp, T(0.5) * T(d), A, ld, n, sigma2, flag);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void launch_predict_mma(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, int64_t nfu, const T* FV, int64_t nfv,
                        int d, const T* alpha, int64_t n, int m, int64_t q, T* mean, hipStream_t s) {
    const int Kr = pr::kr_of(K, d), Kp = pr::kp_of(K, d);
    const dim3 grid((unsigned)(nfu / GT));
    ProfScope ps(KC_PREDICT, s, (double)q * n * (2.0 * d + 2.0 * m), (double)sizeof(T) * (double)(q + n) * d);
    GPRX_PAIRS_DISPATCH(predict_mma_kernel, Kd, FU, nfu, FV, nfv, Kr, Kp, T(0.5) * T(d), alpha, n, m, q, mean);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
TileBuild<T> pairs_tile_build(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, const T* FV, int64_t nf, int d,
                              int64_t n, T sigma2, int* flag) {
    TileBuild<T> b;
    b.Kd = Kd;
    b.FU = FU;
    b.FV = FV;
    b.nf = nf;
    b.Kr = pr::kr_of(K, d);
    b.Kp = pr::kp_of(K, d);
    b.hd = T(0.5) * T(d);
    b.sigma2 = sigma2;
    b.n = n;
    b.flag = flag;
    // as GPRX_PAIRS_DISPATCH.  0 (no fused build: the caller launches kbuild_mma_kernel) for
    // trees with products, which build_tile_sum does not separate, and for RationalQuadratic
    // leaves: the fused path carries exp-form leaves only, to keep the factorisation kernel
    // small (its code and register budget are shared with every other task type)
    bool expform = K.sum_leaves != 0;
    for (int l = 0; l < K.nleaf; l++)
        if (K.leaf[l].type != L_GAUSS && K.leaf[l].type != L_GAUSS_EXP && K.leaf[l].type != L_PERIODIC) expform = false;
    b.mode = !expform ? 0 : (K.nper && K.need_r2) ? 1 : (K.nper ? 3 : 2);
    return b;
}

#define GPRX_PAIRS_INST(T)                                                                                    \
    template TileBuild<T> pairs_tile_build<T>(const KCanon<T>&, const KCanon<T>*, const T*, const T*, int64_t, int, \
                                              int64_t, T, int*);                                              \
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
