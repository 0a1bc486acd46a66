// k_syrk.hip — split-K rank-k accumulation C_p += alpha A_p A_p^T on the tile mainloop of
// k_mma.h (LDS-DMA operand ring, 8 waves, v_mfma_f64_16x16x4f64 / f32).
//
// The sparse fit's normal equations sigma^-2 [Kmn; Y^T][Kmn; Y^T]^T accumulated over the
// streamed dense-row chunks (include/SparseGaussianProcess.h:274-313: Knm^T Knm and Knm^T Y).
// A is (ld rows x K*P columns, column-major); partial p multiplies columns [pK, (p+1)K) into
// C + p*cstride.  Tiles: the lower triangle of the ntn x ntn leading block, then the full
// rows below it (the label rows).  One workgroup per CU (the ring takes 139 KB of LDS).
#include "k_mma.h"

#include <cstdint>
#include <cstdlib>
#include <type_traits>

namespace gprx {
namespace sy {

template <typename T>
__global__ __launch_bounds__(mm::NT) void syrk_splitk_kernel(T* __restrict__ C, int64_t ldc, int64_t cstride,
                                                             const T* __restrict__ A, int64_t lda, int K, int64_t ntn,
                                                             T alpha) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* smem = reinterpret_cast<T*>(smem_raw);
    const int64_t p = blockIdx.y;
    A += p * (int64_t)K * lda;
    C += p * cstride;
    int64_t ti, tj;
    {
        const int64_t b = blockIdx.x, tri = ntn * (ntn + 1) / 2;
        if (b < tri) {
            int64_t i = (int64_t)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
            while ((i + 1) * (i + 2) / 2 <= b) i++;
            while (i * (i + 1) / 2 > b) i--;
            ti = i;
            tj = b - i * (i + 1) / 2;
        } else {
            ti = ntn + (b - tri) / ntn;
            tj = (b - tri) % ntn;
        }
    }
    const int64_t i0 = ti * GT, j0 = tj * GT;
    typedef mm::Mfma<T> Tr;
    typename Tr::acc_t acc[2][4];
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    const int lr = lane & 15, lk = lane >> 4;
    const bool diag = ti == tj;
    int wr, wc;
    // (K: multiples of 16) a diagonal tile skips its 16 x 16 tiles above the diagonal, waves
    // mapped so each SIMD's pair carries the same number of live tiles (k_mma.h wave_block<2>):
    // the 16 diagonal tiles of M = 2048 are 12% of the launch's tiles
    if (diag) {
        mm::tile_mma<T, 2, false, mm::BKS>(acc, A + i0, lda, A + j0, lda, K, K, smem, t);
        mm::wave_block<2>(w, wr, wc);
    } else {
        mm::tile_mma<T, 0, false, mm::BKS>(acc, A + i0, lda, A + j0, lda, K, K, smem, t);
        mm::wave_block<0>(w, wr, wc);
    }
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int reg = 0; reg < 4; reg++) {
            const int64_t gj = j0 + wc * 32 + x * 16 + Tr::orow(lk, reg);
            T* col = C + gj * ldc;
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const int64_t gi = i0 + wr * 64 + y * 16 + lr;
                if (diag && gi < gj) continue;
                col[gi] = fma(alpha, acc[x][y][reg], col[gi]);
            }
        }
}

// C (M x N, ldc) = alpha A B^T + beta C on 256 x 128 tiles (k_mma.h tile_mma_tall): the
// stand-alone f64 GEMMs of the posterior variance's recursive solves (launch_gemm_nt); A: M x K,
// B: N x K, column-major
template <typename T, bool BETA>
__global__ __launch_bounds__(mm::NT) void gemm_tall_kernel(T* __restrict__ C, int64_t ldc, const T* __restrict__ A,
                                                           int64_t lda, const T* __restrict__ B, int64_t ldb, int K,
                                                           T alpha, T beta, int64_t ntm) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* smem = reinterpret_cast<T*>(smem_raw);
    const int64_t ti = blockIdx.x % ntm, tj = blockIdx.x / ntm;
    const int64_t i0 = ti * 2 * GT, j0 = tj * GT;
    typedef mm::Mfma<T> Tr;
    typename Tr::acc_t acc[4][4];
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    const int lr = lane & 15, lk = lane >> 4, wr = w & 3, wc = w >> 2;
    mm::tile_mma_tall<T>(acc, A + i0, lda, B + j0, ldb, K, smem, t);
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int reg = 0; reg < 4; reg++) {
            T* col = C + (j0 + wc * 64 + x * 16 + Tr::orow(lk, reg)) * ldc + i0 + wr * 64 + lr;
#pragma unroll
            for (int y = 0; y < 4; y++) {
                T v = alpha * acc[x][y][reg];
                if (BETA) v = fma(beta, col[y * 16], v);
                col[y * 16] = v;
            }
        }
}

}  // namespace sy

// the tall-tile GEMM when its shape applies (f64, M a multiple of 256, N of 128, K of the stage
// depth, 16-byte aligned columns); false: the caller takes its own path
template <typename T>
bool launch_gemm_tall(T* C, int64_t ldc, const T* A, int64_t lda, const T* B, int64_t ldb, int64_t M, int64_t N,
                      int64_t K, T alpha, T beta, hipStream_t s) {
    static const bool off = [] {
        const char* e = std::getenv("GPRX_GEMM_TALL");
        return e && e[0] == '0';
    }();
    if (off || !std::is_same<T, double>::value || M <= 0 || N <= 0 || K <= 0) return false;
    if (M % (2 * GT) || N % GT || K % mm::BkOf<T>::v || lda % 2 || ldb % 2 || K > INT32_MAX) return false;
    if (((uintptr_t)A | (uintptr_t)B) % 16) return false;
    const int64_t ntm = M / (2 * GT), ntiles = ntm * (N / GT);
    const size_t lds = mm::tall_lds<T>();
    const bool use_beta = beta != T(0);
    auto go = [&](auto kfn) {
        GPRX_HIP(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(kfn, dim3((unsigned)ntiles), dim3(mm::NT), lds, s, C, ldc, A, lda, B, ldb, (int)K, alpha,
                           beta, ntm);
    };
    if (use_beta) go(sy::gemm_tall_kernel<T, true>);
    else go(sy::gemm_tall_kernel<T, false>);
    GPRX_HIP(hipGetLastError());
    return true;
}
template bool launch_gemm_tall<double>(double*, int64_t, const double*, int64_t, const double*, int64_t, int64_t,
                                       int64_t, int64_t, double, double, hipStream_t);
template bool launch_gemm_tall<float>(float*, int64_t, const float*, int64_t, const float*, int64_t, int64_t, int64_t,
                                      int64_t, float, float, hipStream_t);

// C_p (lower, M x N: M = rows of A incl. the rows below the N x N block) += alpha A_p A_p^T,
// p < P, K (multiple of 16) columns per partial.
template <typename T>
void launch_syrk_splitk(T* C, int64_t ldc, int64_t cstride, const T* A, int64_t lda, int64_t M, int64_t N, int64_t K,
                        int P, T alpha, hipStream_t s) {
    if (M <= 0 || N <= 0 || K <= 0 || P <= 0) return;
    GPRX_REQUIRE(M % GT == 0 && N % GT == 0 && K % mm::BKS == 0 && lda % 2 == 0 && K <= INT32_MAX, GPRX_ERR_ARG,
                 "launch_syrk_splitk: tile-aligned operands required");
    const int64_t ntm = M / GT, ntn = N / GT;
    const int64_t ntiles = ntn * (ntn + 1) / 2 + (ntm - ntn) * ntn;
    const double elems = (double)N * (N + 1) / 2 + (double)(M - N) * N;
    ProfScope ps(KC_OTHER, s, 2.0 * elems * K * P, (double)sizeof(T) * (2 * elems * P + (double)M * K * P));
    const size_t lds = mm::gemm_lds<T>();
    static bool attr_done = false;
    if (!attr_done) {
        GPRX_HIP(hipFuncSetAttribute((const void*)sy::syrk_splitk_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
        attr_done = true;
    }
    hipLaunchKernelGGL(sy::syrk_splitk_kernel<T>, dim3((unsigned)ntiles, (unsigned)P), dim3(mm::NT), lds, s, C, ldc,
                       cstride, A, lda, (int)K, ntn, alpha);
    GPRX_HIP(hipGetLastError());
}

template void launch_syrk_splitk<double>(double*, int64_t, int64_t, const double*, int64_t, int64_t, int64_t, int64_t,
                                         int, double, hipStream_t);
template void launch_syrk_splitk<float>(float*, int64_t, int64_t, const float*, int64_t, int64_t, int64_t, int64_t,
                                        int, float, hipStream_t);

}  // namespace gprx
