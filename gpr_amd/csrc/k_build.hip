// k_build.hip — covariance construction on gfx950.
//
// Replaces the OpenMP pair loop of GaussianProcess::ComputeKernelMatrixInternal
// (lib/GaussianProcess.cpp:384-402), AddNoiseToKernelMatrix (:375-381), the cross matrix of
// SparseGaussianProcess::ComputeKernelVectorMatrix (include/SparseGaussianProcess.h:218-235)
// and the derivative matrices of ComputeDerivativeKernelMatrixInternal
// (lib/GaussianProcess.cpp:472-495).
//
// kbuild: one 256-thread workgroup per 64x64 output tile; the 64 row samples and 64 column
// samples of a 16-dimension chunk are staged in LDS dimension-major (coalesced row-major
// global reads, conflict-free ds_read_b128 on the compute side); each thread accumulates a
// 4x4 register block of pair statistics (r2 and the periodic sums), then evaluates the
// canonical kernel and stores 4 consecutive rows per column (column-major output).
// Roofline (N=16384, d=32, fp64): 1.08e9 algorithmic bytes (lower triangle + X) vs
// ~1.3e8 pairs x (2..5 d + exp) VALU flops: VALU-bound for Periodic, balanced for Gaussian.
#include "gprx_internal.h"
#include "k_tile.h"

#include <climits>
#include <cmath>
#include <cstdint>

namespace gprx {

template <typename T>
__global__ void sincos_tables_kernel(const T* __restrict__ X, int64_t nd, T b0, T b1, int nper,
                                     T* __restrict__ tab) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nd) return;
    T x = X[e];
    T s, c;
    gsincos(b0 * x, &s, &c);
    tab[e] = s;
    tab[nd + e] = c;
    if (nper > 1) {
        gsincos(b1 * x, &s, &c);
        tab[2 * nd + e] = s;
        tab[3 * nd + e] = c;
    }
}

template <typename T>
void launch_sincos_tables(const KCanon<T>& K, const T* X, int64_t n, int d, T* tab, hipStream_t s) {
    if (K.nper == 0 || n == 0) return;
    int64_t nd = n * (int64_t)d;
    unsigned grid = (unsigned)((nd + 255) / 256);
    T b1 = K.nper > 1 ? K.b[1] : T(0);
    hipLaunchKernelGGL(sincos_tables_kernel<T>, dim3(grid), dim3(256), 0, s, X, nd, K.b[0], b1, K.nper, tab);
}

// Triangular tile index -> (ti, tj), tj <= ti.
__device__ __forceinline__ void tri_index(int64_t b, int64_t& ti, int64_t& tj) {
    int64_t i = (int64_t)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
    while ((i + 1) * (i + 2) / 2 <= b) i++;
    while (i * (i + 1) / 2 > b) i--;
    ti = i;
    tj = b - i * (i + 1) / 2;
}

template <typename T, int NPER, bool R2>
__global__ __launch_bounds__(256) void kbuild_kernel(KCanon<T> K, const T* __restrict__ Xa,
                                                     const T* __restrict__ tabA, int64_t na,
                                                     const T* __restrict__ Xb, const T* __restrict__ tabB,
                                                     int64_t nb, int d, T* __restrict__ A, int64_t ld,
                                                     int64_t npad, int lower, int64_t ntr, T sigma2,
                                                     int* __restrict__ flag) {
    __shared__ __attribute__((aligned(16))) TileSmem<T, NPER, R2> sm;

    int64_t ti, tj;
    if (lower) {
        tri_index(blockIdx.x, ti, tj);
    } else {
        ti = blockIdx.x % ntr;
        tj = blockIdx.x / ntr;
    }
    const int64_t i0 = ti * BT, j0 = tj * BT;
    const int t = threadIdx.x;
    const int tx = t & 15, ty = t >> 4;

    T r2[4][4], s0[4][4], s1[4][4];
    // Tiles entirely in the identity padding (square mode) need no kernel work.
    const bool pad_tile = lower && (i0 >= na || j0 >= nb);
    if (!pad_tile) {
        tile_stats<T, NPER, R2>(sm, Xa, tabA, na, i0, Xb, tabB, nb, j0, d, r2, s0, s1);
    } else {
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 4; b++) r2[a][b] = s0[a][b] = s1[a][b] = T(0);
    }

    // Stores: each thread owns 4 consecutive rows of 4 columns; the 16 lanes of a column
    // cover 64 consecutive rows, so one 32-byte store per thread and column gives 512
    // contiguous bytes per column and wave (whole cache lines: no read-for-ownership of
    // partial lines at the memory side).
    bool bad = false;
    const bool vec_ok = ((ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(A) & 31) == 0);
#pragma unroll
    for (int b = 0; b < 4; b++) {
        const int64_t gj = j0 + ty * 4 + b;
        const int64_t gi0 = i0 + tx * 4;
        T v[4];
        bool ok[4];
#pragma unroll
        for (int a = 0; a < 4; a++) {
            const int64_t gi = gi0 + a;
            if (lower) {
                ok[a] = gi < npad && gj < npad;
                if (gi >= na || gj >= nb) {
                    v[a] = (gi == gj) ? T(1) : T(0);
                } else {
                    v[a] = kernel_value(K, r2[a][b], s0[a][b], s1[a][b]);
                    if (!isfinite(v[a])) bad = true;
                    if (gi == gj) v[a] += sigma2;
                }
            } else {
                ok[a] = gi < na && gj < nb;
                v[a] = ok[a] ? kernel_value(K, r2[a][b], s0[a][b], s1[a][b]) : T(0);
                if (ok[a] && !isfinite(v[a])) bad = true;
            }
        }
        T* dst = A + gi0 + gj * ld;
        if (vec_ok && ok[3]) {  // ok[3] implies ok[0..2]
            if constexpr (sizeof(T) == 8) {
                typedef double d2 __attribute__((ext_vector_type(2)));
                reinterpret_cast<d2*>(dst)[0] = d2{v[0], v[1]};
                reinterpret_cast<d2*>(dst)[1] = d2{v[2], v[3]};
            } else {
                typedef float f4 __attribute__((ext_vector_type(4)));
                *reinterpret_cast<f4*>(dst) = f4{v[0], v[1], v[2], v[3]};
            }
        } else {
#pragma unroll
            for (int a = 0; a < 4; a++)
                if (ok[a]) dst[a] = v[a];
        }
    }
    if (bad) atomicOr(flag, 1);
}

template <typename T>
void launch_kbuild(const KCanon<T>& K, const T* Xa, const T* tabA, int64_t na, const T* Xb, const T* tabB,
                   int64_t nb, int d, T* A, int64_t ld, int64_t npad, bool lower, T sigma2, int* flag,
                   hipStream_t s) {
    int64_t ntr, ntc, ntiles;
    if (lower) {
        ntr = ntc = (npad + BT - 1) / BT;
        ntiles = ntr * (ntr + 1) / 2;
    } else {
        ntr = (na + BT - 1) / BT;
        ntc = (nb + BT - 1) / BT;
        ntiles = ntr * ntc;
    }
    if (ntiles == 0) return;
    const bool r2 = K.need_r2 != 0;
    const double bytes = lower ? (double)sizeof(T) * ((double)na * d + (double)npad * (npad + 1) / 2)
                               : (double)sizeof(T) * ((double)(na + nb) * d + (double)na * nb);
    ProfScope ps(KC_BUILD, s, 0.0, bytes);
    dim3 grid((unsigned)ntiles), block(256);
#define GPRX_KB(NP, R)                                                                                   \
    hipLaunchKernelGGL((kbuild_kernel<T, NP, R>), grid, block, 0, s, K, Xa, tabA, na, Xb, tabB, nb, d, A, \
                       ld, npad, (int)lower, ntr, sigma2, flag)
    if (K.nper == 0) {
        GPRX_KB(0, true);
    } else if (K.nper == 1) {
        if (r2) GPRX_KB(1, true);
        else GPRX_KB(1, false);
    } else {
        if (r2) GPRX_KB(2, true);
        else GPRX_KB(2, false);
    }
#undef GPRX_KB
}

// ---------------------------------------------------------------------------------------
// Derivative matrices (parity tests / small N): one thread per (i, j) pair, gradient of the
// canonical form by the product rule (equivalent to the reference's Sum/Product
// concatenation, include/Kernel.h:169-178, 318-327).
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void deriv_matrix_kernel(KCanon<T> K, const T* __restrict__ X, int64_t n, int d, T* __restrict__ D) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * n) return;
    int64_t i = e % n, j = e / n;
    T r2, s0, s1, f0, f1;
    pair_stats(K, X + i * d, X + j * d, d, r2, s0, s1, f0, f1);
    T g[GPRX_MAX_KPARAMS];
    kernel_grad(K, r2, s0, s1, f0, f1, g);
    for (int p = 0; p < K.nparams; p++) D[(int64_t)p * n * n + i + j * n] = g[p];
}

template <typename T>
void launch_deriv_matrix(const KCanon<T>& K, const T* X, const T* tab, int64_t n, int d, T* D, hipStream_t s) {
    (void)tab;
    int64_t e = n * n;
    if (e == 0) return;
    hipLaunchKernelGGL(deriv_matrix_kernel<T>, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, K, X, n, d, D);
}

// ---------------------------------------------------------------------------------------
// Augmented label rows for the fused forward solve.
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void aug_rows_kernel(const T* __restrict__ Y, int64_t n, int m, T* __restrict__ A, int64_t ld,
                                int64_t row0, int64_t ncols, int64_t mp) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= mp * ncols) return;
    int64_t r = e % mp, j = e / mp;
    T v = T(0);
    if (r < m && j < n) v = Y[j * m + r];
    A[row0 + r + j * ld] = v;
}

template <typename T>
void launch_label_rows(const T* Y, int64_t n, int m, T* A, int64_t ld, int64_t row0, int64_t ncols, int64_t mp,
                       hipStream_t s) {
    int64_t e = mp * ncols;
    if (e == 0) return;
    hipLaunchKernelGGL(aug_rows_kernel<T>, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, Y, n, m, A, ld, row0,
                       ncols, mp);
}

template <typename T>
void launch_aug_rows(const T* Y, int64_t n, int m, T* A, int64_t ld, int64_t np, int64_t mp, hipStream_t s) {
    launch_label_rows<T>(Y, n, m, A, ld, np, np, mp, s);
}

// A fit's status words: info = INT_MAX (no failed pivot), flag = 0 (no non-finite entry), in
// one launch (two memsets were two fill kernels, each with its dispatch gap, on every fit)
__global__ void fit_status_init_kernel(int* __restrict__ info, int* __restrict__ flag) {
    if (threadIdx.x == 0) {
        *info = INT_MAX;
        *flag = 0;
    }
}
void launch_fit_status_init(int* info, int* flag, hipStream_t s) {
    hipLaunchKernelGGL(fit_status_init_kernel, dim3(1), dim3(64), 0, s, info, flag);
    GPRX_HIP(hipGetLastError());
}

// ... and back to the host: flag, info and the two reduced scalars into mapped pinned memory
// (out[0], out[1] as ints, out[2..3]) by one kernel instead of three copy launches
__global__ void fit_status_gather_kernel(const int* __restrict__ flag, const int* __restrict__ info,
                                         const double* __restrict__ red, double* __restrict__ out) {
    const int t = threadIdx.x;
    if (t < 2) {
        const int v = t == 0 ? *flag : *info;
        __hip_atomic_store(reinterpret_cast<int*>(out + t), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (t < 4) {
        __hip_atomic_store(out + t, red[t - 2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}
void launch_fit_status_gather(const int* flag, const int* info, const double* red, double* out_mapped, hipStream_t s) {
    hipLaunchKernelGGL(fit_status_gather_kernel, dim3(1), dim3(64), 0, s, flag, info, red, out_mapped);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
__global__ void diag_fix_kernel(T* __restrict__ A, int64_t ld, int64_t c0, int64_t w, int64_t n, T sigma2) {
    const int64_t i = c0 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= c0 + w) return;
    A[i + i * ld] = (i < n) ? A[i + i * ld] + sigma2 : T(1);
}

// Diagonal of columns [c0, c0+w): += sigma2 for i < n (AddNoiseToKernelMatrix,
// lib/GaussianProcess.cpp:375-381), 1 for the padding.
template <typename T>
void launch_diag_fix(T* A, int64_t ld, int64_t c0, int64_t w, int64_t n, T sigma2, hipStream_t s) {
    if (w <= 0) return;
    hipLaunchKernelGGL(diag_fix_kernel<T>, dim3((unsigned)((w + 255) / 256)), dim3(256), 0, s, A, ld, c0, w, n, sigma2);
}

#define GPRX_INST(T)                                                                                       \
    template void launch_sincos_tables<T>(const KCanon<T>&, const T*, int64_t, int, T*, hipStream_t);     \
    template void launch_kbuild<T>(const KCanon<T>&, const T*, const T*, int64_t, const T*, const T*,     \
                                   int64_t, int, T*, int64_t, int64_t, bool, T, int*, hipStream_t);       \
    template void launch_deriv_matrix<T>(const KCanon<T>&, const T*, const T*, int64_t, int, T*,          \
                                         hipStream_t);                                                     \
    template void launch_aug_rows<T>(const T*, int64_t, int, T*, int64_t, int64_t, int64_t, hipStream_t); \
    template void launch_label_rows<T>(const T*, int64_t, int, T*, int64_t, int64_t, int64_t, int64_t,   \
                                       hipStream_t);                                                       \
    template void launch_diag_fix<T>(T*, int64_t, int64_t, int64_t, int64_t, T, hipStream_t);
GPRX_INST(double)
GPRX_INST(float)
#undef GPRX_INST

}  // namespace gprx
