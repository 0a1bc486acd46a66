// k_refine.hip — fp64 iterative refinement of the regression vectors of an fp32 GP (gfx950).
//
// The reference never factorises an fp32 covariance in fp32: lapack::lu_invert<float> casts
// K + sigma^2 I to double, inverts in double and casts back (include/LAPACKUtils.h:85-97).
// libgprx keeps the fast fp32 tile factorisation (k_ptiles.hip) and recovers fp64-accurate
// alpha by mixed-precision iterative refinement:
//     r = Y - (K + sigma^2 I) alpha      K re-evaluated in fp64 from the pair statistics
//                                        (k_pairs.hip predict path, q = the training set)
//     delta = (L L^T)^{-1} r             the fp32 factor: forward solve trsm_rows, back
//                                        substitution launch_backsolve_chain
//     alpha += delta                      accumulated in fp64
// Each step contracts the error by about cond(K) * 2^-24, so two steps reach fp64-level
// agreement with the double solve for cond up to ~1e5 (C4: cond ~ 1.1e3).  The kernels
// here are the elementwise glue between those solves.
#include "gprx_internal.h"

namespace gprx {

namespace rf {

template <typename S, typename D>
__global__ void convert_kernel(const S* __restrict__ in, D* __restrict__ out, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (D)in[i];
}

// r = Y - Kx - s2 a (fp64), stored as fp32 into the label rows of the factor workspace:
// A[row0 + c + j ld] = r[j][c] for j < n, c < m; zero for the padding rows c in [m, mp)
// and columns j in [n, ncols).  One thread per (column j, row c).
__global__ void residual_rows_kernel(const double* __restrict__ Y, const double* __restrict__ Kx,
                                     const double* __restrict__ a, double s2, int64_t n, int m, float* __restrict__ A,
                                     int64_t ld, int64_t row0, int64_t ncols, int mp) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ncols * mp) return;
    const int64_t j = e / mp;
    const int c = (int)(e % mp);
    float v = 0.f;
    if (j < n && c < m) {
        const int64_t k = j * m + c;
        v = (float)(Y[k] - Kx[k] - s2 * a[k]);
    }
    A[row0 + c + j * ld] = v;
}

// a += delta (fp64), alpha = (float) a; nrm[0] = max |delta|, nrm[1] = max |a| (the bit
// patterns of non-negative doubles order like the values: unsigned atomicMax)
__global__ void accumulate_kernel(const float* __restrict__ delta, double* __restrict__ a, float* __restrict__ alpha,
                                  int64_t e_n, unsigned long long* __restrict__ nrm) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    double dd = 0, aa = 0;
    if (e < e_n) {
        dd = (double)delta[e];
        aa = a[e] + dd;
        a[e] = aa;
        alpha[e] = (float)aa;
    }
    dd = fabs(dd);
    aa = fabs(aa);
    for (int off = 32; off > 0; off >>= 1) {
        dd = fmax(dd, __shfl_xor(dd, off));
        aa = fmax(aa, __shfl_xor(aa, off));
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMax(nrm, (unsigned long long)__double_as_longlong(dd));
        atomicMax(nrm + 1, (unsigned long long)__double_as_longlong(aa));
    }
}

// the sharded refinement (gprx_dist.cpp owns the rows): out[t][k] = X[idx[t]][k]
__global__ void gather_rows_kernel(const double* __restrict__ X, const int64_t* __restrict__ idx, int64_t q, int d,
                                   double* __restrict__ out) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= q * d) return;
    const int64_t t = e / d;
    out[e] = X[idx[t] * d + (e % d)];
}

// rhs[idx[t]][c] = Y - Kx - s2 a at the rows this process's ranks own (Kx: q x m, row t)
__global__ void residual_scatter_kernel(const double* __restrict__ Y, const double* __restrict__ Kx,
                                        const double* __restrict__ a, double s2, const int64_t* __restrict__ idx,
                                        int64_t q, int m, float* __restrict__ rhs) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= q * m) return;
    const int64_t t = e / m;
    const int c = (int)(e % m);
    const int64_t k = idx[t] * m + c;
    rhs[k] = (float)(Y[k] - Kx[e] - s2 * a[k]);
}

}  // namespace rf

void launch_gather_rows(const double* X, const int64_t* idx, int64_t q, int d, double* out, hipStream_t s) {
    if (q * d <= 0) return;
    hipLaunchKernelGGL(rf::gather_rows_kernel, dim3((unsigned)((q * d + 255) / 256)), dim3(256), 0, s, X, idx, q, d, out);
}

void launch_residual_scatter(const double* Y, const double* Kx, const double* a, double s2, const int64_t* idx,
                             int64_t q, int m, float* rhs, hipStream_t s) {
    if (q * m <= 0) return;
    hipLaunchKernelGGL(rf::residual_scatter_kernel, dim3((unsigned)((q * m + 255) / 256)), dim3(256), 0, s, Y, Kx, a,
                       s2, idx, q, m, rhs);
}

template <typename S, typename D>
void launch_convert(const S* in, D* out, int64_t n, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL((rf::convert_kernel<S, D>), dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, out, n);
}

void launch_residual_rows(const double* Y, const double* Kx, const double* a, double s2, int64_t n, int m, float* A,
                          int64_t ld, int64_t row0, int64_t ncols, int mp, hipStream_t s) {
    const int64_t e = ncols * mp;
    hipLaunchKernelGGL(rf::residual_rows_kernel, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, Y, Kx, a, s2, n,
                       m, A, ld, row0, ncols, mp);
}

void launch_refine_accumulate(const float* delta, double* a, float* alpha, int64_t e, unsigned long long* nrm,
                              hipStream_t s) {
    GPRX_HIP(hipMemsetAsync(nrm, 0, 2 * sizeof(unsigned long long), s));
    hipLaunchKernelGGL(rf::accumulate_kernel, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, delta, a, alpha, e,
                       nrm);
}

template void launch_convert<float, double>(const float*, double*, int64_t, hipStream_t);
template void launch_convert<double, float>(const double*, float*, int64_t, hipStream_t);

}  // namespace gprx
