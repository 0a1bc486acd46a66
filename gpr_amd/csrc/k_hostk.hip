// k_hostk.hip — kernels with no device form: the caller evaluates them (the reference's
// virtual Kernel<T>::operator() / GetDerivative, include/Kernel.h:52-59, 465-479) and hands
// the evaluated matrices over; the matrix-shaped work stays here.
//
//   kext_build     K + sigma^2 I from the caller's K (n x n, row-major) into the np x np
//                  column-major factor storage, identity on the padding, non-finite flag
//                  (lib/GaussianProcess.cpp:375-402)
//   kx_predict     mean = Kx alpha and the reference's derivative D(:,c) = -Xd^T (Kx o alpha_c)
//                  with Xd_i = x - x_i (lib/GaussianProcess.cpp:54-81) from the caller's Kx
//   dk_grad        grad_p = 1/2 sum_ij (alpha_i alpha_j - C_ij) dK_p,ij from the caller's
//                  derivative matrices (include/Likelihood.h:204-229)
#include "gprx_internal.h"

namespace gprx {

namespace {

template <typename T>
__global__ __launch_bounds__(256) void kext_build_kernel(const T* __restrict__ Kx, int64_t n, T* __restrict__ A,
                                                         int64_t ld, int64_t np, T sigma2, int* __restrict__ flag) {
    const int64_t c = blockIdx.y;  // column of A
    bool bad = false;
    for (int64_t r = blockIdx.x * 256 + threadIdx.x; r < np; r += (int64_t)gridDim.x * 256) {
        T v;
        if (r < n && c < n) {
            v = Kx[r * n + c];
            if (!isfinite(v)) bad = true;
            if (r == c) v += sigma2;
        } else {
            v = (r == c) ? T(1) : T(0);
        }
        A[r + c * ld] = v;
    }
    if (bad) atomicOr(flag, 1);
}

// one thread per (query, output column); and per (query, input dimension, output column)
template <typename T>
__global__ __launch_bounds__(256) void kx_mean_kernel(const T* __restrict__ Kx, int64_t q, int64_t n,
                                                      const T* __restrict__ alpha, int m, T* __restrict__ mean) {
    const int64_t e = blockIdx.x * (int64_t)256 + threadIdx.x;
    if (e >= q * m) return;
    const int64_t qi = e / m;
    const int c = (int)(e % m);
    T acc = T(0);
    for (int64_t i = 0; i < n; i++) acc += Kx[qi * n + i] * alpha[i * m + c];
    mean[e] = acc;
}

template <typename T>
__global__ __launch_bounds__(256) void kx_deriv_kernel(const T* __restrict__ Kx, const T* __restrict__ Xq,
                                                       const T* __restrict__ X, int64_t q, int64_t n, int d,
                                                       const T* __restrict__ alpha, int m, T* __restrict__ D) {
    const int64_t e = blockIdx.x * (int64_t)256 + threadIdx.x;  // D[qi][k][c], q x d x m
    if (e >= q * d * m) return;
    const int64_t qi = e / ((int64_t)d * m);
    const int k = (int)((e / m) % d), c = (int)(e % m);
    const T xk = Xq[qi * d + k];
    T acc = T(0);
    for (int64_t i = 0; i < n; i++) acc += (xk - X[i * d + k]) * Kx[qi * n + i] * alpha[i * m + c];
    D[e] = -acc;
}

// blockIdx.y = parameter p; C lower (column-major, ldc), symmetric use
template <typename T>
__global__ __launch_bounds__(256) void dk_grad_kernel(const T* __restrict__ dK, int64_t n, const T* __restrict__ alpha,
                                                      const T* __restrict__ C, int64_t ldc, double* __restrict__ out) {
    __shared__ double red[256];
    const int p = blockIdx.y;
    const T* D = dK + (int64_t)p * n * n;
    double acc = 0;
    for (int64_t e = blockIdx.x * (int64_t)256 + threadIdx.x; e < n * n; e += (int64_t)gridDim.x * 256) {
        const int64_t i = e / n, j = e % n;
        const int64_t lo = i > j ? i : j, hi = i > j ? j : i;  // C(lo, hi): the stored lower half
        acc += ((double)alpha[i] * (double)alpha[j] - (double)C[lo + hi * ldc]) * (double)D[e];
    }
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[(int64_t)p * gridDim.x + blockIdx.x] = 0.5 * red[0];  // this block's slot
}

// out[p] = sum of the gx slots of parameter p in a fixed order (the same bits on every call)
__global__ __launch_bounds__(256) void dk_grad_sum_kernel(const double* __restrict__ part, int gx,
                                                          double* __restrict__ out) {
    __shared__ double red[256];
    const int p = blockIdx.x;
    double v = 0;
    for (int b = threadIdx.x; b < gx; b += 256) v += part[(int64_t)p * gx + b];
    red[threadIdx.x] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[p] = red[0];
}

}  // namespace

template <typename T>
void launch_kext_build(const T* Kx, int64_t n, T* A, int64_t ld, int64_t np, T sigma2, int* flag, hipStream_t s) {
    hipLaunchKernelGGL(kext_build_kernel<T>, dim3((unsigned)((np + 255) / 256), (unsigned)np), dim3(256), 0, s, Kx, n,
                       A, ld, np, sigma2, flag);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void launch_kx_predict(const T* Kx, const T* Xq, const T* X, int64_t q, int64_t n, int d, const T* alpha, int m,
                       T* mean, T* D, hipStream_t s) {
    if (q <= 0) return;
    hipLaunchKernelGGL(kx_mean_kernel<T>, dim3((unsigned)((q * m + 255) / 256)), dim3(256), 0, s, Kx, q, n, alpha, m,
                       mean);
    if (D)
        hipLaunchKernelGGL(kx_deriv_kernel<T>, dim3((unsigned)((q * d * m + 255) / 256)), dim3(256), 0, s, Kx, Xq, X, q,
                           n, d, alpha, m, D);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void launch_dk_grad(const T* dK, int P, int64_t n, const T* alpha, const T* C, int64_t ldc, double* out,
                    hipStream_t s) {
    GPRX_HIP(hipMemsetAsync(out, 0, sizeof(double) * P, s));
    if (P <= 0 || n <= 0) return;
    const unsigned gx = (unsigned)std::min<int64_t>(1024, (n * n + 255) / 256);
    double* part = nullptr;  // per-block slots (stream-ordered scratch)
    GPRX_HIP(hipMallocAsync((void**)&part, sizeof(double) * gx * (size_t)P, s));
    hipLaunchKernelGGL(dk_grad_kernel<T>, dim3(gx, (unsigned)P), dim3(256), 0, s, dK, n, alpha, C, ldc, part);
    hipLaunchKernelGGL(dk_grad_sum_kernel, dim3((unsigned)P), dim3(256), 0, s, (const double*)part, (int)gx, out);
    GPRX_HIP(hipGetLastError());
    GPRX_HIP(hipFreeAsync(part, s));
}

#define GPRX_INST(T)                                                                                              \
    template void launch_kext_build<T>(const T*, int64_t, T*, int64_t, int64_t, T, int*, hipStream_t);           \
    template void launch_kx_predict<T>(const T*, const T*, const T*, int64_t, int64_t, int, const T*, int, T*, T*, \
                                       hipStream_t);                                                              \
    template void launch_dk_grad<T>(const T*, int, int64_t, const T*, const T*, int64_t, double*, hipStream_t);
GPRX_INST(double)
GPRX_INST(float)
#undef GPRX_INST

}  // namespace gprx
