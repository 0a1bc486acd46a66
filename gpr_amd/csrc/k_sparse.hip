// k_sparse.hip — small device pieces of the sparse GP's log-marginal likelihood
// (SparseGaussianLogLikelihood, include/SparseLikelihood.h:113-535), evaluated in the
// O(N M^2) form described in gprx_api.cpp (sparse_lml_impl): the data-fit residual rows, the
// label norm y^T y and the M x M difference Kmm^{-1} - Sigma.  The heavy parts run on the
// shared machinery: Kmn blocks (kcross_mma_kernel), the GEMM K(Xc, Xm) Sigma (tile GEMM), the
// weighted derivative sums (grad_mma_kernel / lml_grad_kernel in their cross forms).
#include "gprx_internal.h"

namespace gprx {

// out[i] = alpha (y[i] - sum_j A[i + j lda] u[j]): one thread per row, the column loop walks
// A column by column so consecutive threads read consecutive addresses.
template <typename T>
__global__ __launch_bounds__(256) void sparse_resid_kernel(const T* __restrict__ A, int64_t lda, int64_t n, int64_t M,
                                                           const T* __restrict__ u, const T* __restrict__ y, T alpha,
                                                           T* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    T acc = 0;
    for (int64_t j = 0; j < M; j++) acc = fma(A[i + j * lda], u[j], acc);
    out[i] = alpha * (y[i] - acc);
}

// one workgroup: per-thread strided partial sums, then a fixed-order tree (deterministic)
template <typename T>
__global__ __launch_bounds__(256) void sq_sum_kernel(const T* __restrict__ y, int64_t n, double* __restrict__ out) {
    __shared__ double red[256];
    const int t = threadIdx.x;
    double v = 0;
    for (int64_t i = t; i < n; i += 256) {
        const double a = (double)y[i];
        v = fma(a, a, v);
    }
    red[t] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) red[t] += red[t + o];
        __syncthreads();
    }
    if (t == 0) out[0] = red[0];
}

template <typename T>
__global__ void sub_kernel(const T* __restrict__ X, const T* __restrict__ Y, T* __restrict__ Z, int64_t e) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < e) Z[i] = X[i] - Y[i];
}

template <typename T>
void launch_sparse_resid(const T* A, int64_t lda, int64_t n, int64_t M, const T* u, const T* y, T alpha, T* out,
                         hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(sparse_resid_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, A, lda, n, M, u, y,
                       alpha, out);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void launch_sq_sum(const T* y, int64_t n, double* out, hipStream_t s) {
    hipLaunchKernelGGL(sq_sum_kernel<T>, dim3(1), dim3(256), 0, s, y, n, out);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void launch_sub(const T* X, const T* Y, T* Z, int64_t e, hipStream_t s) {
    if (e <= 0) return;
    hipLaunchKernelGGL(sub_kernel<T>, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, X, Y, Z, e);
    GPRX_HIP(hipGetLastError());
}

#define GPRX_INST(T)                                                                                             \
    template void launch_sparse_resid<T>(const T*, int64_t, int64_t, int64_t, const T*, const T*, T, T*,        \
                                         hipStream_t);                                                           \
    template void launch_sq_sum<T>(const T*, int64_t, double*, hipStream_t);                                     \
    template void launch_sub<T>(const T*, const T*, T*, int64_t, hipStream_t);
GPRX_INST(double)
GPRX_INST(float)
#undef GPRX_INST

}  // namespace gprx
