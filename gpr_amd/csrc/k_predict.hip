// k_predict.hip — batched prediction on gfx950.
//
// Replaces the per-point serial loop of the reference's prediction path:
//   Predict            (Kx^T alpha)                      lib/GaussianProcess.cpp:54-61, 684-693
//   PredictDerivative  D(:,c) = -X^T (Kx o alpha_c)      lib/GaussianProcess.cpp:64-81, 697-706
//   operator()(x,y)    k(x,y) - Kx^T C Ky                lib/GaussianProcess.cpp:84-99
//
// Mean / derivative: one workgroup per 64 queries streams the training set in 64-point
// tiles: pair statistics and kernel values come from the shared tile (k_tile.h), the
// 64x64 kernel tile goes to LDS and is multiplied against the matching 64 rows of
// Z = [alpha | alpha o X] (never materialising K(Xq, X)).  The derivative uses
//   D[q][k][c] = -(x_qk * mean[q][c] - sum_j k(q,j) alpha_jc x_jk).
// Posterior covariance: V = L^{-1} K(X, Xq) by the blocked triangular solve (MFMA gemm
// against the stored Cholesky factor), then k(x,y) - v_x . v_y.
#include "gprx_internal.h"

#include <algorithm>
#include "k_tile.h"

namespace gprx {

constexpr int PZ = 64;  // Z columns per pass

template <typename T>
__global__ void build_z_kernel(const T* __restrict__ X, const T* __restrict__ alpha, int64_t n, int d, int m,
                               int deriv, T* __restrict__ Z, int64_t ncz) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * ncz) return;
    const int64_t j = e / ncz;
    const int c = (int)(e % ncz);
    T v;
    if (c < m) {
        v = alpha[j * m + c];
    } else {
        const int cc = c - m;
        const int k = cc / m, o = cc % m;
        v = alpha[j * m + o] * X[j * d + k];
    }
    (void)deriv;
    Z[e] = v;
}

template <typename T, int NPER, bool R2>
__global__ __launch_bounds__(256) void predict_kernel(KCanon<T> K, const T* __restrict__ X, const T* __restrict__ tabX,
                                                      int64_t n, int d, const T* __restrict__ Z, int64_t ncz, int col0,
                                                      int ncols, const T* __restrict__ Xq, const T* __restrict__ tabQ,
                                                      int64_t q, T* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) TileSmem<T, NPER, R2> sm;
    __shared__ T sK[BT][BT + 1];
    __shared__ T sZ[BT][PZ + 1];

    const int t = threadIdx.x;
    const int tx = t & 15, ty = t >> 4;
    const int64_t i0 = (int64_t)blockIdx.x * BT;
    const int orow = t & 63;
    const int ocol = t >> 6;  // 0..3, columns ocol + 4u
    T acc[PZ / 4];
#pragma unroll
    for (int u = 0; u < PZ / 4; u++) acc[u] = 0;

    for (int64_t j0 = 0; j0 < n; j0 += BT) {
        T r2[4][4], s0[4][4], s1[4][4];
        tile_stats<T, NPER, R2>(sm, Xq, tabQ, q, i0, X, tabX, n, j0, d, r2, s0, s1);
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const bool ok = (i0 + tx * 4 + a < q) && (j0 + ty * 4 + b < n);
                sK[tx * 4 + a][ty * 4 + b] = ok ? kernel_value(K, r2[a][b], s0[a][b], s1[a][b]) : T(0);
            }
        for (int e = t; e < BT * ncols; e += 256) {
            const int r = e / ncols, c = e % ncols;
            const int64_t j = j0 + r;
            sZ[r][c] = (j < n) ? Z[j * ncz + col0 + c] : T(0);
        }
        __syncthreads();
#pragma unroll
        for (int u = 0; u < PZ / 4; u++) {
            const int c = ocol + 4 * u;
            if (c < ncols) {
                T s = acc[u];
#pragma unroll 8
                for (int b = 0; b < BT; b++) s = fma(sK[orow][b], sZ[b][c], s);
                acc[u] = s;
            }
        }
        __syncthreads();
    }
    const int64_t qi = i0 + orow;
    if (qi < q) {
#pragma unroll
        for (int u = 0; u < PZ / 4; u++) {
            const int c = ocol + 4 * u;
            if (c < ncols) out[qi * ncz + col0 + c] = acc[u];
        }
    }
}

template <typename T>
__global__ void finalize_predict_kernel(const T* __restrict__ out, int64_t ncz, const T* __restrict__ Xq, int64_t q,
                                        int d, int m, T* __restrict__ mean, T* __restrict__ deriv) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= q * m) return;
    const int64_t qi = e / m;
    const int c = (int)(e % m);
    const T mu = out[qi * ncz + c];
    mean[e] = mu;
    if (deriv) {
        for (int k = 0; k < d; k++) {
            const T s = out[qi * ncz + m + k * m + c];
            deriv[(qi * d + k) * m + c] = -(Xq[qi * d + k] * mu - s);
        }
    }
}

template <typename T>
void launch_predict(const KCanon<T>& K, const T* X, const T* tabX, int64_t n, int d, int m, const T* alpha,
                    const T* Xq, const T* tabQ, int64_t q, T* mean, T* deriv, T* Z, T* out, hipStream_t s) {
    // workspace: Z (n x ncz) and out (q x ncz), ncz = m (1 + d if deriv)
    const int64_t ncz = (int64_t)m * (deriv ? (1 + d) : 1);
    ProfScope ps(KC_PREDICT, s, (double)q * n * (2.0 * d + 2.0 * ncz), (double)sizeof(T) * (double)(q + n) * d);
    hipLaunchKernelGGL(build_z_kernel<T>, dim3((unsigned)((n * ncz + 255) / 256)), dim3(256), 0, s, X, alpha, n, d,
                       m, deriv ? 1 : 0, Z, ncz);
    const unsigned grid = (unsigned)((q + BT - 1) / BT);
    for (int64_t c0 = 0; c0 < ncz; c0 += PZ) {
        const int nc = (int)std::min<int64_t>(PZ, ncz - c0);
#define GPRX_PK(NP, R)                                                                                       \
    hipLaunchKernelGGL((predict_kernel<T, NP, R>), dim3(grid), dim3(256), 0, s, K, X, tabX, n, d, Z, ncz,     \
                       (int)c0, nc, Xq, tabQ, q, out)
        if (K.nper == 0) GPRX_PK(0, true);
        else if (K.nper == 1) {
            if (K.need_r2) GPRX_PK(1, true);
            else GPRX_PK(1, false);
        } else {
            if (K.need_r2) GPRX_PK(2, true);
            else GPRX_PK(2, false);
        }
#undef GPRX_PK
    }
    hipLaunchKernelGGL(finalize_predict_kernel<T>, dim3((unsigned)((q * m + 255) / 256)), dim3(256), 0, s, out, ncz,
                       Xq, q, d, m, mean, deriv);
}

// ---------------------------------------------------------------------------------------
// Posterior covariance helpers
// ---------------------------------------------------------------------------------------
// k(a_i, b_i) for q pairs (direct statistics, includes the periodic sums)
template <typename T>
__global__ void pair_kernel_kernel(KCanon<T> K, const T* __restrict__ Xa, const T* __restrict__ Xb, int64_t q, int d,
                                   T* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= q) return;
    T r2, s0, s1, f0, f1;
    pair_stats(K, Xa + i * d, Xb + i * d, d, r2, s0, s1, f0, f1);
    out[i] = kernel_value(K, r2, s0, s1);
}

// out[i] = kab[i] - sum_j Va[i + j ld] Vb[i + j ld]   (one wave per row block of 64 rows)
// out[i] = kab[i] - sum_j Va[i + j ld] Vb[i + j ld]: RD_SPLIT partial sums over contiguous
// j-ranges (64 consecutive rows per wave: 512-B coalesced column segments), then a fixed-order
// sum.  (One thread per row over all n columns used 16 workgroups for q = 4096: 6.8 ms.)
constexpr int RD_SPLIT = 64;
template <typename T>
__global__ __launch_bounds__(256) void rowdot_part_kernel(const T* __restrict__ Va, const T* __restrict__ Vb,
                                                          int64_t ld, int64_t q, int64_t n, T* __restrict__ part) {
    const int64_t i = (int64_t)blockIdx.x * 64 + (threadIdx.x & 63);
    const int sub = threadIdx.x >> 6;  // 4 waves share the split's j-range, interleaved
    const int64_t per = (n + RD_SPLIT - 1) / RD_SPLIT, j0 = per * blockIdx.y, j1 = min(n, j0 + per);
    __shared__ T red[4][64];
    T s = 0;
    if (i < q)
        for (int64_t j = j0 + sub; j < j1; j += 4) s = fma(Va[i + j * ld], Vb[i + j * ld], s);
    red[sub][threadIdx.x & 63] = s;
    __syncthreads();
    if (sub == 0 && i < q)
        part[(int64_t)blockIdx.y * q + i] = ((red[0][threadIdx.x] + red[1][threadIdx.x]) + red[2][threadIdx.x]) +
                                            red[3][threadIdx.x];
}
template <typename T>
__global__ void rowdot_sum_kernel(const T* __restrict__ part, int64_t q, const T* __restrict__ kab,
                                  T* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= q) return;
    T s = 0;
    for (int k = 0; k < RD_SPLIT; k++) s += part[(int64_t)k * q + i];
    out[i] = kab[i] - s;
}

template <typename T>
void launch_pair_kernel(const KCanon<T>& K, const T* Xa, const T* Xb, int64_t q, int d, T* out, hipStream_t s) {
    if (q == 0) return;
    hipLaunchKernelGGL(pair_kernel_kernel<T>, dim3((unsigned)((q + 255) / 256)), dim3(256), 0, s, K, Xa, Xb, q, d,
                       out);
}

template <typename T>
void launch_rowdot(const T* Va, const T* Vb, int64_t ld, int64_t q, int64_t n, const T* kab, T* out, hipStream_t s) {
    if (q == 0) return;
    T* part = nullptr;
    GPRX_HIP(hipMalloc((void**)&part, sizeof(T) * RD_SPLIT * q));
    hipLaunchKernelGGL(rowdot_part_kernel<T>, dim3((unsigned)((q + 63) / 64), RD_SPLIT), dim3(256), 0, s, Va, Vb, ld,
                       q, n, part);
    hipLaunchKernelGGL(rowdot_sum_kernel<T>, dim3((unsigned)((q + 255) / 256)), dim3(256), 0, s, (const T*)part, q,
                       kab, out);
    GPRX_HIP(hipFree(part));  // (synchronises: the caller downloads the result next anyway)
}

// Solve V L^T = R in place for the rows of R (qp x np, column-major, ld), given the
// factor L (column-major, ldA) and its diagonal-block inverses: V = R L^{-T}, i.e. each
// row of V is (L^{-1} r)^T.
// Recursive right-looking: the column range [k0, k1) is solved as its left half, ONE update
// of the right half by the left (K = the left half's width), then the right half; a single
// 128-block is solved with its inverse.  The updates' K doubles at each level up (8192 at the
// top for N = 16384): per-block updates with K = 128 paid the tile mainloop's fill and a launch
// per 128 columns (0.49 of peak); groups of 4 / 8 / 16 blocks gave 0.59 / 0.61 / 0.62.
template <typename T>
static void trsm_rows_rec(const T* A, int64_t ldA, const T* Linv, T* R, int64_t ld, int64_t qp, int64_t k0, int64_t k1,
                          hipStream_t s) {
    if (k1 - k0 <= DB) {
        T* Rk = R + k0 * ld;
        launch_gemm_nt<T>(Rk, ld, Rk, ld, Linv + (k0 / DB) * (int64_t)DB * DB, DB, qp, DB, DB, T(1), T(0), false, s);
        return;
    }
    const int64_t nb = (k1 - k0) / DB, km = k0 + ((nb + 1) / 2) * DB;
    trsm_rows_rec<T>(A, ldA, Linv, R, ld, qp, k0, km, s);
    launch_gemm_nt<T>(R + km * ld, ld, R + k0 * ld, ld, A + km + k0 * ldA, ldA, qp, k1 - km, km - k0, T(-1), T(1), false,
                      s);
    trsm_rows_rec<T>(A, ldA, Linv, R, ld, qp, km, k1, s);
}
template <typename T>
void trsm_rows(const T* A, int64_t ldA, int64_t np, const T* Linv, T* R, int64_t ld, int64_t qp, hipStream_t s) {
    if (np > 0) trsm_rows_rec<T>(A, ldA, Linv, R, ld, qp, 0, np, s);
}

#define GPRX_INST(T)                                                                                         \
    template void launch_predict<T>(const KCanon<T>&, const T*, const T*, int64_t, int, int, const T*, const T*, \
                                    const T*, int64_t, T*, T*, T*, T*, hipStream_t);                          \
    template void launch_pair_kernel<T>(const KCanon<T>&, const T*, const T*, int64_t, int, T*, hipStream_t);   \
    template void launch_rowdot<T>(const T*, const T*, int64_t, int64_t, int64_t, const T*, T*, hipStream_t);    \
    template void trsm_rows<T>(const T*, int64_t, int64_t, const T*, T*, int64_t, int64_t, hipStream_t);
GPRX_INST(double)
GPRX_INST(float)
#undef GPRX_INST

}  // namespace gprx
