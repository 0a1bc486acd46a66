// k_lml.hip — explicit inverse from the Cholesky factor and the fused log-likelihood
// gradient on gfx950.
//
// Replaces, for the GaussianLogLikelihood gradient (include/Likelihood.h:204-229, 258-283):
//   - the explicit core matrix C = (K + sigma^2 I)^{-1} from lapack::lu_invert
//     (include/LAPACKUtils.h:85-97) -> here  V = L^{-T} (triangular solve against the stored
//     factor, only the non-zero upper part is computed) and C = V V^T (lower, the K range of
//     every output tile starts at its row: LAUUM-shaped MFMA gemm);
//   - the stacked derivative matrices D_p (lib/GaussianProcess.cpp:472-495, P*N*N values)
//     and the P dense N^3 products tr((alpha alpha^T - C) D_p) -> one pass over the lower
//     triangle that recomputes dK/dp per pair from the streaming statistics and reduces
//     sum_ij (alpha_i alpha_j - C_ij) dK_ij/dp in registers.
#include "gprx_internal.h"
#include "k_tile.h"

#include <algorithm>

namespace gprx {

template <typename T>
void launch_gemm_nt_kskip(T* C, int64_t ldc, const T* A, int64_t lda, const T* B, int64_t ldb, int64_t M, int64_t N,
                          int64_t K, hipStream_t s);

template <typename T>
__global__ void set_diag_kernel(T* __restrict__ A, int64_t ld, int64_t beg, int64_t end, T v) {
    int64_t i = beg + (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < end) A[i + i * ld] = v;
}

template <typename T>
void launch_set_identity_pad(T* A, int64_t ld, int64_t n, int64_t np, hipStream_t s) {
    if (np <= n) return;
    hipLaunchKernelGGL(set_diag_kernel<T>, dim3((unsigned)((np - n + 255) / 256)), dim3(256), 0, s, A, ld, n, np, T(1));
}

template <typename T>
__global__ void add_lower_kernel(T* __restrict__ S, int64_t lds, const T* __restrict__ K, int64_t ldk, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, j = blockIdx.y;
    if (i < n && i >= j) S[i + j * lds] += K[i + j * ldk];
}

// Mirror the lower triangle of C (n x n, column-major, ld ldc) into its upper triangle:
// 32x32 tiles transposed through LDS, so both the reads and the writes are column runs.
template <typename T>
__global__ __launch_bounds__(256) void sym_fill_kernel(T* __restrict__ C, int64_t ldc, int64_t n) {
    const int64_t bx = blockIdx.x, by = blockIdx.y;  // destination tile: rows bx, columns by
    if (bx > by) return;
    __shared__ T sh[32][33];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
#pragma unroll
    for (int k = 0; k < 4; k++) {  // source tile: rows by, columns bx (lower)
        const int64_t r = by * 32 + tx, c = bx * 32 + ty + 8 * k;
        if (r < n && c < n) sh[ty + 8 * k][tx] = C[r + c * ldc];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int64_t i = bx * 32 + tx, j = by * 32 + ty + 8 * k;
        if (j < n && i < j) C[i + j * ldc] = sh[tx][ty + 8 * k];
    }
}

template <typename T>
void launch_sym_fill(T* C, int64_t ldc, int64_t n, hipStream_t s) {
    if (n <= 0) return;
    const unsigned nt = (unsigned)((n + 31) / 32);
    hipLaunchKernelGGL(sym_fill_kernel<T>, dim3(nt, nt), dim3(256), 0, s, C, ldc, n);
}

// S (lower, n x n, ld lds) += K (lower, ld ldk)
template <typename T>
void launch_gemm_add_lower(T* S, int64_t lds, const T* K, int64_t ldk, int64_t n, hipStream_t s) {
    if (n <= 0) return;
    hipLaunchKernelGGL(add_lower_kernel<T>, dim3((unsigned)((n + 255) / 256), (unsigned)n), dim3(256), 0, s, S, lds, K,
                       ldk, n);
}

template <typename T>
__global__ void sum_partials_kernel(T* __restrict__ S, int64_t stride, int P) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= stride) return;
    T v = S[e];
    for (int p = 1; p < P; p++) v += S[e + p * stride];
    S[e] = v;
}

// S[0:stride] += sum_p S[p*stride : (p+1)*stride] (split-K partials, fixed order)
template <typename T>
void launch_sum_partials(T* S, int64_t stride, int P, hipStream_t s) {
    if (P <= 1) return;
    hipLaunchKernelGGL(sum_partials_kernel<T>, dim3((unsigned)((stride + 255) / 256)), dim3(256), 0, s, S, stride, P);
}

template <typename T>
void launch_spd_inverse_from_factor(const T* A, int64_t ldA, int64_t np, const T* Linv, T* V, T* C, hipStream_t s) {
    Prof* saved = g_prof;  // the trsm/gemm pieces are accounted as one INVERSE phase
    ProfScope ps(KC_INVERSE, s, 2.0 * (double)np * np * np / 3.0, 0.0);
    g_prof = nullptr;
    GPRX_HIP(hipMemsetAsync(V, 0, sizeof(T) * np * np, s));
    hipLaunchKernelGGL(set_diag_kernel<T>, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, V, np, (int64_t)0, np,
                       T(1));
    // rows of V are (L^{-1} e_i)^T: row i is zero left of column i, so at column block k only
    // the rows above the block's end take part.
    for (int64_t k0 = 0; k0 < np; k0 += DB) {
        const int64_t rows = k0 + DB;
        T* Vk = V + k0 * np;
        launch_gemm_nt<T>(Vk, np, Vk, np, Linv + (k0 / DB) * (int64_t)DB * DB, DB, rows, DB, DB, T(1), T(0), false, s);
        const int64_t rem = np - rows;
        if (rem > 0)
            launch_gemm_nt<T>(V + rows * np, np, Vk, np, A + rows + k0 * ldA, ldA, rows, rem, DB, T(-1), T(1), false,
                              s);
    }
    // C = V V^T, lower; V[i][k] = 0 for k < i so tile row i0 starts its K loop at i0
    launch_gemm_nt_kskip<T>(C, np, V, np, V, np, np, np, np, s);
    g_prof = saved;
}

// ---------------------------------------------------------------------------------------
// gradient reduction
// ---------------------------------------------------------------------------------------
template <typename T, int NPER>
struct GradSmem {
    T xa[DC][BT];
    T xb[DC][BT];
    T per[NPER > 0 ? NPER * 4 : 1][DC][BT];
    double red[256];
};

// CROSS: rows from X (n), columns from Xb (nb), every tile (ntr row tiles), weights
// alpha_i beta_j - C_ij without doubling (the sparse likelihood, include/SparseLikelihood.h:317-340).
template <typename T, int NPER, bool CROSS = false>
__global__ __launch_bounds__(256) void lml_grad_kernel(KCanon<T> K, const T* __restrict__ X, const T* __restrict__ tab,
                                                       int64_t n, int d, const T* __restrict__ alpha,
                                                       const T* __restrict__ C, int64_t ldc, double* __restrict__ gout,
                                                       const T* __restrict__ Xb = nullptr,
                                                       const T* __restrict__ tabB = nullptr, int64_t nb = 0,
                                                       const T* __restrict__ beta = nullptr, int64_t ntr = 1) {
    __shared__ __attribute__((aligned(16))) GradSmem<T, NPER> sm;
    const T* __restrict__ Xc = CROSS ? Xb : X;
    const T* __restrict__ tc = CROSS ? tabB : tab;
    const T* __restrict__ bv = CROSS ? beta : alpha;
    const int64_t ncol = CROSS ? nb : n;
    int64_t ti, tj;
    if (CROSS) {
        ti = blockIdx.x % ntr;
        tj = blockIdx.x / ntr;
    } else {
        const int64_t b = blockIdx.x;
        int64_t i = (int64_t)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
        while ((i + 1) * (i + 2) / 2 <= b) i++;
        while (i * (i + 1) / 2 > b) i--;
        ti = i;
        tj = b - i * (i + 1) / 2;
    }
    const int64_t i0 = ti * BT, j0 = tj * BT;
    const int t = threadIdx.x;
    const int tx = t & 15, ty = t >> 4;

    T r2[4][4], s0[4][4], s1[4][4], f0[4][4], f1[4][4];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) r2[a][b] = s0[a][b] = s1[a][b] = f0[a][b] = f1[a][b] = T(0);
    const int64_t nd = n * (int64_t)d;
    for (int k0 = 0; k0 < d; k0 += DC) {
        const int64_t ndc = ncol * (int64_t)d;
        stage_chunk<T>(sm.xa, X, i0, n, d, k0);
        stage_chunk<T>(sm.xb, Xc, j0, ncol, d, k0);
#pragma unroll
        for (int p = 0; p < NPER; p++) {
            stage_chunk<T>(sm.per[4 * p + 0], tab + (2 * p) * nd, i0, n, d, k0);
            stage_chunk<T>(sm.per[4 * p + 1], tab + (2 * p + 1) * nd, i0, n, d, k0);
            stage_chunk<T>(sm.per[4 * p + 2], tc + (2 * p) * ndc, j0, ncol, d, k0);
            stage_chunk<T>(sm.per[4 * p + 3], tc + (2 * p + 1) * ndc, j0, ncol, d, k0);
        }
        __syncthreads();
        const int kmax = min(DC, d - k0);
        for (int k = 0; k < kmax; k++) {
            T xa[4], xb[4];
#pragma unroll
            for (int a = 0; a < 4; a++) xa[a] = sm.xa[k][tx * 4 + a];
#pragma unroll
            for (int b = 0; b < 4; b++) xb[b] = sm.xb[k][ty * 4 + b];
#pragma unroll
            for (int a = 0; a < 4; a++)
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    const T df = xa[a] - xb[b];
                    r2[a][b] = fma(df, df, r2[a][b]);
                }
#pragma unroll
            for (int p = 0; p < NPER; p++) {
                T sa[4], ca[4], sb[4], cb[4];
#pragma unroll
                for (int a = 0; a < 4; a++) {
                    sa[a] = sm.per[4 * p + 0][k][tx * 4 + a];
                    ca[a] = sm.per[4 * p + 1][k][tx * 4 + a];
                }
#pragma unroll
                for (int b = 0; b < 4; b++) {
                    sb[b] = sm.per[4 * p + 2][k][ty * 4 + b];
                    cb[b] = sm.per[4 * p + 3][k][ty * 4 + b];
                }
#pragma unroll
                for (int a = 0; a < 4; a++)
#pragma unroll
                    for (int b = 0; b < 4; b++) {
                        const T sn = fma(sa[a], cb[b], -ca[a] * sb[b]);
                        const T cs = fma(ca[a], cb[b], sa[a] * sb[b]);
                        const T df = xa[a] - xb[b];
                        if (p == 0) {
                            s0[a][b] = fma(sn, sn, s0[a][b]);
                            f0[a][b] = fma(T(2) * df, sn * cs, f0[a][b]);
                        } else {
                            s1[a][b] = fma(sn, sn, s1[a][b]);
                            f1[a][b] = fma(T(2) * df, sn * cs, f1[a][b]);
                        }
                    }
            }
        }
        __syncthreads();
    }

    double acc[MAX_LEAF][3];
#pragma unroll
    for (int l = 0; l < MAX_LEAF; l++) acc[l][0] = acc[l][1] = acc[l][2] = 0.0;

#pragma unroll
    for (int a = 0; a < 4; a++) {
        const int64_t gi = i0 + tx * 4 + a;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const int64_t gj = j0 + ty * 4 + b;
            if (gi >= n || gj >= ncol || (!CROSS && gi < gj)) continue;
            const T w = (alpha[gi] * bv[gj] - C[gi + gj * ldc]) * ((CROSS || gi == gj) ? T(1) : T(2));
            T lv[MAX_LEAF];
#pragma unroll
            for (int l = 0; l < MAX_LEAF; l++)
                lv[l] = (l < K.nleaf) ? leaf_value(K.leaf[l], r2[a][b], s0[a][b], s1[a][b]) : T(0);
#pragma unroll
            for (int l = 0; l < MAX_LEAF; l++) {
                if (l < K.nleaf) {
                    T adj = 0;
                    for (int tt = 0; tt < K.nterm; tt++) {
                        const unsigned msk = K.term_mask[tt];
                        if (!(msk & (1u << l))) continue;
                        T p = 1;
#pragma unroll
                        for (int l2 = 0; l2 < MAX_LEAF; l2++)
                            if (l2 != l && (msk & (1u << l2))) p *= lv[l2];
                        adj += p;
                    }
                    T g[3];
                    leaf_grad(K.leaf[l], r2[a][b], s0[a][b], s1[a][b], f0[a][b], f1[a][b], g);
                    const T wa = w * adj;
                    acc[l][0] += (double)(wa * g[0]);
                    acc[l][1] += (double)(wa * g[1]);
                    acc[l][2] += (double)(wa * g[2]);
                }
            }
        }
    }
    // workgroup reduction of the 3*nleaf partial sums into this workgroup's slot of gout (one
    // writer per value; lml_grad_sum_kernel adds the slots in a fixed order: the gradient is the
    // same bits on every call, which atomics did not give)
    for (int l = 0; l < K.nleaf; l++) {
        for (int q = 0; q < 3; q++) {
            double v = (q == 0) ? acc[l][0] : ((q == 1) ? acc[l][1] : acc[l][2]);
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
            if ((t & 63) == 0) sm.red[t >> 6] = v;
            __syncthreads();
            if (t == 0)
                gout[(int64_t)blockIdx.x * (MAX_LEAF * 3) + l * 3 + q] = (sm.red[0] + sm.red[1]) + (sm.red[2] + sm.red[3]);
            __syncthreads();
        }
    }
}

// acc[p] += sum over the workgroups' slots of value p, in a fixed order (block p: value p)
__global__ void lml_grad_sum_kernel(const double* __restrict__ part, int64_t nblk, double* __restrict__ acc) {
    __shared__ double red[256];
    const int p = blockIdx.x, t = threadIdx.x;
    double v = 0;
    for (int64_t b = t; b < nblk; b += 256) v += part[b * (MAX_LEAF * 3) + p];
    red[t] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) red[t] += red[t + o];
        __syncthreads();
    }
    if (t == 0) acc[p] += red[0];
}

// the per-workgroup slots: stream-ordered scratch (no device-wide synchronisation), summed into acc
struct GradSlots {
    double* p = nullptr;
    hipStream_t s;
    GradSlots(int64_t nblk, hipStream_t st) : s(st) {
        GPRX_HIP(hipMallocAsync((void**)&p, sizeof(double) * MAX_LEAF * 3 * (size_t)std::max<int64_t>(nblk, 1), s));
    }
    void finish(int nleaf, int64_t nblk, double* acc) {
        hipLaunchKernelGGL(lml_grad_sum_kernel, dim3((unsigned)(3 * nleaf)), dim3(256), 0, s, (const double*)p, nblk, acc);
    }
    ~GradSlots() { (void)hipFreeAsync(p, s); }
};

template <typename T>
void launch_lml_grad(const KCanon<T>& K, const T* X, const T* tab, int64_t n, int d, const T* alpha, const T* C,
                     int64_t ldc, double* acc, hipStream_t s) {
    const int64_t nt = (n + BT - 1) / BT;
    const unsigned grid = (unsigned)(nt * (nt + 1) / 2);
    if (grid == 0) return;
    ProfScope ps(KC_LML_GRAD, s, 0.0, (double)sizeof(T) * ((double)n * (n + 1) / 2 + (double)n * d));
    GradSlots slots(grid, s);
    if (K.nper == 0)
        hipLaunchKernelGGL((lml_grad_kernel<T, 0>), dim3(grid), dim3(256), 0, s, K, X, tab, n, d, alpha, C, ldc,
                           slots.p, X, tab, n, alpha, (int64_t)1);
    else if (K.nper == 1)
        hipLaunchKernelGGL((lml_grad_kernel<T, 1>), dim3(grid), dim3(256), 0, s, K, X, tab, n, d, alpha, C, ldc,
                           slots.p, X, tab, n, alpha, (int64_t)1);
    else
        hipLaunchKernelGGL((lml_grad_kernel<T, 2>), dim3(grid), dim3(256), 0, s, K, X, tab, n, d, alpha, C, ldc,
                           slots.p, X, tab, n, alpha, (int64_t)1);
    slots.finish(K.nleaf, grid, acc);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void launch_lml_grad_cross(const KCanon<T>& K, const T* Xa, const T* tabA, int64_t na, const T* Xb, const T* tabB,
                           int64_t nb, int d, const T* a, const T* b, const T* C, int64_t ldc, double* acc,
                           hipStream_t s) {
    const int64_t ntr = (na + BT - 1) / BT, ntc = (nb + BT - 1) / BT;
    if (ntr * ntc == 0) return;
    const unsigned grid = (unsigned)(ntr * ntc);
    ProfScope ps(KC_LML_GRAD, s, 0.0, (double)sizeof(T) * ((double)na * nb + (double)(na + nb) * d));
    GradSlots slots(grid, s);
    if (K.nper == 0)
        hipLaunchKernelGGL((lml_grad_kernel<T, 0, true>), dim3(grid), dim3(256), 0, s, K, Xa, tabA, na, d, a, C, ldc,
                           slots.p, Xb, tabB, nb, b, ntr);
    else if (K.nper == 1)
        hipLaunchKernelGGL((lml_grad_kernel<T, 1, true>), dim3(grid), dim3(256), 0, s, K, Xa, tabA, na, d, a, C, ldc,
                           slots.p, Xb, tabB, nb, b, ntr);
    else
        hipLaunchKernelGGL((lml_grad_kernel<T, 2, true>), dim3(grid), dim3(256), 0, s, K, Xa, tabA, na, d, a, C, ldc,
                           slots.p, Xb, tabB, nb, b, ntr);
    slots.finish(K.nleaf, grid, acc);
    GPRX_HIP(hipGetLastError());
}

#define GPRX_INST(T)                                                                                            \
    template void launch_lml_grad_cross<T>(const KCanon<T>&, const T*, const T*, int64_t, const T*, const T*,  \
                                           int64_t, int, const T*, const T*, const T*, int64_t, double*,      \
                                           hipStream_t);                                                       \
    template void launch_set_identity_pad<T>(T*, int64_t, int64_t, int64_t, hipStream_t);                      \
    template void launch_gemm_add_lower<T>(T*, int64_t, const T*, int64_t, int64_t, hipStream_t);              \
    template void launch_sym_fill<T>(T*, int64_t, int64_t, hipStream_t);                                       \
    template void launch_sum_partials<T>(T*, int64_t, int, hipStream_t);                                        \
    template void launch_spd_inverse_from_factor<T>(const T*, int64_t, int64_t, const T*, T*, T*, hipStream_t); \
    template void launch_lml_grad<T>(const KCanon<T>&, const T*, const T*, int64_t, int, const T*, const T*,   \
                                     int64_t, double*, hipStream_t);
GPRX_INST(double)
GPRX_INST(float)
#undef GPRX_INST

}  // namespace gprx
