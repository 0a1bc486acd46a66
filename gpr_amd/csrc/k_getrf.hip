// k_getrf.hip — LU with partial pivoting on gfx950: the fallback when K + sigma^2 I is not
// numerically positive definite.
//
// Reference semantics: the default InversionMethod is FullPivotLU, which is LAPACK's
// partial-pivot dgetrf_ + dgetri_ on the matrix cast to double (include/LAPACKUtils.h:38-56,
// 85-97, called from GaussianProcess::InvertKernelMatrix, lib/GaussianProcess.cpp:545-559);
// it inverts matrices a Cholesky rejects (e.g. the sigma = 0 fits of
// tests/GaussianProcessTest.cpp:44,86, tests/InversionMethodsTest.cpp:39).  libgprx factors
// with Cholesky (k_ptiles.hip) and, when that reports a non-positive pivot, refactors the
// same matrix here -- always in double, as the reference does for both scalar types -- and
// solves with the factors instead of forming the inverse.
//
// Blocked right-looking getrf, panel width 128 (the MFMA gemm tile):
//   panel    one workgroup factors the (np - k0) x 128 panel column by column: pivot search
//            (max |a|, lowest row on ties, as idamax), row swap inside the panel, scaling by
//            the reciprocal pivot (dgetf2), rank-1 update of the panel's remaining columns
//   laswp    the panel's swaps applied to every other column
//   U12      = L11^{-1} A12 by substitution (dtrsm), A22 -= L21 U12 on the MFMA gemm
//            (launch_gemm_nt, through a transposed copy of U12)
// Solves with m right-hand sides (column-major B): B = P B, then per 128-block a
// substitution with the diagonal block and a block update of the rest (forward with the
// unit-lower L, backward with U) -- no explicit block inverses anywhere, so the solve keeps
// LU's backward stability on the near-singular matrices this fallback is for.
#include "gprx_internal.h"

namespace gprx {

namespace lu {

constexpr int NB = 128;       // panel width = diagonal block edge
constexpr int PT = 1024;      // panel workgroup

// One panel: columns k0 .. k0 + NB of A (np x np, column-major, ld), rows k0 .. np.
// ipiv[j] = the (0-based) row swapped with row j; info: first column with a zero pivot
// (1-based, atomicMin).
__global__ __launch_bounds__(PT) void panel_kernel(double* __restrict__ A, int64_t ld, int64_t np, int64_t k0,
                                                   int* __restrict__ ipiv, int* __restrict__ info) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    double* sU = reinterpret_cast<double*>(smem_raw);        // pivot row segment (NB)
    double* sv = sU + NB;                                    // per-wave maxima (PT / 64)
    int* si = reinterpret_cast<int*>(sv + PT / 64);          // their rows
    int* sp = si + PT / 64;                                  // chosen pivot row
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    for (int c = 0; c < NB; c++) {
        const int64_t j = k0 + c;
        double* colj = A + j * ld;
        // ---- pivot search over rows j .. np: max |a|, lowest row on ties (idamax) -------
        double best = -1.0;
        int64_t bi = np;
        for (int64_t r = j + t; r < np; r += PT) {
            const double v = fabs(colj[r]);
            if (v > best) {  // rows visited in increasing order: strict > keeps the lowest
                best = v;
                bi = r;
            }
        }
        for (int off = 32; off > 0; off >>= 1) {
            const double ov = __shfl_xor(best, off);
            const int64_t oi = __shfl_xor(bi, off);
            if (ov > best || (ov == best && oi < bi)) {
                best = ov;
                bi = oi;
            }
        }
        if (lane == 0) {
            sv[w] = best;
            si[w] = (int)bi;
        }
        __syncthreads();
        if (t == 0) {
            double b = sv[0];
            int bii = si[0];
            for (int u = 1; u < PT / 64; u++)
                if (sv[u] > b || (sv[u] == b && si[u] < bii)) {
                    b = sv[u];
                    bii = si[u];
                }
            if (bii >= np) bii = (int)j;
            *sp = bii;
            ipiv[j] = bii;
        }
        __syncthreads();
        const int64_t p = *sp;
        // ---- swap rows j and p inside the panel ---------------------------------------
        if (p != j && t < NB) {
            double* cc = A + (k0 + t) * ld;
            const double a = cc[j];
            cc[j] = cc[p];
            cc[p] = a;
        }
        __syncthreads();
        const double piv = colj[j];
        if (piv == 0.0) {
            if (t == 0) atomicMin(info, (int)(j + 1));
        } else {
            const double rp = 1.0 / piv;
            for (int64_t r = j + 1 + t; r < np; r += PT) colj[r] *= rp;
        }
        if (t < NB) sU[t] = (t > c) ? A[j + (k0 + t) * ld] : 0.0;
        __syncthreads();
        // ---- rank-1 update of the panel's remaining columns ----------------------------
        if (c + 1 < NB && piv != 0.0) {
            for (int64_t r = j + 1 + t; r < np; r += PT) {
                const double l = colj[r];
                for (int cc = c + 1; cc < NB; cc++) A[r + (k0 + cc) * ld] = fma(-l, sU[cc], A[r + (k0 + cc) * ld]);
            }
        }
        __syncthreads();
    }
}

// the swaps of rows k0 .. k0 + NB applied (in order) to the columns outside the panel
__global__ void laswp_kernel(double* __restrict__ A, int64_t ld, int64_t np, int64_t k0, const int* __restrict__ ipiv) {
    int64_t col = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (col >= np - NB) return;
    if (col >= k0) col += NB;  // skip the panel's own columns
    double* cc = A + col * ld;
    for (int jj = 0; jj < NB; jj++) {
        const int64_t j = k0 + jj, p = ipiv[j];
        if (p != j) {
            const double a = cc[j];
            cc[j] = cc[p];
            cc[p] = a;
        }
    }
}

// out (ncol x NB, ld ldo) = A[r0 .. r0 + NB, c0 .. c0 + ncol]^T  (32 x 32 tiles through LDS)
// back = true: the other direction, A-block = in^T.
__global__ __launch_bounds__(256) void transpose_block_kernel(double* __restrict__ A, int64_t ld, int64_t r0, int64_t c0,
                                                              int64_t ncol, double* __restrict__ T, int64_t ldt,
                                                              int back) {
    __shared__ double sh[32][33];
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
    const int64_t bi = blockIdx.x * 32;  // rows of the NB-row block
    const int64_t bj = blockIdx.y * 32;  // columns (ncol)
    if (!back) {
        for (int k = 0; k < 4; k++) {
            const int64_t r = bi + tx, c = bj + ty + 8 * k;
            if (c < ncol) sh[ty + 8 * k][tx] = A[r0 + r + (c0 + c) * ld];
        }
        __syncthreads();
        for (int k = 0; k < 4; k++) {
            const int64_t c = bj + tx, r = bi + ty + 8 * k;  // T[c][r]
            if (c < ncol) T[c + r * ldt] = sh[tx][ty + 8 * k];
        }
    } else {
        for (int k = 0; k < 4; k++) {
            const int64_t c = bj + tx, r = bi + ty + 8 * k;
            if (c < ncol) sh[ty + 8 * k][tx] = T[c + r * ldt];
        }
        __syncthreads();
        for (int k = 0; k < 4; k++) {
            const int64_t r = bi + tx, c = bj + ty + 8 * k;
            if (c < ncol) A[r0 + r + (c0 + c) * ld] = sh[tx][ty + 8 * k];
        }
    }
}

// ---- solves ---------------------------------------------------------------------------------
// B (np x m, column-major, ldb) <- rows of Y (n x m row-major, in T), zero padding rows
template <typename T>
__global__ void rhs_from_rows_kernel(const T* __restrict__ Y, int64_t n, int m, double* __restrict__ B, int64_t ldb,
                                     int64_t np) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= np * m) return;
    const int64_t r = e % np, c = e / np;
    B[r + c * ldb] = (r < n) ? (double)Y[r * m + c] : 0.0;
}

// rows of X (n x m row-major, T) <- B
template <typename T>
__global__ void rows_from_rhs_kernel(const double* __restrict__ B, int64_t ldb, int64_t n, int m, T* __restrict__ X) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= n * m) return;
    const int64_t r = e / m, c = e % m;
    X[e] = (T)B[r + c * ldb];
}

// B = P B: the row swaps of the whole factorisation in order, one thread per column
__global__ void apply_pivots_kernel(double* __restrict__ B, int64_t ldb, int64_t np, int m, const int* __restrict__ ipiv) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= m) return;
    double* b = B + (int64_t)c * ldb;
    for (int64_t j = 0; j < np; j++) {
        const int64_t p = ipiv[j];
        if (p != j) {
            const double a = b[j];
            b[j] = b[p];
            b[p] = a;
        }
    }
}

constexpr int SC = 8;  // right-hand sides per workgroup in the solve kernels

// B[r0 .. r0 + NB, :] <- T^{-1} B[r0 .. r0 + NB, :] by substitution with the diagonal block
// T = A[r0 .., r0 ..] (upper: U with its diagonal; else unit lower L), as dtrsm does: explicit
// inverses of the blocks would lose backward stability when U is ill conditioned (the
// singular-kernel fits this fallback exists for).  One thread per row, SC right-hand sides
// per workgroup; each step publishes one solved row through LDS.
__global__ __launch_bounds__(NB) void tri_solve_kernel(const double* __restrict__ A, int64_t ld, int64_t r0,
                                                       double* __restrict__ B, int64_t ldb, int m, int upper) {
    __shared__ double sx[SC];
    const int k = threadIdx.x, c0 = blockIdx.x * SC;
    double b[SC];
    for (int u = 0; u < SC; u++) b[u] = (c0 + u < m) ? B[r0 + k + (int64_t)(c0 + u) * ldb] : 0.0;
    const double* Ad = A + r0 + r0 * ld;  // the diagonal block, column-major
    if (upper) {
        const double ukk = Ad[k + (int64_t)k * ld];
        for (int i = NB - 1; i >= 0; i--) {
            if (k == i)
                for (int u = 0; u < SC; u++) {
                    b[u] = b[u] / ukk;
                    sx[u] = b[u];
                }
            __syncthreads();
            if (k < i) {
                const double a = Ad[k + (int64_t)i * ld];
                for (int u = 0; u < SC; u++) b[u] = fma(-a, sx[u], b[u]);
            }
            __syncthreads();
        }
    } else {
        for (int i = 0; i < NB; i++) {
            if (k == i)
                for (int u = 0; u < SC; u++) sx[u] = b[u];
            __syncthreads();
            if (k > i) {
                const double a = Ad[k + (int64_t)i * ld];
                for (int u = 0; u < SC; u++) b[u] = fma(-a, sx[u], b[u]);
            }
            __syncthreads();
        }
    }
    for (int u = 0; u < SC; u++)
        if (c0 + u < m) B[r0 + k + (int64_t)(c0 + u) * ldb] = b[u];
}

// B[r, :] -= sum_k A[r, c0 + k] B[c0 + k, :] for r in [rb, re)
__global__ __launch_bounds__(256) void block_update_kernel(const double* __restrict__ A, int64_t ld,
                                                           double* __restrict__ B, int64_t ldb, int64_t rb, int64_t re,
                                                           int64_t c0, int m) {
    __shared__ double sb[SC][NB];
    const int t = threadIdx.x, cg = blockIdx.y * SC;
    for (int e = t; e < SC * NB; e += 256) {
        const int cc = e / NB, k = e % NB;
        sb[cc][k] = (cg + cc < m) ? B[c0 + k + (int64_t)(cg + cc) * ldb] : 0.0;
    }
    __syncthreads();
    const int64_t r = rb + (int64_t)blockIdx.x * 256 + t;
    if (r >= re) return;
    double acc[SC];
    for (int u = 0; u < SC; u++) acc[u] = 0.0;
    for (int k = 0; k < NB; k++) {
        const double a = A[r + (c0 + k) * ld];
        for (int u = 0; u < SC; u++) acc[u] = fma(a, sb[u][k], acc[u]);
    }
    for (int u = 0; u < SC; u++)
        if (cg + u < m) B[r + (int64_t)(cg + u) * ldb] -= acc[u];
}

// out[0] = sum_{i<n} log |U_ii|, out[1] = sign of det (the row swaps and the signs of U_ii),
// out[2] = 1 if some U_ii == 0
__global__ __launch_bounds__(256) void logdet_kernel(const double* __restrict__ A, int64_t ld, int64_t n,
                                                     const int* __restrict__ ipiv, double* __restrict__ out) {
    __shared__ double sl[256];
    __shared__ int sn[256], sz[256];
    const int t = threadIdx.x;
    double l = 0.0;
    int neg = 0, zero = 0;
    for (int64_t i = t; i < n; i += 256) {
        const double u = A[i + i * ld];
        l += log(fabs(u));
        neg += (u < 0.0) + (ipiv[i] != i);
        zero |= (u == 0.0);
    }
    sl[t] = l;
    sn[t] = neg;
    sz[t] = zero;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) {
            sl[t] += sl[t + o];
            sn[t] += sn[t + o];
            sz[t] |= sz[t + o];
        }
        __syncthreads();
    }
    if (t == 0) {
        out[0] = sl[0];
        out[1] = (sn[0] & 1) ? -1.0 : 1.0;
        out[2] = sz[0] ? 1.0 : 0.0;
    }
}

// out[i] = kab[i] - sum_j Ka[j, i] W[j, i]  (column dot products, one workgroup per column)
template <typename T>
__global__ __launch_bounds__(256) void coldot_kernel(const double* __restrict__ Ka, const double* __restrict__ W,
                                                     int64_t ld, int64_t n, const T* __restrict__ kab,
                                                     T* __restrict__ out) {
    __shared__ double red[256];
    const int64_t c = blockIdx.x;
    double s = 0.0;
    for (int64_t j = threadIdx.x; j < n; j += 256) s = fma(Ka[j + c * ld], W[j + c * ld], s);
    red[threadIdx.x] = s;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) out[c] = (T)((double)kab[c] - red[0]);
}

}  // namespace lu

static size_t lu_panel_lds() { return sizeof(double) * (lu::NB + lu::PT / 64) + sizeof(int) * (lu::PT / 64 + 4); }

// In-place LU with partial pivoting of the np x np column-major A (np a multiple of 128,
// padding rows/columns the identity).  Ut: np x 128 scratch.  info: device int (INT_MAX = no
// zero pivot).
void lu_factor(double* A, int64_t ld, int64_t np, int* ipiv, int* info, double* Ut, hipStream_t s) {
    using namespace lu;
    GPRX_REQUIRE(np % NB == 0, GPRX_ERR_ARG, "lu_factor: np must be a multiple of 128");
    ProfScope ps(KC_OTHER, s, 2.0 / 3.0 * (double)np * np * np, 0.0);
    for (int64_t k0 = 0; k0 < np; k0 += NB) {
        hipLaunchKernelGGL(panel_kernel, dim3(1), dim3(PT), lu_panel_lds(), s, A, ld, np, k0, ipiv, info);
        if (np > NB)
            hipLaunchKernelGGL(laswp_kernel, dim3((unsigned)((np - NB + 255) / 256)), dim3(256), 0, s, A, ld, np, k0,
                               (const int*)ipiv);
        const int64_t rest = np - k0 - NB;
        if (rest <= 0) continue;
        // U12 = L11^{-1} A12 in place (substitution, as dgetrf's dtrsm), then its transpose Ut
        // as the gemm_nt operand: A22 -= L21 U12 = L21 Ut^T on the MFMA tile gemm
        hipLaunchKernelGGL(tri_solve_kernel, dim3((unsigned)((rest + SC - 1) / SC)), dim3(NB), 0, s, (const double*)A,
                           ld, k0, A + (k0 + NB) * ld, ld, (int)rest, 0);
        const dim3 tg((unsigned)(NB / 32), (unsigned)((rest + 31) / 32));
        hipLaunchKernelGGL(transpose_block_kernel, tg, dim3(256), 0, s, A, ld, k0, k0 + NB, rest, Ut, rest, 0);
        launch_gemm_nt<double>(A + (k0 + NB) + (k0 + NB) * ld, ld, A + (k0 + NB) + k0 * ld, ld, Ut, rest, rest, rest,
                               NB, -1.0, 1.0, false, s);
    }
    GPRX_HIP(hipGetLastError());
}

// B (np x m, column-major, ldb) <- A^{-1} B with the factors of lu_factor
void lu_solve(const double* A, int64_t ld, int64_t np, const int* ipiv, double* B, int64_t ldb, int m, hipStream_t s) {
    using namespace lu;
    if (m <= 0) return;
    hipLaunchKernelGGL(apply_pivots_kernel, dim3((unsigned)((m + 63) / 64)), dim3(64), 0, s, B, ldb, np, m, ipiv);
    const unsigned gc = (unsigned)((m + SC - 1) / SC);
    const int64_t nbk = np / NB;
    for (int64_t kb = 0; kb < nbk; kb++) {
        const int64_t r0 = kb * NB;
        hipLaunchKernelGGL(tri_solve_kernel, dim3(gc), dim3(NB), 0, s, A, ld, r0, B, ldb, m, 0);
        const int64_t rb = r0 + NB;
        if (rb < np)
            hipLaunchKernelGGL(block_update_kernel, dim3((unsigned)((np - rb + 255) / 256), gc), dim3(256), 0, s, A, ld,
                               B, ldb, rb, np, r0, m);
    }
    for (int64_t kb = nbk - 1; kb >= 0; kb--) {
        const int64_t r0 = kb * NB;
        hipLaunchKernelGGL(tri_solve_kernel, dim3(gc), dim3(NB), 0, s, A, ld, r0, B, ldb, m, 1);
        if (r0 > 0)
            hipLaunchKernelGGL(block_update_kernel, dim3((unsigned)((r0 + 255) / 256), gc), dim3(256), 0, s, A, ld, B,
                               ldb, (int64_t)0, r0, r0, m);
    }
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void lu_rhs_from_rows(const T* Y, int64_t n, int m, double* B, int64_t ldb, int64_t np, hipStream_t s) {
    const int64_t e = np * m;
    hipLaunchKernelGGL(lu::rhs_from_rows_kernel<T>, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, Y, n, m, B, ldb,
                       np);
}

template <typename T>
void lu_rows_from_rhs(const double* B, int64_t ldb, int64_t n, int m, T* X, hipStream_t s) {
    const int64_t e = n * m;
    if (e <= 0) return;
    hipLaunchKernelGGL(lu::rows_from_rhs_kernel<T>, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, B, ldb, n, m,
                       X);
}

void lu_logdet(const double* A, int64_t ld, int64_t n, const int* ipiv, double* out, hipStream_t s) {
    hipLaunchKernelGGL(lu::logdet_kernel, dim3(1), dim3(256), 0, s, A, ld, n, ipiv, out);
}

template <typename T>
void lu_coldot(const double* Ka, const double* W, int64_t ld, int64_t n, int64_t q, const T* kab, T* out,
               hipStream_t s) {
    if (q <= 0) return;
    hipLaunchKernelGGL(lu::coldot_kernel<T>, dim3((unsigned)q), dim3(256), 0, s, Ka, W, ld, n, kab, out);
}

#define GPRX_LU_INST(T)                                                                                  \
    template void lu_rhs_from_rows<T>(const T*, int64_t, int, double*, int64_t, int64_t, hipStream_t);   \
    template void lu_rows_from_rhs<T>(const double*, int64_t, int64_t, int, T*, hipStream_t);            \
    template void lu_coldot<T>(const double*, const double*, int64_t, int64_t, int64_t, const T*, T*, hipStream_t);
GPRX_LU_INST(double)
GPRX_LU_INST(float)
#undef GPRX_LU_INST

}  // namespace gprx
