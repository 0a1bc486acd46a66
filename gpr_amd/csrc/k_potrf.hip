// k_potrf.hip — Cholesky factorisation and triangular solves on gfx950.
//
// Replaces the reference's factorise/invert step, lapack::lu_invert -> dgetrf_+dgetri_
// (include/LAPACKUtils.h:38-56, 85-97, the default FullPivotLU branch of
// GaussianProcess::InvertKernelMatrix, lib/GaussianProcess.cpp:545-559) and the product
// alpha = C*Y (lib/GaussianProcess.cpp:661), with
//     K + sigma^2 I = L L^T      (right-looking blocked potrf, 128-wide blocks)
//     z = L^{-1} Y               (fused: Y^T rides along as extra rows of the matrix)
//     alpha = L^{-T} z           (blocked back substitution)
//
// Per 128-column block k:
//   diag_potrf_kernel  one workgroup factors the 128x128 diagonal block in LDS (blocked
//                      Crout, 8-wide column blocks) and forms its inverse Linv_k;
//   gemm_nt (trsm)     L_ik = A_ik Linv_k^T for every row block below (in place);
//   gemm_nt (syrk)     A_ij -= L_ik L_jk^T on the lower trailing matrix.
// gemm_nt is an LDS double-buffered MFMA kernel: v_mfma_f64_16x16x4_f64 (fp64) or
// v_mfma_f32_16x16x4_f32 (fp32), 128x128 output tile per 256-thread workgroup, 4 waves of
// 64x64, K staged 16 deep.  The dense fp64 matrix peak of MI355X is 78.6 TFLOP/s.
#include "gprx_internal.h"

#include <rccl/rccl.h>

#include <climits>
#include <cstdlib>

namespace gprx {

// ======================================================================================
// Diagonal block: factor + inverse, one workgroup of 256 threads.
//
// The 128x128 block lives in REGISTERS as a square image S: the lower triangle holds A
// (becoming L), the strict upper triangle the rows of B = L^{-T} (its diagonal in Bd).  B
// comes from appending the identity below A: its rows ride along the elimination and end as
// I L^{-T}; being upper triangular they fit the unused half exactly.  Thread t owns a fixed
// 4-row x 16-column block (two 8-column blocks): wave w holds columns 32w.., lane>>5 picks
// the 16-column half, lane&31 the row block.  Right-looking over 8-column steps J:
//   1  128 threads (waves 0-1, one row each) factor the 8x8 pivot redundantly (rsq +
//      Newton, no divide) and solve their row x = v Ld^{-T} (A rows below J: L panel; B rows
//      above J; pivot rows: identity rows), reading v from the LDS column panel sV that the
//      owners of J published, writing x to sP (and Ld to sLd);
//   2  every thread with trailing columns applies S -= x_r x_c^T to them, unmasked: entries
//      right of the diagonal in rows not yet reached are scratch and are zeroed when their
//      rows become pivot rows (their identity rows are still zero there).  The owners of J
//      take their final values from sP/sLd; the owners of the next column block publish it.
// Two barriers per step, 17 KB of LDS and <= 256 VGPRs, so the kernel fits on a CU next to
// one trailing-update GEMM workgroup (it runs concurrently with them on the panel stream).
// All register arrays use compile-time indices.
// ======================================================================================
constexpr int DT = 256;      // threads of the diagonal kernel
constexpr int SPL = DB + 4;  // panel row stride (elements)

// 1/sqrt(x) to full precision: hardware estimate + Newton steps (no divide on the chain)
__device__ __forceinline__ double rsqrt_full(double x) {
    double y = __builtin_amdgcn_rsq(x);
    const double h = 0.5 * x;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}
__device__ __forceinline__ float rsqrt_full(float x) {
    float y = __builtin_amdgcn_rsqf(x);
    const float h = 0.5f * x;
    y = y * fmaf(-h * y, y, 1.5f);
    return y;
}

template <typename T, bool PROF = false>
__global__ __launch_bounds__(DT) __attribute__((amdgpu_num_vgpr(296))) void diag_potrf_kernel(
    T* __restrict__ A, int64_t ld, T* __restrict__ Linv, int* __restrict__ info, int64_t col0,
    long long* __restrict__ prof = nullptr) {
    long long tp0 = 0, tp1 = 0, tph1 = 0, tph2 = 0, tmark = 0;
    if (PROF) tp0 = __builtin_amdgcn_s_memtime();
    __shared__ __attribute__((aligned(16))) T sV[8][SPL];  // v of column block J (column-major)
    __shared__ __attribute__((aligned(16))) T sP[8][SPL];  // solved x
    __shared__ T sLdW[2][8][9];                             // pivot factor (+ 1/diag), per wave
    T(*sLd)[9] = sLdW[0];

    const int t = threadIdx.x, w = t >> 6, l = t & 63;
    const int R0 = (l & 31) * 4;
    const int C0 = 32 * w + 16 * (l >> 5);  // first of 16 columns
    const int cb0 = C0 >> 3;                 // its first 8-column block

    T S[4][16];
    T Bd[4];
    {
        const T* Ai = A + R0 + (int64_t)C0 * ld;
#pragma unroll
        for (int b = 0; b < 16; b++)
#pragma unroll
            for (int a = 0; a < 4; a++) S[a][b] = Ai[a + (int64_t)b * ld];
    }
#pragma unroll
    for (int a = 0; a < 4; a++) Bd[a] = T(1);
    if (cb0 == 0) {
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 8; b++) sV[b][R0 + a] = S[a][b];
    }
    __syncthreads();
    if (PROF) tp1 = tmark = __builtin_amdgcn_s_memtime();

    int fail_col = -1;
    for (int j0 = 0; j0 < DB; j0 += 8) {
        const int jn = j0 + 8, J = j0 >> 3;
        // ---- 1: pivot factor + row solves, one row per thread ------------------------------
        if (t < DB) {
            // every lane of waves 0-1 factors the pivot and keeps it in its wave's own LDS copy
            // (identical values, no cross-wave sync), so the row solve reads it back instead
            // of holding it in registers next to S
            T(*myLd)[9] = sLdW[w];
            {
                T Ld[8][8];
#pragma unroll
                for (int c = 0; c < 8; c++) {
                    T dsum = sV[c][j0 + c];
#pragma unroll
                    for (int k = 0; k < c; k++) dsum = fma(-Ld[c][k], Ld[c][k], dsum);
                    if (!(dsum > T(0)) && fail_col < 0) fail_col = j0 + c;
                    const T ri = rsqrt_full(dsum);
                    Ld[c][c] = dsum * ri;
                    myLd[c][8] = ri;
                    myLd[c][c] = Ld[c][c];
#pragma unroll
                    for (int r = c + 1; r < 8; r++) {
                        T v = sV[c][j0 + r];
#pragma unroll
                        for (int k = 0; k < c; k++) v = fma(-Ld[r][k], Ld[c][k], v);
                        Ld[r][c] = v * ri;
                        myLd[r][c] = Ld[r][c];
                    }
                }
            }
            const int row = t;
            const bool piv = row >= j0 && row < jn;
            T x[8];
#pragma unroll
            for (int q = 0; q < 8; q++) {
                T v = piv ? ((row - j0 == q) ? T(1) : T(0)) : sV[q][row];
#pragma unroll
                for (int q2 = 0; q2 < q; q2++) v = fma(-x[q2], myLd[q][q2], v);
                x[q] = v * myLd[q][8];
            }
#pragma unroll
            for (int q = 0; q < 8; q++) sP[q][row] = x[q];
        }
        __syncthreads();
        if (PROF) {
            const long long tn = __builtin_amdgcn_s_memtime();
            tph1 += tn - tmark;
            tmark = tn;
        }
        // ---- 2: final values of column block J; rank-8 update of the trailing blocks -------
        const bool pivrows = R0 >= j0 && R0 < jn;
        bool act[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int cb = cb0 + h, c0h = 8 * cb;
            act[h] = c0h >= jn && (R0 < jn || R0 + 3 >= c0h);
            if (cb == J) {
                if (pivrows) {
#pragma unroll
                    for (int a = 0; a < 4; a++) {
                        const int p = R0 + a - j0;
#pragma unroll
                        for (int q = 0; q < 8; q++) {
                            const T xq = sP[q][R0 + a];
                            S[a][8 * h + q] = (q <= p) ? sLd[p][q] : xq;
                            if (q == p) Bd[a] = xq;
                        }
                    }
                } else {
#pragma unroll
                    for (int a = 0; a < 4; a++)
#pragma unroll
                        for (int q = 0; q < 8; q++) S[a][8 * h + q] = sP[q][R0 + a];
                }
            }
            if (act[h] && pivrows) {  // identity rows entering B: still zero right of the pivot
#pragma unroll
                for (int a = 0; a < 4; a++)
#pragma unroll
                    for (int b = 0; b < 8; b++) S[a][8 * h + b] = T(0);
            }
        }
        if (act[0] || act[1]) {
#pragma unroll 2
            for (int q = 0; q < 8; q++) {
                T u[4];
#pragma unroll
                for (int a = 0; a < 4; a++) u[a] = sP[q][R0 + a];
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    if (!act[h]) continue;
                    T v[8];
#pragma unroll
                    for (int b = 0; b < 8; b++) v[b] = sP[q][C0 + 8 * h + b];
#pragma unroll
                    for (int a = 0; a < 4; a++)
#pragma unroll
                        for (int b = 0; b < 8; b++) S[a][8 * h + b] = fma(-u[a], v[b], S[a][8 * h + b]);
                }
            }
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
            if (jn < DB && cb0 + h == (jn >> 3)) {  // publish the next column block
#pragma unroll
                for (int a = 0; a < 4; a++)
#pragma unroll
                    for (int b = 0; b < 8; b++) sV[b][R0 + a] = S[a][8 * h + b];
            }
        }
        __syncthreads();
        if (PROF) {
            const long long tn = __builtin_amdgcn_s_memtime();
            tph2 += tn - tmark;
            tmark = tn;
        }
    }
    if (fail_col >= 0 && t == 0) atomicMin(info, (int)(col0 + fail_col + 1));

    // L (lower) in place; Linv = B^T: row r of B goes to column r of Linv (zeros above its
    // diagonal), 16 consecutive elements per thread and row.  The opaque copies keep the
    // compiler from hoisting these addresses above the loop (they would pin ~40 registers).
    int64_t ldo = ld;
    T* Ao = A;
    T* Lo = Linv;
    int R0o = R0, C0o = C0;
    asm volatile("" : "+s"(ldo), "+s"(Ao), "+s"(Lo), "+v"(R0o), "+v"(C0o));
#pragma unroll
    for (int b = 0; b < 16; b++) {
        const int c = C0o + b;
#pragma unroll
        for (int a = 0; a < 4; a++)
            if (R0o + a >= c) Ao[R0o + a + (int64_t)c * ldo] = S[a][b];
    }
#pragma unroll
    for (int a = 0; a < 4; a++) {
        const int r = R0o + a;
#pragma unroll
        for (int b = 0; b < 16; b++) {
            const int c = C0o + b;
            Lo[c + r * DB] = (r < c) ? S[a][b] : ((r == c) ? Bd[a] : T(0));
        }
    }
    if (PROF) __syncthreads();
    if (PROF && t == 0) {
        const long long te = __builtin_amdgcn_s_memtime();
        prof[0] += tp1 - tp0;
        prof[1] += tph1;
        prof[2] += tph2;
        prof[3] += te - tmark;
        prof[4] += te - tp0;
    }
}

// ======================================================================================
// MFMA GEMM  C = beta C + alpha A B^T   (all column-major, sizes multiples of 128 / 16)
// ======================================================================================
constexpr int BK = 16;
constexpr int PADT = 16;

typedef double d4_t __attribute__((ext_vector_type(4)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef double d2_t __attribute__((ext_vector_type(2)));
typedef float f4v_t __attribute__((ext_vector_type(4)));

template <typename T>
struct MfmaTraits;
template <>
struct MfmaTraits<double> {
    typedef d4_t acc_t;
    typedef d2_t vec_t;  // 16-byte global/LDS move
    static constexpr int VEC = 2;
    __device__ static inline acc_t mma(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // output row (within the 16x16 block) of accumulator register `reg` for lane group lk
    __device__ static inline int orow(int lk, int reg) { return lk + 4 * reg; }
};
template <>
struct MfmaTraits<float> {
    typedef f4_t acc_t;
    typedef f4v_t vec_t;
    static constexpr int VEC = 4;
    __device__ static inline acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    __device__ static inline int orow(int lk, int reg) { return 4 * lk + reg; }
};

// TM = 128: 4 waves of 64x64 (4x4 MFMA blocks each) -- the bulk trailing updates.
// TM = 64:  4 waves of 32x32 (2x2 blocks) -- skinny panel-chain GEMMs (trsm, in-panel and
//           look-ahead updates), 4x the workgroups so the short critical-path launches
//           spread over the whole chip instead of running 64-128 long tiles.
template <typename T, bool LOWER, bool BETA, bool KSKIP, int TM = 128>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(T* __restrict__ C, int64_t ldc, const T* __restrict__ A,
                                                         int64_t lda, const T* __restrict__ B, int64_t ldb,
                                                         int64_t K, T alpha, T beta, int64_t ntm, int64_t ntn,
                                                         int64_t cstride = 0) {
    typedef MfmaTraits<T> Tr;
    typedef typename Tr::acc_t acc_t;
    typedef typename Tr::vec_t vec_t;
    constexpr int VEC = Tr::VEC;
    constexpr int SR = TM + PADT;       // LDS row (one k) length in elements
    constexpr int TPC = TM / VEC;       // threads per staged column
    constexpr int CPP = 256 / TPC;      // columns per pass
    constexpr int PASSES = (BK + CPP - 1) / CPP;
    constexpr int NB = TM / 32;         // 16x16 MFMA blocks per wave edge (4 or 2)
    constexpr int WT = TM / 2;          // wave tile edge

    // split-K: blockIdx.y = p works on k in [p*K, (p+1)*K) and writes its own C + p*cstride
    if (gridDim.y > 1) {
        const int64_t p = blockIdx.y;
        A += p * K * lda;
        B += p * K * ldb;
        C += p * cstride;
    }

    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* sA = reinterpret_cast<T*>(smem_raw);            // [2][BK][SR]
    T* sB = sA + 2 * BK * SR;                            // [2][BK][SR]

    // ---- tile coordinates ---------------------------------------------------------------
    int64_t ti, tj;
    {
        const int64_t b = blockIdx.x;
        if (LOWER) {
            const int64_t tri = ntn * (ntn + 1) / 2;
            if (b < tri) {
                int64_t i = (int64_t)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
                while ((i + 1) * (i + 2) / 2 <= b) i++;
                while (i * (i + 1) / 2 > b) i--;
                ti = i;
                tj = b - i * (i + 1) / 2;
            } else {
                const int64_t b2 = b - tri;
                ti = ntn + b2 / ntn;
                tj = b2 % ntn;
            }
        } else {
            ti = b % ntm;
            tj = b / ntm;
        }
    }
    const int64_t i0 = ti * TM, j0 = tj * TM;
    // KSKIP: both operands are zero left of column i0 (C = V V^T with V upper triangular)
    const int64_t kbeg = KSKIP ? i0 : 0;
    const T* Ablk = A + i0 + kbeg * lda;
    const T* Bblk = B + j0 + kbeg * ldb;

    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    const int wr = w >> 1, wc = w & 1;
    const int lr = lane & 15, lk = lane >> 4;

    // staging coordinates
    const int st_row = (t % TPC) * VEC;
    const int st_col = t / TPC;

    vec_t ra[PASSES], rb[PASSES];
    auto gload = [&](int64_t k0) {
#pragma unroll
        for (int p = 0; p < PASSES; p++) {
            const int64_t kk = k0 + st_col + p * CPP;
            if (st_col + p * CPP < BK) {
                ra[p] = *reinterpret_cast<const vec_t*>(Ablk + st_row + kk * lda);
                rb[p] = *reinterpret_cast<const vec_t*>(Bblk + st_row + kk * ldb);
            }
        }
    };
    auto lstore = [&](int buf) {
        T* a = sA + buf * BK * SR;
        T* bb = sB + buf * BK * SR;
#pragma unroll
        for (int p = 0; p < PASSES; p++) {
            const int kk = st_col + p * CPP;
            if (kk < BK) {
                *reinterpret_cast<vec_t*>(a + kk * SR + st_row) = ra[p];
                *reinterpret_cast<vec_t*>(bb + kk * SR + st_row) = rb[p];
            }
        }
    };

    acc_t acc[NB][NB];
#pragma unroll
    for (int x = 0; x < NB; x++)
#pragma unroll
        for (int y = 0; y < NB; y++) acc[x][y] = acc_t{0};

    const int nstage = (int)((K - kbeg) / BK);
    gload(0);
    lstore(0);
    __syncthreads();
    for (int sidx = 0; sidx < nstage; sidx++) {
        const int buf = sidx & 1;
        if (sidx + 1 < nstage) gload((int64_t)(sidx + 1) * BK);
        const T* a = sA + buf * BK * SR;
        const T* bb = sB + buf * BK * SR;
#pragma unroll
        for (int kq = 0; kq < BK / 4; kq++) {
            const int kr = kq * 4 + lk;
            T fa[NB], fb[NB];
#pragma unroll
            for (int x = 0; x < NB; x++) fb[x] = bb[kr * SR + wc * WT + x * 16 + lr];  // MFMA A: our columns
#pragma unroll
            for (int y = 0; y < NB; y++) fa[y] = a[kr * SR + wr * WT + y * 16 + lr];   // MFMA B: our rows
#pragma unroll
            for (int x = 0; x < NB; x++)
#pragma unroll
                for (int y = 0; y < NB; y++) acc[x][y] = Tr::mma(fb[x], fa[y], acc[x][y]);
        }
        if (sidx + 1 < nstage) lstore(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue: acc[x][y][reg] = C(i = ... y*16 + lr, j = ... x*16 + orow(lk, reg)) ----
    const bool diag_tile = LOWER && (ti == tj);
#pragma unroll
    for (int x = 0; x < NB; x++) {
#pragma unroll
        for (int reg = 0; reg < 4; reg++) {
            const int jl = wc * WT + x * 16 + Tr::orow(lk, reg);
            T* ccol = C + (j0 + jl) * ldc + i0;
#pragma unroll
            for (int y = 0; y < NB; y++) {
                const int il = wr * WT + y * 16 + lr;
                if (diag_tile && il < jl) continue;
                T v = alpha * acc[x][y][reg];
                if (BETA) v = fma(beta, ccol[il], v);
                ccol[il] = v;
            }
        }
    }
}

template <typename T, int TM = 128>
static size_t gemm_lds_bytes() {
    return sizeof(T) * 4 * BK * (TM + PADT);
}

template <typename T, int TM>
static void gemm_launch(T* C, int64_t ldc, const T* A, int64_t lda, const T* B, int64_t ldb, int64_t M, int64_t N,
                        int64_t K, T alpha, T beta, bool lower, hipStream_t s) {
    const int64_t ntm = M / TM, ntn = N / TM;
    const int64_t ntiles = lower ? ntn * (ntn + 1) / 2 + (ntm - ntn) * ntn : ntm * ntn;
    const size_t lds = gemm_lds_bytes<T, TM>();
    const bool use_beta = beta != T(0);
#define GPRX_GEMM(L, Bt)                                                                                  \
    do {                                                                                                  \
        static bool attr_done = false;                                                                    \
        if (!attr_done) {                                                                                 \
            hipFuncSetAttribute((const void*)gemm_nt_kernel<T, L, Bt, false, TM>,                         \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                    \
            attr_done = true;                                                                             \
        }                                                                                                 \
        hipLaunchKernelGGL((gemm_nt_kernel<T, L, Bt, false, TM>), dim3((unsigned)ntiles), dim3(256), lds, s, C, ldc, \
                           A, lda, B, ldb, K, alpha, beta, ntm, ntn, (int64_t)0);                         \
    } while (0)
    if (lower) {
        if (use_beta) GPRX_GEMM(true, true);
        else GPRX_GEMM(true, false);
    } else {
        if (use_beta) GPRX_GEMM(false, true);
        else GPRX_GEMM(false, false);
    }
#undef GPRX_GEMM
}

// Tile choice: 128x128 tiles when they give at least two workgroups per CU (bulk updates),
// 64x64 tiles otherwise (the latency-bound launches of the panel chain).
template <typename T>
void launch_gemm_nt(T* C, int64_t ldc, const T* A, int64_t lda, const T* B, int64_t ldb, int64_t M, int64_t N,
                    int64_t K, T alpha, T beta, bool lower, hipStream_t s) {
    if (M <= 0 || N <= 0) return;
    const bool use_beta = beta != T(0);
    const double elems = lower ? ((double)N * (N + 1) / 2 + (double)(M - N) * N) : (double)M * N;
    ProfScope ps(lower ? KC_UPDATE : (use_beta ? KC_OTHER : KC_TRSM), s, 2.0 * elems * K,
                 (double)sizeof(T) * (elems * (use_beta ? 2 : 1) + (double)(M + N) * K));
    static const int64_t small_tiles = [] {
        const char* e = std::getenv("GPRX_SMALL_TILE_WG");
        return e ? (int64_t)std::atoll(e) : (int64_t)1024;
    }();
    const int64_t ntm = M / GT, ntn = N / GT;
    const int64_t nt128 = lower ? ntn * (ntn + 1) / 2 + (ntm - ntn) * ntn : ntm * ntn;
    // in place (C = A B^T over A's own columns: the row solves' diagonal-block products, k_predict.hip
    // trsm_rows, k_lml.hip, the panel TRSM below): every workgroup must own WHOLE rows, so that no
    // other workgroup still reads the columns it overwrites -- with 64 x 64 tiles the workgroup of
    // columns 64..127 could read columns 0..63 after its neighbour stored them (an intermittent
    // error in a 64-row block of the result).  128 columns at most, the 128 (or 256) row tile.
    const bool inplace = (const void*)C == (const void*)A;
    GPRX_REQUIRE(!inplace || (ldc == lda && N <= GT && !lower), GPRX_ERR_ARG,
                 "gprx: launch_gemm_nt in place needs ldc == lda, N <= 128, a full product");
    if (!lower && nt128 >= 2 * small_tiles && launch_gemm_tall<T>(C, ldc, A, lda, B, ldb, M, N, K, alpha, beta, s))
        return;
    if (nt128 < small_tiles && !inplace)
        gemm_launch<T, 64>(C, ldc, A, lda, B, ldb, M, N, K, alpha, beta, lower, s);
    else
        gemm_launch<T, 128>(C, ldc, A, lda, B, ldb, M, N, K, alpha, beta, lower, s);
}

// Split-K form: P partial products, partial p = A[:, pK:(p+1)K] B[:, pK:(p+1)K]^T accumulated
// (beta = 1) into C + p*cstride, all in one launch (grid.y = P); K is the slice depth.
template <typename T>
void launch_gemm_nt_splitk(T* C, int64_t ldc, int64_t cstride, const T* A, int64_t lda, const T* B, int64_t ldb,
                           int64_t M, int64_t N, int64_t K, int P, T alpha, bool lower, hipStream_t s) {
    if (M <= 0 || N <= 0 || K <= 0) return;
    const int64_t ntm = M / GT, ntn = N / GT;
    const int64_t ntiles = lower ? ntn * (ntn + 1) / 2 + (ntm - ntn) * ntn : ntm * ntn;
    const size_t lds = gemm_lds_bytes<T, 128>();
    const double elems = lower ? ((double)N * (N + 1) / 2 + (double)(M - N) * N) : (double)M * N;
    ProfScope ps(KC_OTHER, s, 2.0 * elems * K * P, (double)sizeof(T) * (2 * elems * P + (double)(M + N) * K * P));
#define GPRX_GEMM_SK(L)                                                                                      \
    do {                                                                                                     \
        static bool attr_done = false;                                                                       \
        if (!attr_done) {                                                                                    \
            hipFuncSetAttribute((const void*)gemm_nt_kernel<T, L, true, false>,                              \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                       \
            attr_done = true;                                                                                \
        }                                                                                                    \
        hipLaunchKernelGGL((gemm_nt_kernel<T, L, true, false>), dim3((unsigned)ntiles, (unsigned)P), dim3(256), \
                           lds, s, C, ldc, A, lda, B, ldb, K, alpha, T(1), ntm, ntn, cstride);               \
    } while (0)
    if (lower) GPRX_GEMM_SK(true);
    else GPRX_GEMM_SK(false);
#undef GPRX_GEMM_SK
}

// C (lower) = A B^T where both operands vanish left of their row (LAUUM shape).
template <typename T>
void launch_gemm_nt_kskip(T* C, int64_t ldc, const T* A, int64_t lda, const T* B, int64_t ldb, int64_t M, int64_t N,
                          int64_t K, hipStream_t s) {
    if (M <= 0 || N <= 0) return;
    const int64_t ntm = M / GT, ntn = N / GT;
    const int64_t ntiles = ntn * (ntn + 1) / 2 + (ntm - ntn) * ntn;
    const size_t lds = gemm_lds_bytes<T, 128>();
    ProfScope ps(KC_INVERSE, s, 2.0 * (double)N * N * N / 6.0, 0.0);
    static bool attr_done = false;
    if (!attr_done) {
        hipFuncSetAttribute((const void*)gemm_nt_kernel<T, true, false, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (int)lds);
        attr_done = true;
    }
    hipLaunchKernelGGL((gemm_nt_kernel<T, true, false, true>), dim3((unsigned)ntiles), dim3(256), lds, s, C, ldc, A, lda,
                       B, ldb, K, T(1), T(0), ntm, ntn);
}

template <typename T>
static void launch_diag(T* Akk, int64_t ld, T* Lk, int* info, int64_t col0, hipStream_t s) {
    ProfScope ps(KC_DIAG, s, 2.0 * DB * DB * DB / 3.0, 0.0);
    hipLaunchKernelGGL((diag_potrf_kernel<T, false>), dim3(1), dim3(DT), 0, s, Akk, ld, Lk, info, col0);
}

template <typename T>
void launch_diag_public(T* Akk, int64_t ld, T* Lk, int* info, int64_t col0, hipStream_t s, int ph) {
    (void)ph;
    launch_diag<T>(Akk, ld, Lk, info, col0, s);
}
// in-kernel phase timing (s_memtime ticks, accumulated): load, solve phases, update
// phases, store, total
template <typename T>
void launch_diag_prof(T* Akk, int64_t ld, T* Lk, int* info, long long* prof, hipStream_t s) {
    hipLaunchKernelGGL((diag_potrf_kernel<T, true>), dim3(1), dim3(DT), 0, s, Akk, ld, Lk, info, (int64_t)0, prof);
}
template void launch_diag_prof<double>(double*, int64_t, double*, int*, long long*, hipStream_t);
template void launch_diag_prof<float>(float*, int64_t, float*, int*, long long*, hipStream_t);
template void launch_diag_public<double>(double*, int64_t, double*, int*, int64_t, hipStream_t, int);
template void launch_diag_public<float>(float*, int64_t, float*, int*, int64_t, hipStream_t, int);

int outer_block() {
    static int nbo = [] {
        int v = 512;
        if (const char* e = std::getenv("GPRX_NBO")) v = std::atoi(e);
        if (v < DB) v = DB;
        return (v / DB) * DB;
    }();
    return nbo;
}

hipEvent_t Exec::event(size_t i) {
    while (ev.size() <= i) {
        hipEvent_t e;
        GPRX_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        ev.push_back(e);
    }
    return ev[i];
}

Exec::~Exec() {
    for (auto e : ev) (void)hipEventDestroy(e);
    pt_state_free(pt);
    if (scratch) (void)hipFree(scratch);
}

int* Exec::scratch_ints(size_t n) {
    if (n > scratch_n) {
        if (scratch) GPRX_HIP(hipFree(scratch));
        scratch = nullptr;
        GPRX_HIP(hipMalloc(&scratch, sizeof(int) * n));
        scratch_n = n;
    }
    return scratch;
}

bool potrf_uses_tiles() {
    static const bool streams = [] {
        const char* e = std::getenv("GPRX_POTRF");
        return e && std::string(e) == "streams";
    }();
    return !streams;
}

template <typename T>
void potrf_auto(T* A, int64_t ld, int64_t np, int64_t nrows, T* Linv, int* info, Exec& ex) {
    if (potrf_uses_tiles()) potrf_tiles<T>(A, ld, np, nrows, Linv, info, ex);
    else potrf_blocked<T>(A, ld, np, nrows, Linv, info, ex);
}

// Two-level right-looking Cholesky with look-ahead.
//   Panel(K)      columns [c0, c0+w) of every row below: per 128-block diag + trsm + the
//                 update of the remaining panel columns (stream P = ex.s0)
//   TrailNext(K)  next panel's columns -= P_K P_K^T   (stream P)
//   TrailRest(K)  the rest of the trailing matrix     (stream B = ex.s1, K = w deep)
// Panel(K+1) runs on P while TrailRest(K) runs on B.
// Factor the (already fully updated) column panel [c0, c0+w) over rows c0..nrows: per
// 128-block the diagonal kernel, the trsm of every row below (GEMM with Linv) and the update
// of the panel's remaining columns.  `skip` is the timing-experiment mask (see below).
// inner_wait (may be null): event the first in-panel update waits for (the look-ahead
// update of the panel's later columns running on another stream).
template <typename T>
static void potrf_panel(T* A, int64_t ld, int64_t nrows, int64_t c0, int64_t w, T* Linv, int* info, hipStream_t P,
                        int skip, hipEvent_t inner_wait = nullptr) {
    for (int64_t kk = c0; kk < c0 + w; kk += DB) {
        T* Lk = Linv + (kk / DB) * (int64_t)DB * DB;
        if (!(skip & 2)) launch_diag<T>(A + kk + kk * ld, ld, Lk, info, kk, P);
        const int64_t rows_below = nrows - (kk + DB);
        if (rows_below <= 0 || (skip & 4)) continue;
        T* Pk = A + (kk + DB) + kk * ld;
        launch_gemm_nt<T>(Pk, ld, Pk, ld, Lk, DB, rows_below, DB, DB, T(1), T(0), false, P);
        const int64_t inner = c0 + w - (kk + DB);
        if (kk == c0 && inner_wait) GPRX_HIP(hipStreamWaitEvent(P, inner_wait, 0));
        if (inner > 0)
            launch_gemm_nt<T>(A + (kk + DB) + (kk + DB) * ld, ld, Pk, ld, Pk, ld, rows_below, inner, DB, T(-1), T(1),
                              true, P);
    }
}

// Two-level right-looking Cholesky with look-ahead.
//   Panel(K)      columns [c0, c0+w) of every row below: per 128-block diag + trsm + the
//                 update of the remaining panel columns (stream P = ex.s0)
//   TrailNext(K)  next panel's columns -= P_K P_K^T: its first 128 columns on P (so the next
//                 diagonal kernel can start), the other columns on stream Q = ex.s2; the
//                 next panel's first in-panel update waits for Q
//   TrailRest(K)  the rest of the trailing matrix     (stream B = ex.s1, K = w deep)
// Panel(K+1) runs on P while TrailRest(K) runs on B.  TrailNext(K) waits for TrailRest(K-1)
// (both accumulate into the next panel's columns).
template <typename T>
void potrf_blocked(T* A, int64_t ld, int64_t np, int64_t nrows, T* Linv, int* info, Exec& ex) {
    const int64_t NBO = outer_block();
    hipStream_t P = ex.s0, B = ex.s1 ? ex.s1 : ex.s0, Q = ex.s2 ? ex.s2 : ex.s0;
    // timing experiments only (results are wrong): 1 = no TrailRest, 2 = no diagonal kernel,
    // 4 = no panel trsm / inner update
    static const int skip = [] {
        const char* e = std::getenv("GPRX_DEBUG_SKIP");
        return e ? std::atoi(e) : 0;
    }();
    const int64_t nK = (np + NBO - 1) / NBO;
    // events: 4K panel(K) done, 4K+1 TrailRest(K) done, 4K+2 TrailNext-b(K) done,
    // 4K+3 TrailNext may start (TrailRest(K-1) done)
    hipEvent_t tnb_prev = nullptr;
    for (int64_t K = 0; K < nK; K++) {
        const int64_t c0 = K * NBO, w = std::min(NBO, np - c0);
        potrf_panel<T>(A, ld, nrows, c0, w, Linv, info, P, skip, tnb_prev);
        tnb_prev = nullptr;
        if (K == nK - 1) break;
        const int64_t c1 = c0 + w, wn = std::min(NBO, np - c1);
        const T* Pan = A + c0 * ld;  // column c0; row offsets added below
        if (B != P) {
            GPRX_HIP(hipEventRecord(ex.event(4 * K), P));
            if (K >= 1) GPRX_HIP(hipStreamWaitEvent(P, ex.event(4 * (K - 1) + 1), 0));
        }
        // TrailNext(K): first 128 columns on P, the rest on Q
        const int64_t wa = (Q != P) ? std::min<int64_t>(DB, wn) : wn;
        launch_gemm_nt<T>(A + c1 + c1 * ld, ld, Pan + c1, ld, Pan + c1, ld, nrows - c1, wa, w, T(-1), T(1), true, P);
        if (wn > wa) {
            const int64_t cb = c1 + wa;
            GPRX_HIP(hipEventRecord(ex.event(4 * K + 3), P));
            GPRX_HIP(hipStreamWaitEvent(Q, ex.event(4 * K + 3), 0));
            launch_gemm_nt<T>(A + cb + cb * ld, ld, Pan + cb, ld, Pan + cb, ld, nrows - cb, wn - wa, w, T(-1), T(1),
                              true, Q);
            GPRX_HIP(hipEventRecord(ex.event(4 * K + 2), Q));
            tnb_prev = ex.event(4 * K + 2);
        }
        // TrailRest(K)
        const int64_t c2 = c1 + wn;
        if (B != P) GPRX_HIP(hipStreamWaitEvent(B, ex.event(4 * K), 0));
        if (c2 < np && !(skip & 1))
            launch_gemm_nt<T>(A + c2 + c2 * ld, ld, Pan + c2, ld, Pan + c2, ld, nrows - c2, np - c2, w, T(-1), T(1),
                              true, B);
        if (B != P) GPRX_HIP(hipEventRecord(ex.event(4 * K + 1), B));
    }
    if (B != P && nK >= 2) GPRX_HIP(hipStreamWaitEvent(P, ex.event(4 * (nK - 2) + 1), 0));
    if (Q != P) {  // everything issued on Q is done before the caller's next work on P
        GPRX_HIP(hipEventRecord(ex.event(4 * nK), Q));
        GPRX_HIP(hipStreamWaitEvent(P, ex.event(4 * nK), 0));
    }
}

// ======================================================================================
// Back substitution  L^T alpha = z   (z: m rows of length np, alpha: np x m row-major)
// ======================================================================================
template <typename T>
__global__ void copy_aug_kernel(const T* __restrict__ A, int64_t ld, int64_t np, int m, T* __restrict__ z) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (int64_t)m * np) return;
    int64_t r = e / np, c = e % np;
    z[e] = A[np + r + c * ld];
}


// alpha_j = Linv_j^T z_j  (one workgroup): the 128x128 block is staged into LDS with
// coalesced loads (row q of the image = column q of Linv), then thread q forms
// sum_{p >= q} Linv[p][q] z[p] from LDS.
template <typename T>
__global__ __launch_bounds__(256) void backsolve_alpha_kernel(int64_t np, int m, const T* __restrict__ Linv,
                                                              const T* __restrict__ z, T* __restrict__ alpha,
                                                              int64_t j0) {
    __shared__ T sLi[DB][DB + 1];
    __shared__ T sz[DB];
    const int t = threadIdx.x;
#pragma unroll 8
    for (int u = 0; u < DB * DB / 256; u++) {
        const int e = t + 256 * u;
        sLi[e / DB][e % DB] = Linv[e];
    }
    for (int r = 0; r < m; r++) {
        if (t < DB) sz[t] = z[(int64_t)r * np + j0 + t];
        __syncthreads();
        if (t < DB) {
            T acc = 0;
            for (int p = t; p < DB; p++) acc = fma(sLi[t][p], sz[p], acc);
            alpha[(j0 + t) * m + r] = acc;
        }
        __syncthreads();
    }
}

// z[c] -= sum_p L[j0+p][c] alpha_j[p] for c < j0.  16 lanes per column (each lane 8
// consecutive rows = 64 contiguous bytes), 4 columns per wave, 16 columns per workgroup.
constexpr int BS_COLS_WG = 16;
template <typename T>
__global__ __launch_bounds__(256) void backsolve_update_kernel(const T* __restrict__ A, int64_t ld, int64_t np, int m,
                                                               const T* __restrict__ alpha, T* __restrict__ z,
                                                               int64_t j0) {
    const int t = threadIdx.x;
    const int lane = t & 63, w = t >> 6;
    const int sub = lane >> 4, l16 = lane & 15;
    const int64_t c = (int64_t)blockIdx.x * BS_COLS_WG + w * 4 + sub;
    const bool ok = c < j0;
    T Lv[8];
    if (ok) {
        const T* Lc = A + j0 + c * ld + l16 * 8;
#pragma unroll
        for (int e = 0; e < 8; e++) Lv[e] = Lc[e];
    }
    for (int r = 0; r < m; r++) {
        T v = 0;
        if (ok) {
#pragma unroll
            for (int e = 0; e < 8; e++) v = fma(Lv[e], alpha[(j0 + l16 * 8 + e) * m + r], v);
        }
        v += __shfl_xor(v, 8);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 1);
        if (ok && l16 == 0) z[(int64_t)r * np + c] -= v;
    }
}

template <typename T>
void launch_backsolve(const T* A, int64_t ld, int64_t np, int m, const T* Linv, T* z, T* alpha, hipStream_t s) {
    const int64_t e = (int64_t)m * np;
    ProfScope ps(KC_BACKSOLVE, s, 2.0 * (double)np * np * m / 2.0, (double)sizeof(T) * np * (np + 1) / 2.0);
    hipLaunchKernelGGL(copy_aug_kernel<T>, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, A, ld, np, m, z);
    for (int64_t j0 = np - DB; j0 >= 0; j0 -= DB) {
        hipLaunchKernelGGL(backsolve_alpha_kernel<T>, dim3(1), dim3(256), 0, s, np, m,
                           Linv + (j0 / DB) * (int64_t)DB * DB, (const T*)z, alpha, j0);
        if (j0 > 0)
            hipLaunchKernelGGL(backsolve_update_kernel<T>, dim3((unsigned)((j0 + BS_COLS_WG - 1) / BS_COLS_WG)),
                               dim3(256), 0, s, A, ld, np, m, (const T*)alpha, z, j0);
    }
}

// ======================================================================================
// logdet = 2 sum log L_ii, datafit = || z ||^2  (double accumulation)
// ======================================================================================
// log det = 2 sum log L_ii and the data fit z^T z (z = L^{-1} Y in the label rows), in two
// steps with a fixed summation order: per 128-row block partials, then their sum.  (One
// 1024-thread block striding over the strided diagonal took 61 us at N = 16384.)
template <typename T>
__global__ __launch_bounds__(256) void fit_reduce_part_kernel(const T* __restrict__ A, int64_t ld, int64_t n,
                                                              int64_t np, int m, double* __restrict__ part) {
    __shared__ double s0[256], s1[256];
    const int t = threadIdx.x;
    const int64_t r0 = (int64_t)blockIdx.x * 128;
    double a = 0, b = 0;
    if (t < 128 && r0 + t < n) a = log((double)A[r0 + t + (r0 + t) * ld]);
    for (int e = t; e < 128 * m; e += 256) {
        const int64_t c = r0 + e / m;
        const int r = e % m;
        if (c < np) {
            const double v = (double)A[np + r + c * ld];
            b += v * v;
        }
    }
    s0[t] = a;
    s1[t] = b;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (t < off) {
            s0[t] += s0[t + off];
            s1[t] += s1[t + off];
        }
        __syncthreads();
    }
    if (t == 0) {
        part[2 * blockIdx.x] = s0[0];
        part[2 * blockIdx.x + 1] = s1[0];
    }
}

__global__ __launch_bounds__(256) void fit_reduce_sum_kernel(const double* __restrict__ part, int nb,
                                                             double* __restrict__ out) {
    __shared__ double s0[256], s1[256];
    const int t = threadIdx.x;
    double a = 0, b = 0;
    for (int k = t; k < nb; k += 256) {
        a += part[2 * k];
        b += part[2 * k + 1];
    }
    s0[t] = a;
    s1[t] = b;
    __syncthreads();
    for (int off = 128; off > 0; off >>= 1) {
        if (t < off) {
            s0[t] += s0[t + off];
            s1[t] += s1[t + off];
        }
        __syncthreads();
    }
    if (t == 0) {
        out[0] = 2.0 * s0[0];
        out[1] = s1[0];
    }
}

// out[0] = log det, out[1] = z^T z; out holds 2 + 2 * (np / 128) doubles (the partials after)
template <typename T>
void launch_fit_reductions(const T* A, int64_t ld, int64_t n, int64_t np, int m, double* out, hipStream_t s) {
    const int nb = (int)((np + 127) / 128);
    hipLaunchKernelGGL(fit_reduce_part_kernel<T>, dim3((unsigned)nb), dim3(256), 0, s, A, ld, n, np, m, out + 2);
    hipLaunchKernelGGL(fit_reduce_sum_kernel, dim3(1), dim3(256), 0, s, (const double*)(out + 2), nb, out);
}

#define GPRX_INST(T)                                                                                      \
    template void potrf_blocked<T>(T*, int64_t, int64_t, int64_t, T*, int*, Exec&);                      \
    template void potrf_auto<T>(T*, int64_t, int64_t, int64_t, T*, int*, Exec&);                         \
    template void launch_gemm_nt_splitk<T>(T*, int64_t, int64_t, const T*, int64_t, const T*, int64_t,   \
                                           int64_t, int64_t, int64_t, int, T, bool, hipStream_t);         \
    template void launch_gemm_nt<T>(T*, int64_t, const T*, int64_t, const T*, int64_t, int64_t, int64_t, \
                                    int64_t, T, T, bool, hipStream_t);                                    \
    template void launch_backsolve<T>(const T*, int64_t, int64_t, int, const T*, T*, T*, hipStream_t);   \
    template void launch_fit_reductions<T>(const T*, int64_t, int64_t, int64_t, int, double*, hipStream_t); \
    template void launch_gemm_nt_kskip<T>(T*, int64_t, const T*, int64_t, const T*, int64_t, int64_t, int64_t,   \
                                          int64_t, hipStream_t);
GPRX_INST(double)
GPRX_INST(float)
#undef GPRX_INST

}  // namespace gprx
