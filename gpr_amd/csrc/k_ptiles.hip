// k_ptiles.hip — tile-dataflow Cholesky in ONE persistent launch (gfx950).
//
// Replaces the same reference step as potrf_blocked (lapack::lu_invert -> dgetrf_+dgetri_,
// include/LAPACKUtils.h:38-56, 85-97, called from GaussianProcess::InvertKernelMatrix,
// lib/GaussianProcess.cpp:545-559) with K + sigma^2 I = L L^T, the forward solve z = L^{-1} Y
// riding along as extra row blocks, exactly as k_potrf.hip does -- but scheduled on the device.
//
// Why: in the stream formulation every step of the panel chain (diagonal factor -> trsm ->
// next-column update) is a kernel that must wait for CU slots held by the bulk trailing
// GEMM, so at N = 16384 the chain (18 ms alone) stretches to most of the 37 ms
// factorisation.  Here one workgroup per CU runs a loop over a ticket list of 128x128 TILE
// TASKS with per-tile dependency counters in HBM:
//
//   DIAGX(k)        T = A_{k,k-1} Linv_{k-1}^T (the trsm of the critical tile),
//                   A_kk -= T T^T, then factor A_kk = L_kk L_kk^T and form Linv_k
//                   (one task = the whole critical step, no hand-off inside it)
//   TRSM(i,k)       L_ik = A_ik Linv_k^T                  (i >= k+2, and the label rows)
//   UPD(i,j,b0,nb)  A_ij -= sum_{b0<=b<b0+nb} L_ib L_jb^T  (nb = W for far-behind panels)
//
// Counters: ver[i][j] = number of b already applied to tile (i,j); lcnt[i] = number of
// final blocks L_i0..L_i,lcnt-1 of row block i.  Wait conditions:
//   DIAGX(k):  ver[k][k-1] == k-1, ver[k][k] == k-1, lcnt[k-1] >= k
//   TRSM(i,k): ver[i][k] == k, lcnt[k] >= k+1
//   UPD:       ver[i][j] == b0, lcnt[i] >= b0+nb, lcnt[j] >= b0+nb
// The ticket order is a list schedule computed on the host (critical-path priorities,
// simulated on P workers): every task's producers hold earlier tickets, and a workgroup that
// holds a ticket is running, so the smallest unfinished ticket can always proceed -- no
// deadlock whatever the real durations.  Every wait is also bounded in wall-clock time: a
// timeout raises an error flag that drains every workgroup and is reported as info = -1.
//
// Hand-offs follow the gfx950 inter-workgroup recipe (MI355X_MICROARCH.md, "Workgroup
// dispatch ... visibility"): producer stores -> s_waitcnt vmcnt(0) in every wave ->
// barrier -> one lane: agent release fence, s_waitcnt vmcnt(0), relaxed agent-scope counter
// store; consumer: one lane polls with relaxed agent loads, agent acquire fence,
// s_waitcnt vmcnt(0), barrier, then plain loads.
//
// Tile GEMM: 512 threads = 8 waves of 64x32 (v_mfma_f64_16x16x4f64 / _f32_16x16x4f32),
// operands staged 32-deep through LDS, double-buffered; 147 KB of LDS per workgroup also
// keeps the launch at one workgroup per CU, so the critical DIAGX step has a whole CU.
#include "gprx_dist.h"
#include "gprx_internal.h"
#include "k_pairs.h"

#include <algorithm>
#include <climits>
#include <cstring>
#include <cstdlib>
#include <functional>
#include <map>
#include <mutex>
#include <queue>
#include <tuple>

namespace gprx {

namespace pt {

using namespace mm;
static_assert(C_NCTL == C_NCTL_DIST, "counter block layout shared with gprx_dist.cpp");

// ------------------------------------------------------------------------------------------
// One 128x128 tile:  C = A B^T (UPDATE = false)  or  C -= A B^T (UPDATE = true), K deep.
// A: 128 rows x K (column-major, lda), B: 128 rows x K (ldb).  lower: diagonal tile, only
// row >= col is stored and the waves wholly above the diagonal skip their MFMAs.  tri: B is
// lower triangular (K = 128, a diagonal-block inverse): output columns 32 wc .. 32 wc + 31
// need only k < 32 wc + 32, the waves skip the MFMAs of the zero part.
// ------------------------------------------------------------------------------------------
// Bpan: B by 128-column panels (tile_mma): the distributed factorisation's window tiles.
// MAP: the wave -> output-block map (k_mma.h wave_block): 1 for triangular B, 2 for lower.
template <typename T, bool UPDATE, int MAP = 0, int FEED = -1>
__device__ __forceinline__ void tile_gemm(T* __restrict__ C, int64_t ldc, const T* __restrict__ A, int64_t lda,
                                          const T* __restrict__ B, int64_t ldb, int K, bool lower, T* smem,
                                          const int t, bool tri = false, const uint64_t* Bpan = nullptr) {
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    const int lane = t & 63, w = t >> 6;
    int wr, wc;
    wave_block<MAP>(w, wr, wc);
    const int lr = lane & 15, lk = lane >> 4;
    const bool active = !(lower && wr == 0 && wc >= 2);
    // UPDATE: the whole C tile is fetched into registers up front (its latency hides under the
    // mainloop; loading it unconditionally, all before any store, avoids hipcc's per-element
    // branches and vmcnt(0) waits)
    T cv[2][4][4];
    if (UPDATE && active) {
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int reg = 0; reg < 4; reg++) {
                const int jl = wc * 32 + x * 16 + Tr::orow(lk, reg);
                const T* ccol = C + (int64_t)jl * ldc;
#pragma unroll
                for (int y = 0; y < 4; y++) cv[x][y][reg] = ccol[wr * 64 + y * 16 + lr];
            }
    }
    acc_t acc[2][4];
    tile_mma<T, MAP, false, BkOf<T>::v, FEED>(acc, A, lda, B, ldb, K, !active ? 0 : (tri ? 32 * (wc + 1) : K), smem, t,
                                           Bpan);
    if (!active) return;
#pragma unroll
    for (int x = 0; x < 2; x++) {
#pragma unroll
        for (int reg = 0; reg < 4; reg++) {
            const int jl = wc * 32 + x * 16 + Tr::orow(lk, reg);
            T* ccol = C + (int64_t)jl * ldc;
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const int il = wr * 64 + y * 16 + lr;
                // stores are unconditional (a branch per element makes hipcc wait for every
                // previous store); above the diagonal of a diagonal tile the old value goes back.
                // sc1 (write-through) stores: the hand-off needs no L2 write-back fence
                if (UPDATE)
                    st_sc1(ccol + il, (lower && il < jl) ? cv[x][y][reg] : cv[x][y][reg] - acc[x][y][reg]);
                else if (!lower || il >= jl)
                    st_sc1(ccol + il, acc[x][y][reg]);
            }
        }
    }
}

// TRSM task: C = A B^T for the lower-triangular B = Linv_k, each wave 16 rows x 128 columns
// (k_mma.h tile_mma_trirows: every stage's triangle split evenly over the waves); C may be A.
// C3 fit trace: TRSM 15.7 -> 13.0 us per task; launch 24.75 -> 24.62 ms same box, C2 within
// noise, C4 unchanged (profiles/r06t_trsm_rows_ab.txt; out of line: 24.78 ms, not kept).
// GPRX_TRSM_ROWS=0 builds the MAP 1 form.
#ifndef GPRX_TRSM_ROWS
#define GPRX_TRSM_ROWS 1
#endif
template <typename T>
__device__ __forceinline__ void tile_trsm(T* C, int64_t ldc, const T* A, int64_t lda,
                                          const T* __restrict__ B, int64_t ldb, T* smem, const int t) {
    if constexpr (!GPRX_TRSM_ROWS) {
        tile_gemm<T, false, 1, GPRX_SHORT_FEED>(C, ldc, A, lda, B, ldb, GT, false, smem, t, true);
    } else {
        typedef Mfma<T> Tr;
        const int lane = t & 63, w = t >> 6, lr = lane & 15, lk = lane >> 4;
        typename Tr::acc_t acc[2][4];
        mm::tile_mma_trirows<T>(acc, A, lda, B, ldb, smem, t);
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 4; y++)
#pragma unroll
                for (int reg = 0; reg < 4; reg++)
                    st_sc1(C + (int64_t)(16 * (4 * x + y) + Tr::orow(lk, reg)) * ldc + 16 * w + lr, acc[x][y][reg]);
    }
}

// ------------------------------------------------------------------------------------------
// Paired update (T_UPD2): C -= A B^T on a 256 x 128 tile -- tiles (i, j) and (i + 1, j), which
// are adjacent rows of the column-major factor (C and A are 256 rows at one ld) -- over K panels
// of the same B (L_j).  The 8 waves take 64 x 64 blocks (tile_mma_tall: 16 MFMAs per 8 fragment
// reads, 384 DMA'd rows per stage for twice the 128 x 128 tile's flops; probe 0.901 of the f64
// MFMA bound against 0.877, f32 0.857 against 0.818, profiles/r05u).  Its 128 accumulator
// registers fit the task loop because the C tile is not prefetched into registers beside them,
// as tile_gemm does: C comes in four column chunks during the first stages and is subtracted
// from the accumulators (tile_mma_tall Csub), and -acc = C - A B^T is stored.  (Starting the
// accumulators from -C held the first MFMA for the whole 256 KB read: C3's launch lost 0.4 ms.)
// Off-diagonal tiles only.
// ------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void tile_gemm_tall(T* __restrict__ C, int64_t ldc, const T* __restrict__ A, int64_t lda,
                                               const T* __restrict__ B, int64_t ldb, int K, T* smem, const int t) {
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    const int lane = t & 63, w = t >> 6;
    const int wr = w & 3, wc = w >> 2, lr = lane & 15, lk = lane >> 4;
    acc_t acc[4][4];
    mm::tile_mma_tall<T, 1>(acc, A, lda, B, ldb, K, smem, t, C, ldc);
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int reg = 0; reg < 4; reg++) {
            T* ccol = C + (int64_t)(64 * wc + 16 * x + Tr::orow(lk, reg)) * ldc;
#pragma unroll
            for (int y = 0; y < 4; y++) st_sc1(ccol + 64 * wr + 16 * y + lr, -acc[x][y][reg]);
        }
}

// ------------------------------------------------------------------------------------------
// Diagonal 128x128 block: L (in place, lower) and Linv (DB x DB, column-major), 512 threads.
//
// The block lives in REGISTERS as a square image S: lower triangle = A (becoming L), strict
// upper triangle = rows of B = L^{-T} (diagonal in Bd).  B comes from the identity appended
// below A riding along the elimination; being upper triangular it fills the unused half.
// Thread t owns rows R0..R0+3 (R0 = 4*(lane&31)) of the 8-column block cb = 2w + (lane>>5).
// Right-looking over 8-column steps:
//   1  waves 0-1 (one row each) factor the 8x8 pivot redundantly (rsq + Newton, no divide)
//      and solve their row x = v Ld^{-T}, v read from the column block published in sV;
//   2  threads with trailing columns apply S -= x_r x_c^T (unmasked: right of the diagonal
//      in rows not yet reached is scratch, zeroed when those rows become pivot rows); the
//      owners of the next column block publish it.
// The image is then staged through LDS so L and Linv leave in coalesced column stores.
// ------------------------------------------------------------------------------------------
constexpr int SPL = DB + 4;
constexpr int SIL = DB + 2;

__device__ __forceinline__ void st_agent(int* p, int v);  // (hand-off helpers, below)

// v_rsq_f64 (relative error ~2^-23) refined by ONE Halley step, y (1 + e/2 + 3e^2/8) with
// e = 1 - x y^2 (cubic convergence: error ~2^-69 before rounding): 4 dependent f64 operations
// after the rsq against the 6 of two Newton steps -- the pivot chain is latency-bound
__device__ __forceinline__ double rsqrt_full(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    const double e = fma(-x * y, y, 1.0);
    return fma(y * e, fma(e, 0.375, 0.5), y);
}
__device__ __forceinline__ float rsqrt_full(float x) {
    float y = __builtin_amdgcn_rsqf(x);
    const float h = 0.5f * x;
    y = y * fmaf(-h * y, y, 1.5f);
    return y;
}

template <typename T>
constexpr size_t diag_lds() {
    // (DB + 2 diagonal words: diag_factor_la keeps a zero after sDi)
    return sizeof(T) * ((size_t)DB * SIL + DB + 2) > sizeof(T) * (2 * 8 * SPL + 144)
               ? sizeof(T) * ((size_t)DB * SIL + DB + 2)
               : sizeof(T) * (2 * 8 * SPL + 144);
}

__device__ __forceinline__ void dbg_mark(int* dbg, int q, int phase, int i, int j) {
    if (dbg && __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) == 0) {
        int* p = dbg + 4 * blockIdx.x;
        __hip_atomic_store(p + 0, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(p + 2, i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(p + 3, j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(p + 1, phase, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <typename T>
__device__ __forceinline__ void diag_factor_rank8(T* __restrict__ A, int64_t ld, T* __restrict__ Linv,
                                                  int* __restrict__ info, int64_t col0, unsigned char* smem_raw,
                                                  const int t, int* dbg = nullptr, long long* prof = nullptr) {
    long long pt0 = prof ? wall_clock64() : 0, pacc1 = 0, pacc2 = 0, pm = 0;
    T(*sV)[SPL] = reinterpret_cast<T(*)[SPL]>(smem_raw);
    T(*sP)[SPL] = reinterpret_cast<T(*)[SPL]>(smem_raw + sizeof(T) * 8 * SPL);
    T(*sLdW)[8][9] = reinterpret_cast<T(*)[8][9]>(smem_raw + sizeof(T) * 16 * SPL);  // per wave 0/1
    T(*sLd)[9] = sLdW[0];

    const int w = t >> 6, l = t & 63;
    const int R0 = (l & 31) * 4;
    const int cbi = 2 * w + (l >> 5);
    const int C0 = cbi * 8;

    T S[4][8];
    T Bd[4];
#pragma unroll
    for (int b = 0; b < 8; b++)
#pragma unroll
        for (int a = 0; a < 4; a++) S[a][b] = A[R0 + a + (int64_t)(C0 + b) * ld];
#pragma unroll
    for (int a = 0; a < 4; a++) Bd[a] = T(1);
    if (cbi == 0) {
#pragma unroll
        for (int a = 0; a < 4; a++)
#pragma unroll
            for (int b = 0; b < 8; b++) sV[b][R0 + a] = S[a][b];
    }
    __syncthreads();
    if (prof) pm = wall_clock64();
    const long long pload = pm;

    int fail_col = -1;
    for (int j0 = 0; j0 < DB; j0 += 8) {
        const int jn = j0 + 8;
        if (t < DB) {
            // every lane of waves 0-1 factors the pivot (identical values) in registers and
            // solves its row with it; wave 0 also leaves the factor in LDS for the pivot rows
            T(*myLd)[9] = sLdW[w];
            const int row = t;
            const bool piv = row >= j0 && row < jn;
            T x[8];
            {
                // the whole pivot block and this row's segment are read up front (one LDS
                // latency: the compiler cannot move these reads above the myLd stores), the
                // factor runs in place in registers, and the stores follow in one branch
                T Ld[8][8], ri[8], vr[8];
#pragma unroll
                for (int c = 0; c < 8; c++)
#pragma unroll
                    for (int r = c; r < 8; r++) Ld[r][c] = sV[c][j0 + r];
#pragma unroll
                for (int q = 0; q < 8; q++) vr[q] = sV[q][row];
#pragma unroll
                for (int c = 0; c < 8; c++) {
                    T dsum = Ld[c][c];
#pragma unroll
                    for (int k = 0; k < c; k++) dsum = fma(-Ld[c][k], Ld[c][k], dsum);
                    if (!(dsum > T(0)) && fail_col < 0) fail_col = j0 + c;
                    ri[c] = rsqrt_full(dsum);
                    Ld[c][c] = dsum * ri[c];
#pragma unroll
                    for (int r = c + 1; r < 8; r++) {
                        T v = Ld[r][c];
#pragma unroll
                        for (int k = 0; k < c; k++) v = fma(-Ld[r][k], Ld[c][k], v);
                        Ld[r][c] = v * ri[c];
                    }
                }
                // one lane per wave writes (64 lanes storing one word serialise in the LDS)
                if (l == 0) {
#pragma unroll
                    for (int c = 0; c < 8; c++) {
                        myLd[c][8] = ri[c];
#pragma unroll
                        for (int r = c; r < 8; r++) myLd[r][c] = Ld[r][c];
                    }
                }
#pragma unroll
                for (int q = 0; q < 8; q++) {
                    T v = piv ? ((row - j0 == q) ? T(1) : T(0)) : vr[q];
#pragma unroll
                    for (int q2 = 0; q2 < q; q2++) v = fma(-x[q2], Ld[q][q2], v);
                    x[q] = v * ri[q];
                }
            }
#pragma unroll
            for (int q = 0; q < 8; q++) sP[q][row] = x[q];
        }
        __syncthreads();
        if (prof) {
            const long long tn = wall_clock64();
            pacc1 += tn - pm;
            pm = tn;
        }
        const bool pivrows = R0 >= j0 && R0 < jn;
        if (cbi == (j0 >> 3)) {
            if (pivrows) {
#pragma unroll
                for (int a = 0; a < 4; a++) {
                    const int p = R0 + a - j0;
#pragma unroll
                    for (int q = 0; q < 8; q++) {
                        const T xq = sP[q][R0 + a];
                        S[a][q] = (q <= p) ? sLd[p][q] : xq;
                        if (q == p) Bd[a] = xq;
                    }
                }
            } else {
#pragma unroll
                for (int a = 0; a < 4; a++)
#pragma unroll
                    for (int q = 0; q < 8; q++) S[a][q] = sP[q][R0 + a];
            }
        }
        if (C0 >= jn && (R0 < jn || R0 + 3 >= C0)) {
            if (pivrows) {
#pragma unroll
                for (int a = 0; a < 4; a++)
#pragma unroll
                    for (int b = 0; b < 8; b++) S[a][b] = T(0);
            }
#pragma unroll
            for (int q = 0; q < 8; q++) {
                T u[4], v[8];
#pragma unroll
                for (int a = 0; a < 4; a++) u[a] = sP[q][R0 + a];
#pragma unroll
                for (int b = 0; b < 8; b++) v[b] = sP[q][C0 + b];
#pragma unroll
                for (int a = 0; a < 4; a++)
#pragma unroll
                    for (int b = 0; b < 8; b++) S[a][b] = fma(-u[a], v[b], S[a][b]);
            }
        }
        if (jn < DB && cbi == (jn >> 3)) {
#pragma unroll
            for (int a = 0; a < 4; a++)
#pragma unroll
                for (int b = 0; b < 8; b++) sV[b][R0 + a] = S[a][b];
        }
        __syncthreads();
        if (prof) {
            const long long tn = wall_clock64();
            pacc2 += tn - pm;
            pm = tn;
        }
    }
    if (prof && t == 0) {
        prof[0] = pload - pt0;
        prof[1] = pacc1;
        prof[2] = pacc2;
    }
    if (fail_col >= 0) atomicMin(info, (int)(col0 + fail_col + 1));  // same value in every lane of waves 0-1

    T(*sI)[SIL] = reinterpret_cast<T(*)[SIL]>(smem_raw);
    T* sBd = reinterpret_cast<T*>(smem_raw + sizeof(T) * DB * SIL);
#pragma unroll
    for (int a = 0; a < 4; a++) {
#pragma unroll
        for (int b = 0; b < 8; b++) sI[R0 + a][C0 + b] = S[a][b];
        if (R0 + a >= C0 && R0 + a < C0 + 8) sBd[R0 + a] = Bd[a];
    }
    __syncthreads();
    {
        const int r = t & (DB - 1);
        for (int c = t >> 7; c < DB; c += NT / DB) {
            if (r >= c) A[r + (int64_t)c * ld] = sI[r][c];
            Linv[r + c * DB] = (r > c) ? sI[c][r] : ((r == c) ? sBd[r] : T(0));
        }
    }
}

// ------------------------------------------------------------------------------------------
// Diagonal 128x128 block, blocked: four 32-column panels, the panel's 32 x 32 diagonal block
// factored by ONE wave in registers and everything else on the MFMA units.
//
// The block lives in LDS (column-major, stride SIL): lower triangle = A becoming L; the
// strict upper triangle collects Linv^T (Linv = L^{-1}), its diagonal goes to sDi.  Per panel
// p (c0 = 32 p):
//   1  wave 0: D = L_pp L_pp^T in registers -- lane l < 32 holds row l of D, lane 32 + i row
//      i of the identity riding along (it ends as row i of L_pp^{-T}); column step c: the
//      pivot and the scaled column are broadcast by readlane (scalar operands), no barrier.
//      L_pp -> lower, Dinv_p = L_pp^{-1} -> upper (transposed) + sDi
//   2  all waves: panel rows below, L_rp = A_rp Dinv_p^T (16x16 MFMA tiles, K = 32)
//   3  all waves: trailing lower tiles A_rr' -= L_rp L_r'p^T
// then the off-diagonal 32-blocks of Linv by distance d = 1..3:
//   Linv_ij = -Dinv_i sum_{k=j}^{i-1} L_ik Linv_kj  (i = j + d; S staged in Linv_ij's slot)
// and L, Linv leave in coalesced column stores.  Replaces the rank-8 in-register image
// (diag_factor_rank8: 16 serial pivot steps of 2 barriers each, 52 us per DIAGX task).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double rl_lane(double v, int lane) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ float rl_lane(float v, int lane) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
}

// GPRX_FACT32_PROF (a profiling build only): core-clock split of fact32's steps into the pivot
// block (readlanes, 4 x 4 factor, its inverse), the panel solve and the trailing MFMAs; each
// mark first makes the wave wait for the phase's last result (readfirstlane)
#ifdef GPRX_FACT32_PROF
#define F32_MARK(acc_, x_)                                                                           \
    do {                                                                                             \
        const int d_ = __builtin_amdgcn_readfirstlane((int)__builtin_bit_cast(unsigned long long, (double)(x_))); \
        asm volatile("" ::"s"(d_) : "memory");                                                       \
        const long long n_ = (long long)__builtin_amdgcn_s_memtime();                               \
        acc_ += n_ - f32_t;                                                                          \
        f32_t = n_;                                                                                  \
    } while (0)
#else
#define F32_MARK(acc_, x_) (void)0
#endif

// One wave factors the 32 x 32 diagonal block D at (c0, c0) of the LDS image: L_D -> lower,
// Dinv = L_D^{-1} -> upper (transposed, Dinv[j][i] at row c0 + i, column c0 + j) and sDi.
//
// (f64; f32 keeps diag_factor_rank8.)  The augmented [D; I] (64 x 32) lives in eight 16x16 MFMA accumulator tiles
// (acc[tr][tc][reg] = row 16 tr + lane % 16, column 16 tc + lane / 16 + 4 reg).  Column steps
// of 4: the 4 x 4 pivot block comes out by readlane, its factor and inverse are formed
// uniformly, the 4 panel columns -- ONE register of the tile column, lanes (row, column) --
// are solved by three shuffles and four FMAs per lane, and the trailing update is one
// v_mfma_f64_16x16x4f64 per tile straight from those panel registers (their (row, k) lane
// layout is the MFMA operand layout), with the finished columns masked to zero in the
// operand.  The identity rows (tiles 2, 3) end as L_D^{-T}.
template <typename T>
__device__ __forceinline__ void fact32(T* __restrict__ sS, T* __restrict__ sDi, int c0, int& fail,
                                       long long* fprof = nullptr) {
    constexpr int SL = SIL;
    const int lane = threadIdx.x & 63, lr = lane & 15, lk = lane >> 4;
    if constexpr (std::is_same<T, double>::value) {
        typedef Mfma<double> Tr;
        // tiles (tile row tr: 0, 1 = D, 2, 3 = identity; tile column tc) that can be nonzero:
        // (0, 1) is above the diagonal and (3, 1)'s partner (3, 0) stays zero (L^{-T} is upper)
        constexpr int TI[4][2] = {{0, -1}, {1, 2}, {3, 4}, {-1, 5}};
        d4_t acc[6];
#pragma unroll
        for (int tr = 0; tr < 4; tr++)
#pragma unroll
            for (int tc = 0; tc < 2; tc++) {
                if (TI[tr][tc] < 0) continue;
#pragma unroll
                for (int rg = 0; rg < 4; rg++) {
                    const int R = 16 * tr + lr, C = 16 * tc + Tr::orow(lk, rg);
                    double v;
                    if (tr < 2) v = (C <= R) ? sS[(c0 + R) + (c0 + C) * SL] : 0.0;
                    else v = (R - 32 == C) ? 1.0 : 0.0;
                    acc[TI[tr][tc]][rg] = v;
                }
            }
#ifdef GPRX_FACT32_PROF
        long long f32_t = (long long)__builtin_amdgcn_s_memtime(), f32_piv = 0, f32_pan = 0, f32_trl = 0;
#endif
        // Trailing MFMAs of step st: tiles (tr, tcp) for tcp = tc..1 (see f32_mfma_on).  Only the
        // one that updates the NEXT pivot tile is issued at once; the others are deferred into
        // the next step's pivot phase, one between each column of its 4 x 4 factor
        // (sched_barrier): issued back to back they held the wave's in-order issue for ~6 x 64
        // cycles in front of the pivot chain, the latency-bound critical path of the factor.
        double pa[2] = {0.0, 0.0}, pb[4] = {0.0, 0.0, 0.0, 0.0};  // the previous step's operands
#pragma unroll
        for (int st = 0; st < 8; st++) {
            const int k0 = 4 * st, tc = k0 / 16, rg = (k0 % 16) / 4, pl = k0 % 16;
            // deferred MFMA number m of step st - 1 (compile-time: the loop is unrolled)
            auto deferred = [&](int m) {
                if (st == 0) return;
                const int tcq = (4 * (st - 1)) / 16, tcn = tc;
                int cnt = 0;
#pragma unroll
                for (int tcp = tcq; tcp < 2; tcp++)
#pragma unroll
                    for (int tr = 0; tr < 4; tr++) {
                        if (TI[tr][tcp] < 0 || TI[tr][tcq] < 0) continue;
                        if (tr < 2 && tr < tcp) continue;
                        if (tr == tcn && tcp == tcn) continue;  // the critical one, already issued
                        if (cnt++ == m) acc[TI[tr][tcp]] = Tr::mma(pa[tcp], pb[tr], acc[TI[tr][tcp]]);
                    }
            };
            // the 4 x 4 pivot block (lower) of tile (tc, tc): P[i][j] at lane (pl + i) + 16 j;
            // its factor, then Q = L_P^{-1}, reduced to this lane's row qr = Q[lk][.]
            double qr[4];
            // the panel operands a[r][k0 + i] of every row, gathered to the lanes of column i: their
            // shuffles go out right after the last deferred MFMA of step st - 1 (the last write to
            // this tile column), so their LDS latency hides under the pivot chain of column 3 and the
            // 4 x 4 inverse instead of following them (GPRX_F32_LATE_SHFL: the round-3 order)
            double sv[4][4];
            auto gather_panel = [&]() {
#pragma unroll
                for (int tr = 0; tr < 4; tr++) {
                    if (TI[tr][tc] < 0) continue;
#pragma unroll
                    for (int i = 0; i < 4; i++) sv[tr][i] = __shfl(acc[TI[tr][tc]][rg], lr + 16 * i, 64);
                }
            };
            {
                double Lp[4][4], rq[4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    __builtin_amdgcn_sched_barrier(0);
                    deferred(i == 0 ? 0 : i + 1);
                    if (i == 0) deferred(1);
#ifndef GPRX_F32_LATE_SHFL
                    if (i == 3) gather_panel();
#endif
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int j = 0; j < i; j++) {
                        double v = rl_lane(acc[TI[tc][tc]][rg], pl + i + 16 * j);
#pragma unroll
                        for (int k = 0; k < j; k++) v = fma(-Lp[i][k], Lp[j][k], v);
                        Lp[i][j] = v * rq[j];
                    }
                    double dsum = rl_lane(acc[TI[tc][tc]][rg], pl + i + 16 * i);
#pragma unroll
                    for (int k = 0; k < i; k++) dsum = fma(-Lp[i][k], Lp[i][k], dsum);
                    rq[i] = rsqrt_full(dsum);  // (a non-positive or NaN dsum gives a NaN L_ii: checked at the end)
                    Lp[i][i] = dsum * rq[i];
                }
                __builtin_amdgcn_sched_barrier(0);
                // L_P goes to the image directly (lane 0; the output stage below skips the
                // diagonal 4 x 4 blocks): the pivot rows' panel values A_P Q^T would cost
                // accuracy on ill-conditioned blocks, and a per-lane select of L_P cost ~26
                // instructions on the latency-bound pivot chain
                if (lane == 0) {
#pragma unroll
                    for (int i = 0; i < 4; i++)
#pragma unroll
                        for (int j = 0; j <= i; j++) sS[(c0 + k0 + i) + (c0 + k0 + j) * SL] = Lp[i][j];
                }
                double Q[4][4];
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    Q[i][i] = rq[i];
#pragma unroll
                    for (int j = 0; j < i; j++) {
                        double v = 0.0;
#pragma unroll
                        for (int k = j; k < i; k++) v = fma(Lp[i][k], Q[k][j], v);
                        Q[i][j] = -v * rq[i];
                    }
                }
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    double v = 0.0;
#pragma unroll
                    for (int j = i; j < 4; j++) v = (lk == j) ? Q[j][i] : v;
                    qr[i] = v;
                }
            }
            F32_MARK(f32_piv, qr[0] + qr[1] + qr[2] + qr[3]);
#ifdef GPRX_F32_LATE_SHFL
            gather_panel();
#endif
            // panel: L[r][k0 + lk] = sum_{i <= lk} a[r][k0 + i] Q[lk][i] (D rows above k0 kept)
            double pv[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int tr = 0; tr < 4; tr++) {
                if (TI[tr][tc] < 0) continue;
                const double v = acc[TI[tr][tc]][rg];
                double nv = 0.0;
#pragma unroll
                for (int i = 0; i < 4; i++) nv = fma(sv[tr][i], qr[i], nv);
                const bool keep = tr < 2 && 16 * tr + lr < k0;
                pv[tr] = keep ? v : nv;  // (pivot rows: masked out of the trailing operands)
                acc[TI[tr][tc]][rg] = pv[tr];
            }
            F32_MARK(f32_pan, pv[0] + pv[1] + pv[2] + pv[3]);
            // trailing: tile (tr, tcp) -= panel(tr) panel_D(tcp)^T over the columns > k0 + 3:
            // operands for this step's MFMAs; the next pivot tile's one now, the rest deferred
#pragma unroll
            for (int tcp = 0; tcp < 2; tcp++) pa[tcp] = (16 * tcp + lr > k0 + 3) ? -pv[tcp] : 0.0;
#pragma unroll
            for (int tr = 0; tr < 4; tr++) pb[tr] = (tr < 2 && 16 * tr + lr < k0 + 4) ? 0.0 : pv[tr];
            if (st < 7) {
                const int tcn = (k0 + 4) / 16;
                acc[TI[tcn][tcn]] = Tr::mma(pa[tcn], pb[tcn], acc[TI[tcn][tcn]]);
            } else {  // last step: everything now
#pragma unroll
                for (int tcp = tc; tcp < 2; tcp++)
#pragma unroll
                    for (int tr = 0; tr < 4; tr++) {
                        if (TI[tr][tcp] < 0 || TI[tr][tc] < 0) continue;
                        if (tr < 2 && tr < tcp) continue;
                        acc[TI[tr][tcp]] = Tr::mma(pa[tcp], pb[tr], acc[TI[tr][tcp]]);
                    }
            }
        }
#ifdef GPRX_FACT32_PROF
        F32_MARK(f32_trl, acc[0][3] + acc[2][3] + acc[5][3]);
        if (fprof) {
            fprof[0] += f32_piv;
            fprof[1] += f32_pan;
            fprof[2] += f32_trl;
        }
#endif
        // out: L_D (lower incl. diagonal); Dinv from the identity rows (X = L_D^{-T},
        // Dinv[j][i] = X[i][j]) transposed into the upper triangle, its diagonal into sDi
#pragma unroll
        for (int tr = 0; tr < 4; tr++)
#pragma unroll
            for (int tc = 0; tc < 2; tc++) {
                if (TI[tr][tc] < 0) continue;
#pragma unroll
                for (int rg = 0; rg < 4; rg++) {
                    const int R = 16 * tr + lr, C = 16 * tc + Tr::orow(lk, rg);
                    const double v = acc[TI[tr][tc]][rg];
                    if (tr < 2) {
                        if (C <= R && (R >> 2) != (C >> 2)) sS[(c0 + R) + (c0 + C) * SL] = v;  // L_P: above
                    } else {
                        const int i = R - 32;
                        if (C > i) sS[(c0 + i) + (c0 + C) * SL] = v;
                        else if (C == i) sDi[c0 + i] = v;
                    }
                }
            }
        // info: the first column whose pivot was not positive (its L_ii and every later one NaN)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const double dg = sS[(c0 + (lane & 31)) * (SL + 1)];
        const unsigned long long bad = __ballot(lane < 32 && !(dg > 0.0));
        if (bad && fail < 0) fail = c0 + (int)__builtin_ctzll(bad);
    }
}

template <typename T>
__device__ __forceinline__ void diag_factor_blocked(T* __restrict__ A, int64_t ld, T* __restrict__ Linv,
                                                    int* __restrict__ info, int64_t col0, unsigned char* smem_raw,
                                                    const int t, long long* prof = nullptr) {
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    constexpr int SL = SIL;
    T* sS = reinterpret_cast<T*>(smem_raw);
    T* sDi = sS + (size_t)DB * SL;
    const int w = t >> 6, lane = t & 63, lr = lane & 15, lk = lane >> 4;
    long long pt0 = prof ? wall_clock64() : 0, pf = 0, pm = 0, pinv = 0;
    // ---- load (column c, rows r: coalesced; all loads in flight before the LDS stores) --
    {
        const int r = t & (DB - 1), cq = t >> 7;
        T v[DB / (NT / DB)];
#pragma unroll
        for (int u = 0; u < DB / (NT / DB); u++) v[u] = A[r + (int64_t)(cq + u * (NT / DB)) * ld];
#pragma unroll
        for (int u = 0; u < DB / (NT / DB); u++) sS[r + (cq + u * (NT / DB)) * SL] = v[u];
    }
    __syncthreads();
    const long long pload = prof ? wall_clock64() : 0;
    int fail = -1;
#pragma unroll 1
    for (int p = 0; p < 4; p++) {
        const int c0 = 32 * p;
        const long long tf0 = prof ? wall_clock64() : 0;
        // ---- 1: the 32 x 32 diagonal block, wave 0 -----------------------------------------
        if (w == 0) fact32<T>(sS, sDi, c0, fail);
        __syncthreads();
        if (prof) {
            const long long tn = wall_clock64();
            pf += tn - tf0;
            pm = tn;
        }
        if (p == 3) break;
        // ---- 2: L_rp = A_rp Dinv_p^T for the rows below (output tiles 16 x 16) -------------
        const int r0 = c0 + 32, nrt = (DB - r0) / 16;
        {
            acc_t acc[2];
            int tl[2];
            int nt = 0;
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int tt = w + 8 * u;
                tl[u] = tt;
                acc[u] = acc_t{0};
                if (tt < nrt * 2) {
                    nt = u + 1;
                    const int rt = tt >> 1, ct = tt & 1;
                    const int cc = ct * 16 + lr;  // output column (Dinv row)
#pragma unroll
                    for (int kq = 0; kq < 8; kq++) {
                        const int k = kq * 4 + lk;
                        const T av = (k < cc) ? sS[(c0 + k) + (c0 + cc) * SL] : (k == cc ? sDi[c0 + cc] : T(0));
                        const T bv = sS[(r0 + rt * 16 + lr) + (c0 + k) * SL];
                        acc[u] = Tr::mma(av, bv, acc[u]);
                    }
                }
            }
            __syncthreads();  // every read of A_rp done before the panel is overwritten
#pragma unroll
            for (int u = 0; u < 2; u++) {
                if (u < nt) {
                    const int rt = tl[u] >> 1, ct = tl[u] & 1;
#pragma unroll
                    for (int reg = 0; reg < 4; reg++)
                        sS[(r0 + rt * 16 + lr) + (c0 + ct * 16 + Tr::orow(lk, reg)) * SL] = acc[u][reg];
                }
            }
        }
        __syncthreads();
        // ---- 3: trailing lower tiles A_rr' -= L_rp L_r'p^T ---------------------------------
        {
            const int ntl = nrt * (nrt + 1) / 2;
#pragma unroll 1
            for (int tt = w; tt < ntl; tt += 8) {
                int rt = 0;
                while ((rt + 1) * (rt + 2) / 2 <= tt) rt++;
                const int ct = tt - rt * (rt + 1) / 2;
                acc_t acc = acc_t{0};
#pragma unroll
                for (int kq = 0; kq < 8; kq++) {
                    const int k = kq * 4 + lk;
                    const T av = sS[(r0 + ct * 16 + lr) + (c0 + k) * SL];
                    const T bv = sS[(r0 + rt * 16 + lr) + (c0 + k) * SL];
                    acc = Tr::mma(av, bv, acc);
                }
#pragma unroll
                for (int reg = 0; reg < 4; reg++) {
                    T& dst = sS[(r0 + rt * 16 + lr) + (r0 + ct * 16 + Tr::orow(lk, reg)) * SL];
                    dst -= acc[reg];
                }
            }
        }
        __syncthreads();
    }
    if (prof) pinv = wall_clock64();
    if (fail >= 0) atomicMin(info, (int)(col0 + fail + 1));  // wave 0, every lane the same value
    // ---- the off-diagonal 32-blocks of Linv, by distance --------------------------------------
    // Linv_ij (i > j) is kept transposed in the upper block (j, i): element (r, c) of Linv_ij at
    // sS[(32 j + c) + (32 i + r) SL].  Dinv_j's elements: (kk > c) upper of block (j, j), sDi.
#pragma unroll 1
    for (int dd = 1; dd < 4; dd++) {
        const int nb = 4 - dd, ntt = nb * 4;  // blocks j = 0 .. nb-1, four 16x16 tiles each
        // ntt <= 12 tiles: wave w takes tile w and tile w + 8
        // S = sum_{k=j}^{i-1} L_ik Linv_kj: out[r][c], b = L_i k-block rows, a = Linv_kj cols
        acc_t acc = acc_t{0}, acc2 = acc_t{0};
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int tt = w + 8 * u;
            if (tt >= ntt) continue;
            const int j = tt >> 2, i = j + dd, rt = (tt >> 1) & 1, ct = tt & 1;
            acc_t a0 = acc_t{0};
#pragma unroll 1
            for (int kb = j; kb < i; kb++) {
#pragma unroll
                for (int kq = 0; kq < 8; kq++) {
                    const int kk = kq * 4 + lk, cc = ct * 16 + lr;
                    T av;  // Linv_{kb, j}[kk][cc]
                    if (kb == j) av = (kk > cc) ? sS[(32 * j + cc) + (32 * j + kk) * SL] : (kk == cc ? sDi[32 * j + cc] : T(0));
                    else av = sS[(32 * j + cc) + (32 * kb + kk) * SL];
                    const T bv = sS[(32 * i + rt * 16 + lr) + (32 * kb + kk) * SL];  // L_{i,kb}[r][kk]
                    a0 = Tr::mma(av, bv, a0);
                }
            }
            if (u == 0) acc = a0;
            else acc2 = a0;
        }
        __syncthreads();  // reads of the previous level's blocks done
        // stage S (transposed, like Linv) in block (j, i)'s slot
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int tt = w + 8 * u;
            if (tt >= ntt) continue;
            const int j = tt >> 2, i = j + dd, rt = (tt >> 1) & 1, ct = tt & 1;
            const acc_t& a0 = u == 0 ? acc : acc2;
#pragma unroll
            for (int reg = 0; reg < 4; reg++) {
                const int r = rt * 16 + lr, c = ct * 16 + Tr::orow(lk, reg);
                sS[(32 * j + c) + (32 * i + r) * SL] = a0[reg];
            }
        }
        __syncthreads();
        // Linv_ij = -Dinv_i S: out[r][c] = -sum_k Dinv_i[r][k] S[k][c]
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int tt = w + 8 * u;
            if (tt >= ntt) continue;
            const int j = tt >> 2, i = j + dd, rt = (tt >> 1) & 1, ct = tt & 1;
            acc_t a0 = acc_t{0};
#pragma unroll
            for (int kq = 0; kq < 8; kq++) {
                const int kk = kq * 4 + lk, rr = rt * 16 + lr, cc = ct * 16 + lr;
                const T av = sS[(32 * j + cc) + (32 * i + kk) * SL];  // S[kk][cc]
                const T bv = (kk < rr) ? sS[(32 * i + kk) + (32 * i + rr) * SL]
                                       : (kk == rr ? sDi[32 * i + rr] : T(0));  // Dinv_i[rr][kk]
                a0 = Tr::mma(av, bv, a0);
            }
            if (u == 0) acc = a0;
            else acc2 = a0;
        }
        __syncthreads();  // S read before it is overwritten by Linv_ij
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int tt = w + 8 * u;
            if (tt >= ntt) continue;
            const int j = tt >> 2, i = j + dd, rt = (tt >> 1) & 1, ct = tt & 1;
            const acc_t& a0 = u == 0 ? acc : acc2;
#pragma unroll
            for (int reg = 0; reg < 4; reg++) {
                const int r = rt * 16 + lr, c = ct * 16 + Tr::orow(lk, reg);
                sS[(32 * j + c) + (32 * i + r) * SL] = -a0[reg];
            }
        }
        __syncthreads();
    }
    if (prof && t == 0) {
        const long long te = wall_clock64();
        prof[0] = pload - pt0;
        prof[1] = pf;
        prof[2] = pinv - pload - pf;
        prof[3] = te - pinv;
        (void)pm;
    }
    // ---- L and Linv out: coalesced columns ------------------------------------------------
    {
        const int r = t & (DB - 1);
        for (int c = t >> 7; c < DB; c += NT / DB) {
            if (r >= c) A[r + (int64_t)c * ld] = sS[r + c * SL];
            Linv[r + c * DB] = (r > c) ? sS[c + r * SL] : ((r == c) ? sDi[r] : T(0));
        }
    }
}

// ------------------------------------------------------------------------------------------
// Diagonal 128x128 block, blocked with LOOK-AHEAD (f64): the same LDS image and 32-column
// panels as diag_factor_blocked, but only the critical chain stays serial.  Per panel p
// (c0 = 32 p), 16 x 16 tile indices R, C = 0..7:
//   F(p)   wave 0: fact32 (the 32 x 32 diagonal block: L_pp, Dinv_p)
//          waves 1-7 meanwhile: the far trailing tiles of panel p-1 (C >= 2p + 2) and Linv's
//          row block p-1 (Linv_{p-1,j} = -Dinv_{p-1} sum_{k=j}^{p-2} L_{p-1,k} Linv_kj, one wave
//          per (j, 16-column) unit: S staged in the unit's own slot, wave-private, no barrier)
//   P(p)   all waves: L_rp = A_rp Dinv_p^T for the rows below
//   Ua(p)  all waves: the trailing tiles of the NEXT panel's columns only (C = 2p+2, 2p+3)
// so F(p+1) starts after a panel solve and a 32-column update instead of the whole trailing
// update and the Linv assembly.  Linv's last row block follows F(3).  Every region a phase
// writes is disjoint from what the concurrent waves read or write (see the phase comments).
// ------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T linv_at(const T* __restrict__ sS, const T* __restrict__ sDi, int R, int C) {
    // Linv[R][C] of the LDS image: strict lower part kept transposed in the upper triangle, the
    // diagonal in sDi (= sS + DB SIL), a zero in sDi[DB].  One unconditional load from a selected
    // address: a conditional load compiles to an exec-masked branch per element.
    (void)sDi;
    const int idx = (R > C) ? C + R * SIL : DB * SIL + (R == C ? R : DB);
    return sS[idx];
}

// one 16 x 16 lower tile (R, C) of the trailing matrix: A_RC -= L_{R,panel} L_{C,panel}^T (K = 32)
template <typename T>
__device__ __forceinline__ void la_trail_tile(T* __restrict__ sS, int c0, int R, int C, int lr, int lk) {
    typedef Mfma<T> Tr;
    typename Tr::acc_t acc = typename Tr::acc_t{0};
#pragma unroll
    for (int kq = 0; kq < 8; kq++) {
        const int k = c0 + kq * 4 + lk;
        acc = Tr::mma(sS[(16 * C + lr) + k * SIL], sS[(16 * R + lr) + k * SIL], acc);
    }
#pragma unroll
    for (int reg = 0; reg < 4; reg++) sS[(16 * R + lr) + (16 * C + Tr::orow(lk, reg)) * SIL] -= acc[reg];
}

// Linv row block p, column block j, 16-column half ct (rows 32 p .. 32 p + 31): one wave.
// S = sum_{kb_lo <= kb < kb_hi} L_{p,kb} Linv_{kb,j} (LA_LOAD: plus the partial S staged by an
// earlier call), staged transposed in the unit's own Linv slot; LA_FINISH: Linv_pj = -Dinv_p S.
enum { LA_LOAD = 1, LA_FINISH = 2 };
// gout (LA_FINISH): the finished Linv_pj half also goes straight to global memory (Linv,
// column-major, ld DB; write-through) from the registers
template <typename T>
__device__ __forceinline__ void la_linv_unit(T* __restrict__ sS, const T* __restrict__ sDi, int p, int j, int ct,
                                             int kb_lo, int kb_hi, int mode, int lr, int lk, T* gout = nullptr) {
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    acc_t s0 = acc_t{0}, s1 = acc_t{0};
    const int cc = 32 * j + 16 * ct + lr;  // Linv column this lane feeds
    if (mode & LA_LOAD) {
#pragma unroll
        for (int reg = 0; reg < 4; reg++) {
            const int c = 32 * j + 16 * ct + Tr::orow(lk, reg);
            s0[reg] = sS[c + (32 * p + lr) * SIL];
            s1[reg] = sS[c + (32 * p + 16 + lr) * SIL];
        }
    }
#pragma unroll 1
    for (int kb = kb_lo; kb < kb_hi; kb++) {
#pragma unroll
        for (int kq = 0; kq < 8; kq++) {
            const int kk = 32 * kb + kq * 4 + lk;
            const T av = linv_at(sS, sDi, kk, cc);  // Linv[kk][cc]
            s0 = Tr::mma(av, sS[(32 * p + lr) + kk * SIL], s0);
            s1 = Tr::mma(av, sS[(32 * p + 16 + lr) + kk * SIL], s1);
        }
    }
    // stage S (rows 32p + r, columns 32j + 16ct + c) transposed in the unit's own Linv slot
#pragma unroll
    for (int reg = 0; reg < 4; reg++) {
        const int c = 32 * j + 16 * ct + Tr::orow(lk, reg);
        sS[c + (32 * p + lr) * SIL] = s0[reg];
        sS[c + (32 * p + 16 + lr) * SIL] = s1[reg];
    }
    if (!(mode & LA_FINISH)) return;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // Linv_pj = -Dinv_p S
    acc_t o0 = acc_t{0}, o1 = acc_t{0};
#pragma unroll
    for (int kq = 0; kq < 8; kq++) {
        const int kk = kq * 4 + lk;
        const T av = sS[cc + (32 * p + kk) * SIL];  // S[kk][cc]
        o0 = Tr::mma(av, linv_at(sS, sDi, 32 * p + lr, 32 * p + kk), o0);
        o1 = Tr::mma(av, linv_at(sS, sDi, 32 * p + 16 + lr, 32 * p + kk), o1);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int reg = 0; reg < 4; reg++) {
        const int c = 32 * j + 16 * ct + Tr::orow(lk, reg);
        sS[c + (32 * p + lr) * SIL] = -o0[reg];
        sS[c + (32 * p + 16 + lr) * SIL] = -o1[reg];
        if (gout) {
            st_sc1(gout + (32 * p + lr) + (int64_t)c * DB, -o0[reg]);
            st_sc1(gout + (32 * p + 16 + lr) + (int64_t)c * DB, -o1[reg]);
        }
    }
}

// global stores of finished pieces, spread over the threads tid0 .. tid0 + nth - 1:
// L's panel q (rows 32 q .. 127, columns 32 q .. 32 q + 31) and Linv's row block q (all columns)
template <typename T>
__device__ __forceinline__ void la_store_lpanel(T* __restrict__ A, int64_t ld, const T* __restrict__ sS, int q, int tid,
                                                int nth) {
    const int nr = DB - 32 * q;
    for (int e = tid; e < 32 * nr; e += nth) {
        const int c = 32 * q + e / nr, r = 32 * q + e % nr;
        st_sc1(A + r + (int64_t)c * ld, sS[r + c * SIL]);  // write-through: no release fence needed
    }
}
template <typename T>
__device__ __forceinline__ void la_store_linv_rows(T* __restrict__ Linv, const T* __restrict__ sS,
                                                   const T* __restrict__ sDi, int q, int tid, int nth) {
    for (int e = tid; e < 32 * DB; e += nth) {
        const int c = e >> 5, r = 32 * q + (e & 31);
        st_sc1(Linv + r + c * DB, linv_at(sS, sDi, r, c));
    }
}

// row block q of Linv, columns 32 q .. 127 (Dinv_q and the zeros right of it); its columns < 32 q
// go out from the registers of the units that finish them (la_linv_unit gout), so the whole
// row block is stored during the next F phase, not in the factor's tail
template <typename T>
__device__ __forceinline__ void la_store_linv_diag(T* __restrict__ Linv, const T* __restrict__ sS,
                                                   const T* __restrict__ sDi, int q, int tid, int nth) {
    const int nc = DB - 32 * q;
    for (int e = tid; e < 32 * nc; e += nth) {
        const int r = 32 * q + (e & 31), c = 32 * q + (e >> 5);
        st_sc1(Linv + r + c * DB, linv_at(sS, sDi, r, c));
    }
}

// Dinv_q = L_qq^{-1} (the 32 x 32 diagonal block q of Linv, lower, zeros above) into Linv: the
// progressive TPART(k + 1, .) read it as soon as DIAGX(k)'s panel counter says so (the full row
// block q of Linv follows later with the same values)
template <typename T>
__device__ __forceinline__ void la_store_dinv(T* __restrict__ Linv, const T* __restrict__ sS, const T* __restrict__ sDi,
                                              int q, int tid, int nth) {
    for (int e = tid; e < 32 * 32; e += nth) {
        const int r = 32 * q + (e & 31), c = 32 * q + (e >> 5);
        st_sc1(Linv + r + c * DB, linv_at(sS, sDi, r, c));
    }
}

// F(p)'s side phase, waves wlo..7: the stores of what panel p-1 finished (L panel p-1; Linv row
// block p-1 right of column 32 (p-1), Dinv_{p-1} included), then the jobs -- Linv row block p-1
// (2 (p-1) units, each storing its finished half from its registers), at p = 3 also the partial
// sums of Linv row block 3 over kb < 2 (4 units), then the far trailing tiles of panel p-1
// (C >= 2p + 2, R >= C).  (Row block p-2 was stored here whole, and row block 2 in the factor's
// tail: 4096 of the tail's 6144 stores; chain step 53.0 -> 51.6 us, C2 523 -> 529 fits/s,
// profiles/r05r.  Also moving row block 3's kb = 2 term into F(3)'s side phase, by the waves
// that finish Linv_{2,j}, lengthened the F and P phases: 53.1 us.)
template <typename T>
__device__ __forceinline__ void la_side(T* __restrict__ A, int64_t ld, T* __restrict__ Linv, T* __restrict__ sS,
                                        const T* __restrict__ sDi, int p, int t, int w, int wlo, int lr, int lk) {
    const int nth = NT - 64 * wlo, tid = t - 64 * wlo;
    la_store_lpanel<T>(A, ld, sS, p - 1, tid, nth);
    la_store_linv_diag<T>(Linv, sS, sDi, p - 1, tid, nth);
    const int pl = p - 1, nl = 2 * pl, np3 = (p == 3) ? 4 : 0;
    const int cmin = 2 * p + 2, nc = 8 - cmin, nt = nc > 0 ? nc * (nc + 1) / 2 : 0;
    const int nw = 8 - wlo;
#pragma unroll 1
    for (int job = w - wlo; job < nl + np3 + nt; job += nw) {
        if (job < nl) {
            la_linv_unit<T>(sS, sDi, pl, job >> 1, job & 1, job >> 1, pl, LA_FINISH, lr, lk, Linv);
        } else if (job < nl + np3) {
            const int u = job - nl;
            la_linv_unit<T>(sS, sDi, 3, u >> 1, u & 1, u >> 1, 2, 0, lr, lk);
        } else {
            const int tt = job - nl - np3;  // lower tiles of the C >= cmin square, row-major
            int rr = 0;
            while ((rr + 1) * (rr + 2) / 2 <= tt) rr++;
            const int cc = tt - rr * (rr + 1) / 2;
            la_trail_tile<T>(sS, 32 * pl, cmin + rr, cmin + cc, lr, lk);
        }
    }
}

// from_lds: the block is already in the LDS image (diagx_ts left the syrk result there)
// pan (optional): the panel counter -- after F(p), p = 1..3, *pan = p: L panels 0..p-1 and
// Dinv_0..Dinv_{p-1} are stored (write-through); Dinv_3 right after F(3): *pan = 4
template <typename T>
__device__ __forceinline__ void diag_factor_la(T* __restrict__ A, int64_t ld, T* __restrict__ Linv,
                                               int* __restrict__ info, int64_t col0, unsigned char* smem_raw,
                                               const int t, long long* prof = nullptr, bool from_lds = false,
                                               int* pan = nullptr) {
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    constexpr int SL = SIL;
    T* sS = reinterpret_cast<T*>(smem_raw);
    T* sDi = sS + (size_t)DB * SL;
    const int w = t >> 6, lane = t & 63, lr = lane & 15, lk = lane >> 4;
    long long pt0 = prof ? wall_clock64() : 0, pf = 0, pside = 0, pfw = 0;
    if (!from_lds) {
        const int r = t & (DB - 1), cq = t >> 7;
        T v[DB / (NT / DB)];
#pragma unroll
        for (int u = 0; u < DB / (NT / DB); u++) v[u] = A[r + (int64_t)(cq + u * (NT / DB)) * ld];
#pragma unroll
        for (int u = 0; u < DB / (NT / DB); u++) sS[r + (cq + u * (NT / DB)) * SL] = v[u];
    }
    if (t == 0) sDi[DB] = T(0);  // linv_at's zero
    __syncthreads();
    const long long pload = prof ? wall_clock64() : 0;
    int fail = -1;
#pragma unroll 1
    for (int p = 0; p < 4; p++) {
        const int c0 = 32 * p;
        const long long tf0 = prof ? wall_clock64() : 0;
        // ---- F(p): wave 0 factors the diagonal block; the others finish panel p-1's side work
        // (fact32 touches block (p, p) only; the far trailing tiles have C >= 2p + 2; the Linv
        // units write rows 32 (p - 1) .. 32 p - 1 (p = 3: also 96 .. 127) of columns < 32 (p - 1),
        // transposed: LDS columns >= 32 (p - 1), rows < 32 (p - 1); the stores only read)
        if (w == 0) {
            fact32<T>(sS, sDi, c0, fail, prof ? prof + 4 : nullptr);
            if (prof) pfw += wall_clock64() - tf0;
        } else if (p > 0) {
            la_side<T>(A, ld, Linv, sS, sDi, p, t, w, 1, lr, lk);
            if (pan) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the panel's stores drained
        }
        __syncthreads();
        if (pan && p > 0 && w == 0) st_agent(pan, p);
        if (prof) {
            const long long tn = wall_clock64();
            pf += tn - tf0;
        }
        if (p == 3) break;
        const long long ts0 = prof ? wall_clock64() : 0;
        // ---- P(p): L_rp = A_rp Dinv_p^T for the rows below; one 16-row tile per wave (both of
        // its 16-column halves), so a wave overwrites only what it read: no barrier inside.
        // The explicit inverse alone is not backward stable when L_pp is ill-conditioned (a
        // sparse-GP normal matrix with cond 1.5e13 lost positive definiteness at pivot 35):
        // one step of refinement, X += (A - X L_pp^T) Dinv_p^T, restores the substitution's
        // accuracy (numpy emulation: residual 5.8e-10 against 4.7e-10 for dtrsm).
        const int r0 = c0 + 32, nrt = (DB - r0) / 16;
        if (w < nrt) {
            acc_t a0 = acc_t{0}, a1 = acc_t{0};
            const int rr = r0 + w * 16 + lr;
            T av0[4], av1[4];
#pragma unroll
            for (int reg = 0; reg < 4; reg++) {  // A_rp in the accumulator layout (for the residual)
                av0[reg] = sS[rr + (c0 + Tr::orow(lk, reg)) * SL];
                av1[reg] = sS[rr + (c0 + 16 + Tr::orow(lk, reg)) * SL];
            }
            T dmax = T(0);  // max |Dinv_p| over the entries this lane feeds
#pragma unroll
            for (int kq = 0; kq < 8; kq++) {
                const int k = kq * 4 + lk;
                const T bv = sS[rr + (c0 + k) * SL];
                const T d0 = linv_at(sS, sDi, c0 + lr, c0 + k), d1 = linv_at(sS, sDi, c0 + 16 + lr, c0 + k);
                dmax = fmax(dmax, fmax(fabs(d0), fabs(d1)));
                a0 = Tr::mma(d0, bv, a0);
                a1 = Tr::mma(d1, bv, a1);
            }
            // est = max|Dinv_p| max_i L_ii (<= cond_2(L_pp), within a factor 32^2 of it): a
            // well-conditioned block skips the refinement -- its explicit-inverse error is then
            // no larger than that of the 128-block TRSM tasks (which also use explicit inverses)
            // (min of the 32 diagonal words by broadcast LDS reads, the max test by one ballot:
            // two 6-step shuffle reductions cost ~0.45 us per panel on the chain)
            T dimin = sDi[c0];  // 1 / L_ii
#pragma unroll
            for (int i = 1; i < 32; i++) dimin = fmin(dimin, sDi[c0 + i]);
            const bool refine = __ballot(dmax > T(32) * dimin) != 0;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int reg = 0; reg < 4; reg++) {  // X0 (kept in a0, a1) through LDS to the operand layout
                sS[rr + (c0 + Tr::orow(lk, reg)) * SL] = a0[reg];
                sS[rr + (c0 + 16 + Tr::orow(lk, reg)) * SL] = a1[reg];
            }
            if (refine) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            acc_t q0 = acc_t{0}, q1 = acc_t{0};  // X0 L_pp^T
#pragma unroll
            for (int kq = 0; kq < 8; kq++) {
                const int k = kq * 4 + lk;
                const T xv = sS[rr + (c0 + k) * SL];
                const T l0v = sS[(c0 + lr) + (c0 + k) * SL], l1v = sS[(c0 + 16 + lr) + (c0 + k) * SL];
                const T l0 = (lr >= k) ? l0v : T(0), l1 = (16 + lr >= k) ? l1v : T(0);  // above: Dinv
                q0 = Tr::mma(l0, xv, q0);
                q1 = Tr::mma(l1, xv, q1);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int reg = 0; reg < 4; reg++) {  // R = A - X0 L^T, to the operand layout
                sS[rr + (c0 + Tr::orow(lk, reg)) * SL] = av0[reg] - q0[reg];
                sS[rr + (c0 + 16 + Tr::orow(lk, reg)) * SL] = av1[reg] - q1[reg];
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int kq = 0; kq < 8; kq++) {
                const int k = kq * 4 + lk;
                const T rv = sS[rr + (c0 + k) * SL];
                a0 = Tr::mma(linv_at(sS, sDi, c0 + lr, c0 + k), rv, a0);
                a1 = Tr::mma(linv_at(sS, sDi, c0 + 16 + lr, c0 + k), rv, a1);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
            for (int reg = 0; reg < 4; reg++) {
                sS[rr + (c0 + Tr::orow(lk, reg)) * SL] = a0[reg];
                sS[rr + (c0 + 16 + Tr::orow(lk, reg)) * SL] = a1[reg];
            }
            }  // refine
        }
        __syncthreads();
        // ---- Ua(p): the next panel's columns (C = 2p+2, 2p+3; R >= C), all waves -------------
        {
            const int Cn = 2 * p + 2, n0 = 8 - Cn, ntl = n0 + (n0 - 1);
#pragma unroll 1
            for (int tt = w; tt < ntl; tt += 8) {
                const int C = tt < n0 ? Cn : Cn + 1;
                const int R = tt < n0 ? Cn + tt : Cn + 1 + (tt - n0);
                la_trail_tile<T>(sS, c0, R, C, lr, lk);
            }
        }
        __syncthreads();
        if (prof) pside += wall_clock64() - ts0;
    }
    if (fail >= 0) atomicMin(info, (int)(col0 + fail + 1));  // wave 0, every lane the same value
    // Linv's last row block: the kb = 2 term and -Dinv_3 S (6 units, waves 0-5), each storing its
    // half block to global memory from its registers; the stores of L panel 3 and the rest of row
    // block 3 (its diagonal block Dinv_3 and the zeros right of it) by waves 6-7 meanwhile
    // (GPRX_LA_TAIL_LDS: row block 3 from LDS after a barrier, the round-3 order)
#ifndef GPRX_LA_TAIL_LDS
    constexpr bool direct = true;
#else
    constexpr bool direct = false;
#endif
    if (w < 6) {
        const int j = w >> 1;
        la_linv_unit<T>(sS, sDi, 3, j, w & 1, 2, 3, (j < 2 ? LA_LOAD : 0) | LA_FINISH, lr, lk, direct ? Linv : nullptr);
    } else {
        if (pan && w == 6) {  // Dinv_3 first: the progressive parts' last input
            la_store_dinv<T>(Linv, sS, sDi, 3, lane, 64);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            st_agent(pan, 4);
        }
        la_store_lpanel<T>(A, ld, sS, 3, t - 384, 128);
        if (direct)  // row block 3, columns 96..127 (Dinv_3, zeros above its diagonal)
            for (int e = t - 384; e < 32 * 32; e += 128) {
                const int r = 96 + (e & 31), c = 96 + (e >> 5);
                st_sc1(Linv + r + c * DB, linv_at(sS, sDi, r, c));
            }
    }
    __syncthreads();
    if (!direct) la_store_linv_rows<T>(Linv, sS, sDi, 3, t, NT);
    if (prof && t == 0) {  // load, F phases (barrier to barrier), P + Ua phases, fact32 alone
        prof[0] = pload - pt0;
        prof[1] = pf;
        prof[2] = pside;
        prof[3] = pfw;
    }
}

// GPRX_TP_PROG (A/B builds): the progressive parts (tpart_prog) and DIAGX's panel counter.  Off
// by default: same-box A/Bs (profiles/r04c_*, r04d_*) measured the chain step unchanged (C2
// 1829 us against 1815 for the Linv form without the panel counter; the counter's stores and
// drains cost DIAGX ~1.3 us per step, the early X_3 saves ~2 us of the parts' T phase, and the
// parts' S phase, not T, dominates after DIAGX(k-1) ends) and C3 0.1-0.4% slower.
#ifdef GPRX_TP_PROG
__host__ __device__ constexpr bool tp_linv_form() { return false; }
#else
__host__ __device__ constexpr bool tp_linv_form() { return true; }
#endif
// TPART workgroups per split diagonal step: f64 (the Linv form) eight -- part p = C + 4 h takes
// the column groups C, 7 - C of T's rows 64 h .. 64 h + 63 and the S quarter of tile-rows C, 7 - C
// over T's columns 64 h .. 64 h + 63 (tpart_run8) -- f32 and the progressive form four
// (GPRX_TP_PARTS4: four for f64 too)
#ifdef GPRX_TP_PARTS4
__host__ __device__ constexpr int tp_parts(bool f64) { return (void)f64, 4; }
#else
__host__ __device__ constexpr int tp_parts(bool f64) { return f64 && tp_linv_form() ? 8 : 4; }
#endif
#ifdef GPRX_NO_SPLIT  // (A/B builds: the split diagonal step compiled out)
constexpr bool SPLIT_CODE = false;
#else
constexpr bool SPLIT_CODE = true;
#endif
#ifndef GPRX_DIAG_RANK8
constexpr bool DIAG_LA = true;
#else
constexpr bool DIAG_LA = false;
#endif
// from_lds (f64 look-ahead form only): the block is in the LDS image already (diagx_ts)
// (out of line: its registers (fact32's accumulators, the pivot block) no longer count against
// the task loop, which sits at 256 VGPRs -- inlined, any growth of the loop spilled, and a
// spill reload inside the update mainloop broke its counted vmcnt pipelining)
// pub (optional): publish *pub = pub_v when the block is stored, inside the call -- the
// callee-saved registers are restored after it (scratch loads), not before the chain goes on
__device__ __forceinline__ void publish(int* flag, int v, bool release);
template <typename T>
__device__ __noinline__ void diag_factor(T* __restrict__ A, int64_t ld, T* __restrict__ Linv, int* __restrict__ info,
                                         int64_t col0, unsigned char* smem_raw, const int t, int* dbg = nullptr,
                                         long long* prof = nullptr, bool from_lds = false, int* pub = nullptr,
                                         int pub_v = 0, int* pan = nullptr) {
    // f64: the blocked factor with look-ahead (diag_factor_la: 43 us per block in isolation
    // against 50.6 for the rank-8 image, scripts/diag_bench.py); its stores are write-through
    // (sc1), so the publication needs no release fence.  f32 (and GPRX_DIAG_RANK8): the
    // rank-8 register image, plain stores and the release fence.
    constexpr bool la = std::is_same<T, double>::value && DIAG_LA;
    if constexpr (la) diag_factor_la<T>(A, ld, Linv, info, col0, smem_raw, t, prof, from_lds, pan);
    else diag_factor_rank8<T>(A, ld, Linv, info, col0, smem_raw, t, dbg, prof);
    if (pub) publish(pub, pub_v, !la);
}

// Developer microbenchmark (gprx_dev_bench what 11 / 12): one workgroup factors `reps` fresh
// 128 x 128 blocks (A + r * DB * ld) back to back with variant V (0 rank-8, 1 blocked, 2 look-ahead); prof
// accumulates the variant's phase ticks (wall clock, 100 MHz) over the reps.
template <typename T, int V>
__global__ __launch_bounds__(NT) void diag_bench_kernel(T* A, int64_t ld, T* Linv, int* info, long long* prof,
                                                        int reps) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    long long acc[5] = {0, 0, 0, 0, 0};
    long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // [4..6]: fact32 core-clock split (GPRX_FACT32_PROF)
    for (int r = 0; r < reps; r++) {
        const long long t0 = wall_clock64();
        if (V == 0) diag_factor_rank8<T>(A + (int64_t)r * DB * ld, ld, Linv, info, 0, smem_raw, threadIdx.x, nullptr, ph);
        else if (V == 1) diag_factor_blocked<T>(A + (int64_t)r * DB * ld, ld, Linv, info, 0, smem_raw, threadIdx.x, ph);
        else diag_factor_la<T>(A + (int64_t)r * DB * ld, ld, Linv, info, 0, smem_raw, threadIdx.x, ph);
        __syncthreads();
        const long long t1 = wall_clock64();
        acc[0] += ph[0];
        acc[1] += ph[1];
        acc[2] += ph[2];
        acc[3] += ph[3];
        acc[4] += t1 - t0;
    }
    if (threadIdx.x == 0) {
        for (int u = 0; u < 5; u++) prof[u] = acc[u];
        for (int u = 0; u < 3; u++) prof[5 + u] = ph[4 + u];
    }
}

template <typename T>
void launch_diag_bench(int variant, T* A, int64_t ld, T* Linv, int* info, long long* prof, int reps, hipStream_t s) {
    const size_t lds = diag_lds<T>() + 64;
    auto go = [&](auto kfn) {
        GPRX_HIP(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(kfn, dim3(1), dim3(NT), lds, s, A, ld, Linv, info, prof, reps);
    };
    if (variant == 0 || !std::is_same<T, double>::value) go(diag_bench_kernel<T, 0>);
    else if (variant == 1) go(diag_bench_kernel<T, 1>);
    else go(diag_bench_kernel<T, 2>);
    GPRX_HIP(hipGetLastError());
}
template void launch_diag_bench<double>(int, double*, int64_t, double*, int*, long long*, int, hipStream_t);
template void launch_diag_bench<float>(int, float*, int64_t, float*, int*, long long*, int, hipStream_t);

// ------------------------------------------------------------------------------------------
// Hand-off helpers
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int ld_agent(const int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(int* p, int v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// every wave's stores complete, then wave 0 releases and publishes *flag = v.  Wave 0 acts
// with ALL its lanes (same value to the same word): no lane-divergent code near the task
// loop's back edge, where the structurizer was seen to sink a `lane == 0` block past the
// next iteration's barrier (a hang).
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// release = false: every handed-off byte was stored sc1 (tile_gemm), so draining the stores
// (vmcnt(0) in every wave, then the barrier) is the release; the consumer still acquires.
__device__ __forceinline__ void publish(int* flag, int v, bool release) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave_id() == 0) {
        if (release) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_agent(flag, v);
    }
}

// two counters after one drain (a paired update's tiles)
__device__ __forceinline__ void publish2(int* f1, int* f2, int v) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave_id() == 0) {
        st_agent(f1, v);
        st_agent(f2, v);
    }
}

// stores of this workgroup visible to its own later loads (same CU)
__device__ __forceinline__ void local_sync() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

template <typename T>
constexpr size_t pt_lds_bytes() {
    return gemm_lds<T>() > diag_lds<T>() ? gemm_lds<T>() : diag_lds<T>();
}
static_assert(tall_lds<double>() <= pt_lds_bytes<double>() && tall_lds<float>() <= pt_lds_bytes<float>(),
              "the paired update's ring exceeds the LDS of the launch");

template <typename T>
struct Args {
    T* A;
    int64_t ld;
    T* Linv;
    const int4* tasks;
    int ntasks;
    int nc;        // column blocks (= diagonal blocks)
    int nv;        // columns of the ver counter array (nc; 2 nc with the C tiles of DIST LML mode)
    int* ctl;      // [C_NCTL] control words, then lcnt[nr], then ver[nr * nc]
    int* lcnt;
    int* ver;
    int* info;
    long long tlimit;  // wall-clock ticks (100 MHz) a single wait may take
    int* dbg;          // GPRX_PT_DEBUG: per-workgroup {ticket, phase, i, j} in pinned host memory
    int variant;       // GPRX_PT_VARIANT debug bits: 1 no TRSM math, 2 no UPD math, 4 no diag factor
    long long* trace;  // GPRX_PT_TRACE: per ticket {ticket taken, inputs ready, published, workgroup}
    long long* xt;     // GPRX_PT_TRACE, one GPU: the split step's phase stamps (TpCtx::xt)
    const TileBuild<T>* tb;  // BUILD tasks: covariance tiles from pair statistics (device copy,
                             // read per task: as kernel arguments they stayed live in SGPRs and
                             // pushed the whole kernel into spills)
    const PtDist<T>* dist;   // distributed factorisation (potrf_tiles_kernel<T, true> only)
    // split diagonal step (f64): TPART(k, p) tasks form L_{k,k-1} and S = A_kk - L L^T in
    // quarters; DIAGX(k) copies S and factors it (diagx_split)
    int split;
    T* pbuf;     // DB x DB: S, its lower tiles written by the parts
    int* tflag;  // [nc][TP_STRIDE] TPART(k, p) state: 1 its A operand is read, 2 its T stored, 3 its S quarter
                 // stored; [TP_DPAN] DIAGX(k)'s published panels
};


// Wave 0 waits until the task's inputs are final (all lanes load the same words; the values
// are made wave-uniform, so the loop is a scalar loop with no divergence).  Returns false on
// timeout or when another workgroup raised the error flag.
__device__ __forceinline__ int ld_uni(const int* p) { return __builtin_amdgcn_readfirstlane(ld_agent(p)); }
// flag words another rank stores into this rank's mailbox: system scope
__device__ __forceinline__ unsigned ld_sys(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A timed-out wait of the distributed factorisation leaves one record (the first) at
// check_err[DIST_TO_REC..+7]: kind (1 inputs, 2 window release), task type, i, j, b0 | nb << 16,
// detail (inputs: bit mask of the unmet conditions; release: the consumer rank), the value seen,
// the ticket.  gprx_dist.cpp prints it with the fit's timeout error.
constexpr int DIST_TO_REC = 132;
__device__ __forceinline__ void dist_note_timeout(int* rec, int kind, int type, int i, int j, int b0nb, int detail,
                                                  int seen) {
    if (!rec) return;
    if (__hip_atomic_fetch_add(rec, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
    if (atomicCAS(rec, 0, kind) != 0) return;
    rec[1] = type;
    rec[2] = i;
    rec[3] = j;
    rec[4] = b0nb;
    rec[5] = detail;
    rec[6] = seen;
}

// ---- distributed factorisation (DIST): packed storage, mailbox pushes -----------------------
// tile (i, j) of this rank's own row block i in the packed storage (ld DB): matrix / label rows
// keep columns 0..i, identity row E_a = nc + 1 + a columns a..nc-1, then C columns E_0..E_a
template <typename T>
__device__ __forceinline__ T* dist_tile(T* A, const PtDist<T>& D, int i, int j) {
    const int li = __builtin_amdgcn_readfirstlane(D.loc[i]);
    int col = j;
    if (i > D.nc) {
        const int aa = i - D.nc - 1;
        col = (j < D.nc) ? j - aa : D.nc - aa + (j - D.nc - 1);
    }
    const int64_t ro = D.roff[li];
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)ro), hi = __builtin_amdgcn_readfirstlane((uint32_t)(ro >> 32));
    return A + (int64_t)(((uint64_t)hi << 32) | lo) + (int64_t)col * DB * DB;
}
// counter column of tile (i, j): the C tiles (j = E_c) after the nc matrix columns
__device__ __forceinline__ int dist_col(int nc, int j) { return j > nc ? j - 1 : j; }

template <typename T>
__device__ __forceinline__ unsigned* dist_flags(const PtDist<T>& D, int q) {
    const uint64_t b = D.mb[q] + (uint64_t)D.o_flags;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return reinterpret_cast<unsigned*>(((uint64_t)hi << 32) | lo);
}
// window slot t (= (b mod ww) nr + j) of rank q
template <typename T>
__device__ __forceinline__ char* dist_win(const PtDist<T>& D, int q, int64_t t) {
    const int64_t tpp = D.tpp;
    const int64_t pc = t / tpp;
    const uint64_t b = D.wpc[(int64_t)q * D.npc + pc] + (uint64_t)((t - pc * tpp) * DB * DB * (int64_t)sizeof(T));
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return reinterpret_cast<char*>(((uint64_t)hi << 32) | lo);
}
template <typename T>
__device__ __forceinline__ char* dist_mb(const PtDist<T>& D, int q, int64_t off) {
    const uint64_t b = D.mb[q] + (uint64_t)off;
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b), hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return reinterpret_cast<char*>(((uint64_t)hi << 32) | lo);
}

// ranks other than r that consume row block j (bit q)
template <typename T>
__device__ __forceinline__ unsigned dist_consumers(const PtDist<T>& D, int j) {
    unsigned m = 0;
    for (int q = 0; q < D.g; q++)
        if (q != D.r && D.cons[(int64_t)q * D.nr + j]) m |= 1u << q;
    return __builtin_amdgcn_readfirstlane(m);
}

// Wave 0: wait until every rank in `mask` released panel p (its window slot may be refilled);
// ranks with no window-reading chunk on p never store the flag and are not waited for.
template <typename T>
__device__ bool dist_wait_release(const Args<T>& a, const PtDist<T>& D, unsigned mask, int p) {
    if (p < 0) return true;
    const unsigned* fl = dist_flags(D, D.r) + dist_f_rel(D.nr, D.nc);
    const long long t0 = wall_clock64();
    for (int q = 0; q < D.g; q++) {
        if (!((mask >> q) & 1) || __builtin_amdgcn_readfirstlane(D.need[(int64_t)q * D.nc + p]) == 0) continue;
        unsigned seen;
        while ((seen = __builtin_amdgcn_readfirstlane(ld_sys(fl + (int64_t)q * D.nc + p))) != D.ep) {
            if (ld_uni(a.ctl + C_ERR)) return false;
            if (wall_clock64() - t0 > a.tlimit) {
                if ((threadIdx.x & 63) == 0) dist_note_timeout(D.check_err + DIST_TO_REC, 2, -1, D.r, p, 0, q, (int)seen);
                st_agent(a.ctl + C_ERR, 1);
                return false;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    return true;
}

// The whole workgroup: copy one DB x DB tile (contiguous, written by this workgroup and
// drained: its stores are visible to this CU) to byte offset `off` of the mailbox of every
// rank in `mask` (off < 0: to window slot tag_idx), then set each one's flag word `fidx` to the
// epoch.  Across devices (D.wt) the
// copies are 16-byte `sc0 sc1` stores (written through to the destination, not left dirty in
// this XCD's L2), so the flag needs only every wave's s_waitcnt vmcnt(0) and a barrier -- no
// buffer_wbl2, which would write back every dirty line of the XCD's L2 (the update tasks'
// tiles) on each push (MI355X_MICROARCH.md, the {sc0 sc1 stores} form; the consumer acquires
// before its loads).  Ranks of one device: plain stores and one system-scope release.
template <typename T>
__device__ void dist_push(const T* src, const PtDist<T>& D, unsigned mask, int64_t off, int64_t fidx, const int t,
                          int64_t tag_idx = -1, unsigned tag = 0) {
    if (!mask) return;
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    constexpr int NV = DB * DB * (int)sizeof(T) / 16 / NT;  // 16-byte vectors per thread
    constexpr int CH = 4;
    const bool wt = __builtin_amdgcn_readfirstlane(D.wt) != 0;
    if (wave_id() == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // this CU's L1: no stale lines of src
    __syncthreads();
    const u4* s4 = reinterpret_cast<const u4*>(src);
#pragma unroll
    for (int c = 0; c < NV; c += CH) {
        u4 v[CH];
#pragma unroll
        for (int u = 0; u < CH; u++) v[u] = s4[t + (c + u) * NT];
        for (int q = 0; q < D.g; q++) {
            if (!((mask >> q) & 1)) continue;
            u4* d4 = reinterpret_cast<u4*>(off < 0 ? dist_win(D, q, tag_idx) : dist_mb(D, q, off));
            if (wt) {
#pragma unroll
                for (int u = 0; u < CH; u++)
                    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(d4 + t + (c + u) * NT), "v"(v[u])
                                 : "memory");
            } else {
#pragma unroll
                for (int u = 0; u < CH; u++) d4[t + (c + u) * NT] = v[u];
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (wave_id() == 0) {
        if (!wt) {  // ranks of one device: plain stores, one release
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (D.check && tag_idx >= 0)
            for (int q = 0; q < D.g; q++)
                if ((mask >> q) & 1) st_sys(reinterpret_cast<unsigned*>(dist_mb(D, q, D.o_tags)) + tag_idx, tag);
        for (int q = 0; q < D.g; q++)
            if ((mask >> q) & 1) st_sys(dist_flags(D, q) + fidx, D.ep);
    }
}

// GPRX_DIST_CHECK: the window slots of row j, panels b0.. b0 + nb - 1, hold exactly those tiles
// of this fit (tag = epoch << 16 | panel + 1); counts mismatches into check_err[which]
template <typename T>
__device__ void dist_check_tags(const PtDist<T>& D, int j, int b0, int nb, int which) {
    const int lane = threadIdx.x & 63;
    if (lane < nb) {
        const int b = b0 + lane;
        const unsigned* tg = reinterpret_cast<const unsigned*>(dist_mb(D, D.r, D.o_tags)) + (int64_t)(b % D.ww) * D.nr + j;
        const unsigned want = (D.ep << 16) | (unsigned)(b + 1);
        const unsigned got = ld_sys(tg);
        if (got != want) {
            atomicAdd(D.check_err + which, 1);
            const int e = atomicAdd(D.check_err + 2, 1);
            if (e < 32) {  // log: which, row, panel, time
                int* lg = D.check_err + 4 + 4 * e;
                lg[0] = which;
                lg[1] = j;
                lg[2] = b;
                lg[3] = (int)(wall_clock64() & 0x7fffffff);
            }
        }
    }
}

// Wave 0 of an update that read row j from the window: count the chunk on its panels; the
// chunk completing a panel's count stores the release flag into every other rank's mailbox.
template <typename T>
__device__ void dist_release(const PtDist<T>& D, int b0, int nb) {
    // lane l < nb counts the chunk on panel b0 + l (its own counter word); the others add 0.
    // Integer masks throughout: the 64-bit ballot / count-trailing-zeros form of this loop was
    // seen to release panel b0 + 32 together with panel b0 (lane 32 of a 32-wide chunk).
    const int lane = threadIdx.x & 63;
    const int valid = lane < nb ? 1 : 0;
    const int p = b0 + (valid ? lane : 0);
    const int old = __hip_atomic_fetch_add(D.ucnt + p, valid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int needv = D.need[(int64_t)D.r * D.nc + p];
    const int dn = valid & (old + 1 == needv ? 1 : 0);
    for (int l = 0; l < nb; l++) {
        if (!__builtin_amdgcn_readfirstlane(__shfl(dn, l))) continue;
        for (int q = 0; q < D.g; q++)
            if (q != D.r) st_sys(dist_flags(D, q) + dist_f_rel(D.nr, D.nc) + (int64_t)D.r * D.nc + b0 + l, D.ep);
    }
}

template <typename T, bool DIST>
__device__ bool wait_inputs(const Args<T>& a, int type, int i, int j, int b0, int nb) {
    const int* vp;
    int vwant;
    const int* vp2;
    int vwant2;
    const int* lp1;
    int lwant1;
    const int* lp2;
    int lwant2;
    // DIST: one dependency may be data of another rank: its flag words in this rank's mailbox
    // (Linv_k: one word; the tiles of a remote row: one word per panel of the chunk)
    const unsigned* rp = nullptr;
    int rn = 0;
    unsigned ep = 0;
    const int* lp3 = nullptr;  // T_UPD2: the second row's final blocks (>= lwant1)
    if (type == T_TPART) {  // its A operand final (Linv_{i-1} is waited for inside the task)
        vp = a.ver + (int64_t)i * a.nv + (i - 1);
        vwant = i - 1;
        vp2 = vp;
        vwant2 = vwant;
        lp1 = a.lcnt + i;
        lwant1 = 0;
        lp2 = lp1;
        lwant2 = 0;
    } else if (type == T_DIAGX && i > 0 && a.split) {  // A_ii through panel i-2
        vp = a.ver + (int64_t)i * a.nv + i;
        vwant = i - 1;
        vp2 = vp;
        vwant2 = vwant;
        lp1 = a.lcnt + i;
        lwant1 = 0;
        lp2 = lp1;
        lwant2 = 0;
        // (A_kk only: the TPART products are waited for inside the task, A_kk loads meanwhile)
    } else if (type == T_DIAGX && i == 0) {  // the first diagonal tile is built
        vp = a.ver;
        vwant = 0;
        vp2 = vp;
        vwant2 = 0;
        lp1 = a.lcnt;
        lwant1 = 0;
        lp2 = lp1;
        lwant2 = 0;
    } else if (type == T_BUILD) {
        return true;
    } else if (type == T_DIAGX) {
        vp = a.ver + (int64_t)i * a.nv + (i - 1);
        vwant = i - 1;
        vp2 = a.ver + (int64_t)i * a.nv + i;
        vwant2 = i - 1;
        lp1 = a.lcnt + (i - 1);
        lwant1 = i;
        lp2 = lp1;
        lwant2 = lwant1;
        if constexpr (DIST) {
            const PtDist<T>& D = *a.dist;
            if (__builtin_amdgcn_readfirstlane(D.loc[i - 1]) < 0) {  // Linv_{i-1} pushed by its rank
                lp1 = lp2 = a.lcnt + i;
                lwant1 = lwant2 = 0;
                rp = dist_flags(D, D.r) + dist_f_linv(D.nr, D.nc) + (i - 1);
                rn = 1;
                ep = D.ep;
            }
        }
    } else if (!DIST && type == T_UPD2) {  // tiles (i, j), (i + 1, j); rows i, i + 1 and j final through the chunk
        vp = a.ver + (int64_t)i * a.nv + j;
        vwant = b0;
        vp2 = a.ver + (int64_t)(i + 1) * a.nv + j;
        vwant2 = b0;
        lp1 = a.lcnt + i;
        lwant1 = b0 + nb;
        lp2 = a.lcnt + j;
        lwant2 = b0 + nb;
        lp3 = a.lcnt + i + 1;
    } else if (type == T_TRSM) {
        vp = a.ver + (int64_t)i * a.nv + j;
        vwant = j;
        vp2 = vp;
        vwant2 = vwant;
        lp1 = a.lcnt + j;
        lwant1 = j + 1;
        lp2 = lp1;
        lwant2 = lwant1;
        if constexpr (DIST) {
            const PtDist<T>& D = *a.dist;
            if (__builtin_amdgcn_readfirstlane(D.loc[j]) < 0) {  // Linv_j pushed by its rank
                lp1 = lp2 = a.lcnt + i;
                lwant1 = lwant2 = 0;
                rp = dist_flags(D, D.r) + dist_f_linv(D.nr, D.nc) + j;
                rn = 1;
                ep = D.ep;
            }
        }
    } else {
        const int jc = DIST ? dist_col(a.dist->nc, j) : j;
        vp = a.ver + (int64_t)i * a.nv + jc;
        vwant = b0;
        vp2 = vp;
        vwant2 = vwant;
        lp1 = a.lcnt + i;
        lwant1 = b0 + nb;
        lp2 = a.lcnt + j;
        lwant2 = b0 + nb;
        if constexpr (DIST) {
            const PtDist<T>& D = *a.dist;
            if (__builtin_amdgcn_readfirstlane(D.loc[j]) < 0) {  // row j's tiles: pushed, one flag per panel
                lp2 = lp1;
                rp = dist_flags(D, D.r) + dist_f_tile() + (int64_t)j * D.nc + b0;
                rn = nb;
                ep = D.ep;
            }
        }
    }
    const int lane = threadIdx.x & 63;
    const long long t0 = wall_clock64();
    for (;;) {
        // bitwise: all four loads are issued before any compare resolves
        int ok = int(ld_uni(vp) == vwant) & int(ld_uni(vp2) == vwant2) & int(ld_uni(lp1) >= lwant1) &
                 int(ld_uni(lp2) >= lwant2);
        if (!DIST && lp3) ok &= int(ld_uni(lp3) >= lwant1);
        if constexpr (DIST) {
            if (rp) {  // lane l checks flag l (l < rn): one vector load, one ballot
                const bool good = lane >= rn || ld_sys(rp + (lane < rn ? lane : 0)) == ep;
                ok &= int(__builtin_amdgcn_readfirstlane((uint32_t)(__ballot(!good) == 0)));
            }
        }
        if (ok) return true;
        if (ld_uni(a.ctl + C_ERR)) return false;
        if (wall_clock64() - t0 > a.tlimit) {
            if constexpr (DIST) {
                int miss = int(ld_uni(vp) != vwant) | (int(ld_uni(vp2) != vwant2) << 1) | (int(ld_uni(lp1) < lwant1) << 2) |
                           (int(ld_uni(lp2) < lwant2) << 3);
                int seen = ld_uni(vp);
                if (rp) {
                    const bool good = lane >= rn || ld_sys(rp + (lane < rn ? lane : 0)) == ep;
                    const unsigned long long bad = __ballot(!good);
                    if (bad) {
                        miss |= 16 | ((int)__builtin_ctzll(bad) << 8);
                        seen = (int)__builtin_amdgcn_readfirstlane(ld_sys(rp + (int)__builtin_ctzll(bad)));
                    }
                }
                if (lane == 0) dist_note_timeout(a.dist->check_err + DIST_TO_REC, 1, type, i, j, b0 | (nb << 16), miss, seen);
            }
            st_agent(a.ctl + C_ERR, 1);
            return false;
        }
        __builtin_amdgcn_s_sleep(2);
    }
}

// DIAGX(k > 0)'s two products before the diagonal factor, with the result left in the
// factor's LDS image (f64, diag_factor_la):
//   T = A_{k,k-1} Linv_{k-1}^T  on the staging ring (triangular B, MAP 1), stored to HBM as
//       L_{k,k-1} AND into the LDS image as an operand;
//   A_kk - T T^T  with both fragments read from that image (no second HBM round trip, no
//       ring fill), the diagonal tile's lower 16 x 16 tiles only (MAP 2), accumulated onto
//       A_kk itself (loaded while T is stored); the result overwrites the image (lower part).
// Publishes L_{k,k-1} (lcnt[k] = k) after S (the two-call form published between the two).
// (The distributed form pushes L_{k,k-1} to the other ranks after the diagonal factor.)
template <typename T>
__device__ __forceinline__ long long diagx_ts(T* __restrict__ Akm, T* __restrict__ Akk, int64_t ld,
                                              const T* __restrict__ Lp, int* lflag, int k, T* smem, const int t,
                                              bool mark) {
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    const int lane = t & 63, w = t >> 6, lr = lane & 15, lk = lane >> 4;
    int sr, sc;
    wave_block<2>(w, sr, sc);
    // the S accumulators start from A_kk: its loads are in flight during T's mainloop
    // (MAP 2 layout; every element, the upper ones unused)
    acc_t sacc[2][4];
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int reg = 0; reg < 4; reg++) {
            const T* ccol = Akk + (int64_t)(sc * 32 + x * 16 + Tr::orow(lk, reg)) * ld;
#pragma unroll
            for (int y = 0; y < 4; y++) sacc[x][y][reg] = ccol[sr * 64 + y * 16 + lr];
        }
    // ---- T on the ring ---------------------------------------------------------------------
    {
        int tr_, tc_;
        wave_block<1>(w, tr_, tc_);
        acc_t acc[2][4];
        tile_mma<T, 1>(acc, Akm, ld, Lp, DB, GT, 32 * (tc_ + 1), smem, t);
        __syncthreads();  // every wave done with the ring before the image overwrites it
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int reg = 0; reg < 4; reg++) {
                const int jl = tc_ * 32 + x * 16 + Tr::orow(lk, reg);
#pragma unroll
                for (int y = 0; y < 4; y++) {
                    const int il = tr_ * 64 + y * 16 + lr;
                    st_sc1(Akm + il + (int64_t)jl * ld, acc[x][y][reg]);
                    smem[il + jl * SIL] = acc[x][y][reg];
                }
            }
    }
    __syncthreads();  // the image holds T
    const long long tm = mark ? wall_clock64() : 0;  // (GPRX_PT_TRACE: end of the T phase)
    // ---- A_kk - T T^T from the image ----------------------------------------------------------
    // fragments of step kq + 1 are read while the MFMAs of step kq run (as tile_mma)
    T fb[2][2], fa[2][4];
    auto frag = [&](int kq, int r) {
        const int kc = kq * 4 + lk;
#pragma unroll
        for (int x = 0; x < 2; x++) fb[r][x] = smem[(sc * 32 + x * 16 + lr) + kc * SIL];
#pragma unroll
        for (int y = 0; y < 4; y++) fa[r][y] = smem[(sr * 64 + y * 16 + lr) + kc * SIL];
    };
    frag(0, 0);
#pragma unroll 2
    for (int kq = 0; kq < GT / 4; kq++) {
        if (kq + 1 < GT / 4) frag(kq + 1, (kq + 1) & 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 4; y++)
                if (4 * sr + y >= 2 * sc + x) sacc[x][y] = Tr::mma(-fb[kq & 1][x], fa[kq & 1][y], sacc[x][y]);
    }
    // L_{k,k-1} final: unblocks the updates of column k.  Published after S so the HBM stores'
    // latency hides under S; its barrier is also "every read of T done" for the image below.
    publish(lflag, k, false);
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int reg = 0; reg < 4; reg++) {
            const int jl = sc * 32 + x * 16 + Tr::orow(lk, reg);
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const int il = sr * 64 + y * 16 + lr;
                if (4 * sr + y >= 2 * sc + x) smem[il + jl * SIL] = sacc[x][y][reg];
            }
        }
    __syncthreads();
    return tm;
}

// ---- the split diagonal step (f64) ---------------------------------------------------------
// DIAGX(k)'s two products before the factor (T = A_{k,k-1} Linv_{k-1}^T, A_kk - T T^T: 2432
// MFMAs, 31 us on the one CU of the chain) spread over four more workgroups, in two phases
// (tpart_run):
//   1. TPART(k, p), p = 0..3: the 16-column groups p and 7 - p of T = L_{k,k-1}, stored in
//      place.  A part's stores overwrite A columns the other parts read: each part raises
//      "A read" (tflag 1) once its operand is in registers, stores only after all four have,
//      then raises "T stored" (tflag 2);
//   2. once all of T is stored and A_kk is final, part p forms the S = A_kk - T T^T quarter of
//      tile-rows p and 7 - p (T staged in LDS) into pbuf (f64: DIAGX copies the quarters
//      into its LDS image, diagx_split) or in place into A_kk (f32), and raises tflag 3.
// Tickets: TPART(k, np-1) .. (k, 0) in that order (order_tparts; np = tp_parts), after DIAGX(k-1)
// and before DIAGX(k), and no other k's parts between them (test_schedule.py checks this).
// Nothing but DIAGX(k) depends on the parts, so every ticket between them completes; a part
// waits only on its siblings, so at most np - 1 workgroups wait at once and with P >= np one
// is always free to claim the next sibling (split_for: fewer workers keep the whole step
// inside DIAGX).
// (the out-of-line functions read these through a pointer to the copy the kernel keeps in LDS,
// pt_lds_ctx_off: a reference to the kernel's Args put the whole struct in scratch memory, and
// every a.x of every task became a scratch load)
template <typename T>
struct TpCtx {
    int* ctl;
    int* lcnt;
    int* tflag;
    T* pbuf;
    const PtDist<T>* dist;
    long long tlimit;
    long long* xt;  // GPRX_PT_TRACE (one GPU): phase stamps, TPART(k, c) at 4 (4 k + c), DIAGX(k) at 4 (4 nc + k)
    int nc;
    const int* ver;  // tile versions (A_kk final: ver[k][k] = k - 1)
    int nv;
};
// LDS of a TPART: phase 1 the part's 32 Linv rows (column stride LSB: 16-B aligned vectors);
// phase 2 all of T (the 128 columns of L_{k,k-1}, CPI columns per LDS-DMA instruction, groups
// TQ apart), then the 9th tile's eight k-slices in the same area
template <typename T>
struct TpL {
    static constexpr int E = 16 / (int)sizeof(T);                    // elements per 16-B vector
    static constexpr int LSB = sizeof(T) == 8 ? 34 : 36;
    static constexpr int CPI = 64 * 16 / (DB * (int)sizeof(T));      // 1 (f64), 2 (f32)
    static constexpr int TQ = CPI * DB + (sizeof(T) == 8 ? 4 : 8);
    __device__ static int tcol(int c) { return (c / CPI) * TQ + (c % CPI) * DB; }
};
static_assert(DB * TpL<double>::LSB * sizeof(double) <= gemm_lds<double>(), "TPART staging exceeds the LDS of the launch");
static_assert(DB / TpL<double>::CPI * TpL<double>::TQ * sizeof(double) <= gemm_lds<double>(), "TPART staging exceeds the LDS");
static_assert(DB * TpL<float>::LSB * sizeof(float) <= gemm_lds<float>(), "TPART staging exceeds the LDS of the launch");
static_assert(DB / TpL<float>::CPI * TpL<float>::TQ * sizeof(float) <= gemm_lds<float>(), "TPART staging exceeds the LDS");

// wave 0: Linv_kk available to this rank (local publication, or the owner's push)
template <typename T, bool DIST>
__device__ bool tpart_wait_linv(const TpCtx<T>& a, int kk, bool& remote) {
    const unsigned* rp = nullptr;
    unsigned ep = 0;
    remote = false;
    if constexpr (DIST) {
        const PtDist<T>& D = *a.dist;
        if (__builtin_amdgcn_readfirstlane(D.loc[kk]) < 0) {
            rp = dist_flags(D, D.r) + dist_f_linv(D.nr, D.nc) + kk;
            ep = D.ep;
            remote = !__builtin_amdgcn_readfirstlane(D.acq_agent);
        }
    }
    const long long t0 = wall_clock64();
    for (;;) {
        const bool ok = rp ? (__builtin_amdgcn_readfirstlane(ld_sys(rp)) == ep) : (ld_uni(a.lcnt + kk) >= kk + 1);
        if (ok) return true;
        if (ld_uni(a.ctl + C_ERR)) return false;
        if (wall_clock64() - t0 > a.tlimit) {
            st_agent(a.ctl + C_ERR, 1);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// wave 0: *v == want (A_kk final)
template <typename T>
__device__ bool tpart_wait_ver(const TpCtx<T>& a, const int* v, int want) {
    const long long t0 = wall_clock64();
    for (;;) {
        if (ld_uni(v) == want) return true;
        if (ld_uni(a.ctl + C_ERR)) return false;
        if (wall_clock64() - t0 > a.tlimit) {
            st_agent(a.ctl + C_ERR, 1);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// wave 0: lane l < n checks f[l] >= want (one vector load, one ballot per poll)
template <typename T>
__device__ bool tpart_wait_flags(const TpCtx<T>& a, const int* f, int n, int want) {
    const int lane = threadIdx.x & 63;
    const long long t0 = wall_clock64();
    for (;;) {
        const bool good = lane >= n || ld_agent(f + (lane < n ? lane : 0)) >= want;
        if (__builtin_amdgcn_readfirstlane((uint32_t)(__ballot(!good) == 0))) return true;
        if (ld_uni(a.ctl + C_ERR)) return false;
        if (wall_clock64() - t0 > a.tlimit) {
            st_agent(a.ctl + C_ERR, 1);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
}

// TPART(k, p), two phases.
// 1. The 16-column groups p and 7 - p of T = L_{k,k-1} = A_{k,k-1} Linv_{k-1}^T (group g needs
//    K = 16 (g + 1): 36 MFMAs per wave in every part).  Wave w forms rows 16 w .. 16 w + 15: its
//    A fragments (every A element read by one lane of one part) go to registers at task start,
//    before Linv_{k-1} is even waited for; the 32 Linv rows, shared by all waves, through LDS.
//    Stored in place once every part has read its A (tflag 1); then tflag 2.
// 2. Once all of T is stored and A_kk is final: the part's quarter of S = A_kk - T T^T, the 9
//    lower 16 x 16 tiles of tile-rows p and 7 - p (p + 1 and 8 - p of them), from all of T in
//    LDS.  Wave w forms tile w over K = 128 and the 16-deep k-slice w of the 9th tile (36
//    MFMAs each, the slices summed in a fixed order); the tiles go to the shared S buffer;
//    tflag 3.  DIAGX(k) then copies 72 KB, not four 72 KB products (the products' sum had
//    cost it 6 us of loads per step).
// Out of line, one body for every p: inlined into the task loop the parts' code made every
// other task type 2-3x slower (TRSM 16 -> 44 us, even with no TPART in the list) -- the loop's
// registers (it sits at 256 VGPRs) and its hot code in the instruction cache.

// TPART(k, p) phase 1, PROGRESSIVE form (f64 look-ahead factor; on a sharded fit when DIAGX(k-1)
// is this rank's): the part's 32 rows R = 32 p .. 32 p + 31 of T = L_{k,k-1} by blocked forward
// substitution against the factor of block k - 1 AS DIAGX(k-1) PRODUCES IT, following its panel
// counter (TP_DPAN >= c + 1: L panels 0..c and Dinv_0..Dinv_c stored):
//     X_c = V_c Dinv_c^T,   then V_c' -= X_c L_{c'c}^T for c' > c,   V = A_{k,k-1}[R, :] at start
// (T L_{k-1,k-1}^T = A_{k,k-1}, column panel by column panel).  Rows are independent, so the
// parts need nothing from each other in this phase (no "A read" round).  After DIAGX(k-1)'s last
// fact32 only Dinv_3's store, X_3 (8 MFMAs per tile) and the T store remain on the chain: the
// Linv_{k-1} form waited for the whole inverse (its last row block, stores and publication, ~8 us
// of DIAGX(k-1) after F(3)) and then formed all of T.
template <typename T>
__device__ __noinline__ bool tpart_prog(const TpCtx<T>* ap, T* __restrict__ Akm, int64_t ld, const T* __restrict__ Lkk,
                                        const T* __restrict__ Lv, const int* pan, int* tf, int k, const int C, T* smem,
                                        int& s_ok, const int t) {
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    const TpCtx<T> a = *ap;
    const int lane = t & 63, w = t >> 6, lr = lane & 15, lk = lane >> 4;
    // LDS (column-major; strides = 16 mod 32 elements: the ds_read_b64 fragment reads of lanes
    // k and k + 1 land in opposite halves of the 64 banks)
    constexpr int WS = 48, LS = 112, DS = 48;
    T* W = smem;             // [128][WS]: V (32 rows), column panel c becoming X_c
    T* Ls = W + DB * WS;     // [32][LS]: rows 32 (c + 1) .. 127 of L panel c
    T* Ds = Ls + 32 * LS;    // [32][DS]: Dinv_c
    const int r0 = 32 * C;
    long long* xs = a.xt ? a.xt + 4 * (4 * (int64_t)k + C) : nullptr;
    for (int e = t; e < 32 * DB; e += NT) {  // V = A_{k,k-1}[R, :] (final: wait_inputs)
        const int r = e & 31, c = e >> 5;
        W[r + c * WS] = Akm[r0 + r + (int64_t)c * ld];
    }
#pragma unroll 1
    for (int c = 0; c < 4; c++) {
        const int c0 = 32 * c, nl = 96 - c0;
        if (w == 0) {
            const bool ok = tpart_wait_flags<T>(a, pan, 1, c + 1);
            if (ok) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            s_ok = ok ? 1 : 0;
        }
        __syncthreads();
        if (!__builtin_amdgcn_readfirstlane(s_ok)) return false;
        if (c == 3 && xs && w == 0) xs[0] = wall_clock64();  // DIAGX(k-1)'s last panel seen
        for (int e = t; e < 32 * 32; e += NT) {
            const int r = e & 31, q = e >> 5;
            Ds[r + q * DS] = Lv[(c0 + r) + (int64_t)(c0 + q) * DB];
        }
        for (int e = t; e < nl * 32; e += NT) {
            const int r = e % nl, q = e / nl;
            Ls[r + q * LS] = Lkk[(c0 + 32 + r) + (int64_t)(c0 + q) * ld];
        }
        __syncthreads();
        // X_c = V_c Dinv_c^T: waves 0-3, one 16 x 16 tile (ty, tx) each
        acc_t x = acc_t{0};
        const int ty = (w >> 1) & 1, tx = w & 1;
        if (w < 4) {
#pragma unroll
            for (int kq = 0; kq < 8; kq++) {
                const int m = 4 * kq + lk;
                x = Tr::mma(Ds[(16 * tx + lr) + m * DS], W[(16 * ty + lr) + (c0 + m) * WS], x);
            }
        }
        __syncthreads();  // every read of V_c done
        if (w < 4) {
#pragma unroll
            for (int reg = 0; reg < 4; reg++) W[(16 * ty + lr) + (c0 + 16 * tx + Tr::orow(lk, reg)) * WS] = x[reg];
        }
        __syncthreads();
        // V_c' -= X_c L_{c'c}^T, c' > c: 2 x (nl / 16) tiles over the eight waves
#pragma unroll 1
        for (int tt = w; tt < 2 * (nl / 16); tt += NT / 64) {
            const int uy = tt & 1, ux = tt >> 1;  // rows 16 uy, columns c0 + 32 + 16 ux
            acc_t v;
#pragma unroll
            for (int reg = 0; reg < 4; reg++) v[reg] = W[(16 * uy + lr) + (c0 + 32 + 16 * ux + Tr::orow(lk, reg)) * WS];
#pragma unroll
            for (int kq = 0; kq < 8; kq++) {
                const int m = 4 * kq + lk;
                v = Tr::mma(-Ls[(16 * ux + lr) + m * LS], W[(16 * uy + lr) + (c0 + m) * WS], v);
            }
#pragma unroll
            for (int reg = 0; reg < 4; reg++) W[(16 * uy + lr) + (c0 + 32 + 16 * ux + Tr::orow(lk, reg)) * WS] = v[reg];
        }
        // (the next round's first barrier orders these writes before any read)
    }
    __syncthreads();
    if (xs && w == 0) xs[1] = wall_clock64();  // X_3 computed
    for (int e = t; e < 32 * DB; e += NT) {  // T rows R in place: L_{k,k-1}
        const int r = e & 31, c = e >> 5;
        st_sc1(Akm + r0 + r + (int64_t)c * ld, W[r + c * WS]);
    }
    publish(tf + C, 2, false);
    if (xs && w == 0) xs[2] = wall_clock64();
    return true;
}

template <typename T, bool DIST>
__device__ __noinline__ bool tpart_run(const TpCtx<T>* ap, T* __restrict__ Akm, const T* __restrict__ Akk, int64_t ld,
                                       const T* __restrict__ Lp, T* __restrict__ sb, int64_t sld, int* tf, int k,
                                       const int C, T* smem, int& s_ok, const int t, const T* Lkk) {
    typedef TpL<T> Q;
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    typedef typename Tr::vec_t vec_t;
    const TpCtx<T> a = *ap;
    const int lane = t & 63, w = t >> 6, lr = lane & 15, lk = lane >> 4;
    const int g0 = C, g1 = 7 - C;                      // the part's column groups (and tile-rows)
    long long* xs = a.xt ? a.xt + 4 * (4 * (int64_t)k + C) : nullptr;
    if (Lkk) {  // ---- phase 1, progressive --------------------------------------------------------
        if (!tpart_prog<T>(ap, Akm, ld, Lkk, Lp, a.tflag + TP_STRIDE * (k - 1) + TP_DPAN, tf, k, C, smem, s_ok, t))
            return false;
    } else {
    const int nk0 = 4 * (g0 + 1), nk1 = 4 * (g1 + 1);  // k-steps of 4 of each group (nk1 > nk0)
    T* Ls = smem;
    // ---- phase 1 ---------------------------------------------------------------------------
    T af[32];  // A fragments: row 16 w + lr, k = 4 kq + lk, kq < nk1 (<= 32)
    {
        const T* ar = Akm + 16 * w + lr + (int64_t)lk * ld;
#pragma unroll
        for (int kq = 0; kq < 32; kq++)
            if (kq < nk1) af[kq] = ar[(int64_t)(4 * kq) * ld];
    }
    if (w == 0) {
        bool remote = false;
        const bool ok = tpart_wait_linv<T, DIST>(a, k - 1, remote);
        if (ok) {
            if (remote) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        }
        s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(s_ok)) return false;
    if (xs && w == 0) xs[0] = wall_clock64();  // Linv_{k-1} seen
    // Linv_{k-1} rows 16 g0 + r (r < 16) and 16 g1 + r - 16 (r >= 16), all 128 columns (zero
    // above the diagonal), as Ls[r + col LSB]: 16-B loads (4 per thread f64, 2 f32), all in flight
    {
        constexpr int VPC = 32 / Q::E, NV = 32 * DB / Q::E / NT;
        vec_t lv[NV];
#pragma unroll
        for (int u = 0; u < NV; u++) {
            const int e = u * NT + t, r = Q::E * (e % VPC), col = e / VPC;
            const int row = (r < 16) ? 16 * g0 + r : 16 * g1 + r - 16;
            lv[u] = *reinterpret_cast<const vec_t*>(Lp + row + (int64_t)col * DB);
        }
#pragma unroll
        for (int u = 0; u < NV; u++) {
            const int e = u * NT + t;
            *reinterpret_cast<vec_t*>(Ls + Q::E * (e % VPC) + (e / VPC) * Q::LSB) = lv[u];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (w == 0) st_agent(tf + C, 1);  // "A read": this part's A fragments have landed
    // acc[x][reg] = T(16 w + lr, 16 g_x + orow(lk, reg))
    acc_t acc[2] = {acc_t{0}, acc_t{0}};
#pragma unroll
    for (int kq = 0; kq < 32; kq++) {
        if (kq < nk1) {
            const int kc = 4 * kq + lk;
            acc[1] = Tr::mma(Ls[(16 + lr) + kc * Q::LSB], af[kq], acc[1]);
            if (kq < nk0) acc[0] = Tr::mma(Ls[lr + kc * Q::LSB], af[kq], acc[0]);
        }
    }
    if (xs && w == 0) xs[1] = wall_clock64();  // T computed
    // the in-place stores overwrite A columns the other parts read: wait for their "A read"
    // (the four parts hold consecutive tickets and need only a CU each: P >= 4, potrf_tiles)
    if (w == 0) s_ok = tpart_wait_flags<T>(a, tf, 4, 1) ? 1 : 0;
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(s_ok)) return false;
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int reg = 0; reg < 4; reg++)
            st_sc1(Akm + 16 * w + lr + (int64_t)(16 * (x ? g1 : g0) + Tr::orow(lk, reg)) * ld, acc[x][reg]);
    publish(tf + C, 2, false);  // this part's columns of L_{k,k-1} stored
    if (xs && w == 0) xs[2] = wall_clock64();
    }
    // ---- phase 2 ---------------------------------------------------------------------------
    if (w == 0) {
        bool ok = tpart_wait_flags<T>(a, tf, 4, 2);                           // all of T
        if (ok) ok = tpart_wait_ver<T>(a, a.ver + (int64_t)k * a.nv + k, k - 1);  // A_kk final
        if (ok) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(s_ok)) return false;
    // T (column c at smem + tcol(c)) by LDS-DMA, CPI 128-row columns per wave instruction
    {
        constexpr int LPC = 64 / Q::CPI;  // lanes per column
        for (int q = w; q < DB / Q::CPI; q += NT / 64)
            __builtin_amdgcn_global_load_lds(
                (const void*)(Akm + Q::E * (lane % LPC) + (int64_t)(Q::CPI * q + lane / LPC) * ld),
                (__attribute__((address_space(3))) void*)(smem + q * Q::TQ), 16, 0, 0);
    }
    // the quarter's tiles: tau <= p -> (p, tau), else (7 - p, tau - p - 1); wave w: tile w, and
    // the k-slice w of tile 8
    auto tile_of = [&](int tau, int& R, int& Cc) {
        R = (tau <= g0) ? g0 : g1;
        Cc = (tau <= g0) ? tau : tau - g0 - 1;
    };
    int R0, C0, R8, C8;
    tile_of(w, R0, C0);
    tile_of(8, R8, C8);
    acc_t s0;  // A_kk's tile w, loaded while T lands
#pragma unroll
    for (int reg = 0; reg < 4; reg++) s0[reg] = Akk[(16 * R0 + lr) + (int64_t)(16 * C0 + Tr::orow(lk, reg)) * ld];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll 8
    for (int kq = 0; kq < 32; kq++) {
        const int kc = 4 * kq + lk;
        s0 = Tr::mma(-smem[Q::tcol(kc) + 16 * C0 + lr], smem[Q::tcol(kc) + 16 * R0 + lr], s0);
    }
    acc_t s8 = acc_t{0};
#pragma unroll
    for (int kq = 4 * w; kq < 4 * w + 4; kq++) {
        const int kc = 4 * kq + lk;
        s8 = Tr::mma(-smem[Q::tcol(kc) + 16 * C8 + lr], smem[Q::tcol(kc) + 16 * R8 + lr], s8);
    }
#pragma unroll
    for (int reg = 0; reg < 4; reg++)
        st_sc1(sb + (16 * R0 + lr) + (int64_t)(16 * C0 + Tr::orow(lk, reg)) * sld, s0[reg]);
    __syncthreads();  // every wave done reading T: its area takes the 9th tile's k-slices
#pragma unroll
    for (int reg = 0; reg < 4; reg++) smem[w * 256 + lane * 4 + reg] = s8[reg];
    __syncthreads();
    if (t < 256) {  // the 9th tile: A_kk + the eight k-slices, in order
        const int ln = t >> 2, reg = t & 3;
        const int r = 16 * R8 + (ln & 15), c = 16 * C8 + Tr::orow(ln >> 4, reg);
        T v = Akk[r + (int64_t)c * ld];
#pragma unroll
        for (int w8 = 0; w8 < 8; w8++) v += smem[w8 * 256 + t];
        st_sc1(sb + r + (int64_t)c * sld, v);
    }
    if (xs && w == 0) xs[3] = wall_clock64();  // S quarter computed (its stores in flight)
    publish(tf + C, 3, false);
    return true;
}

// TPART(k, p), eight parts (f64, the Linv form): p = C + 4 h, column groups g0 = C, g1 = 7 - C.
// 1. T's rows 64 h .. 64 h + 63 of groups g0, g1: wave w forms the 16 x 16 block of row tile
//    w & 3 and group w >> 2 (per SIMD, waves w and w + 4: one block of each group, 4 (g0 + 1) +
//    4 (g1 + 1) = 36 MFMAs, half the four-part form's), stored in place once the four parts of
//    the same rows have read their A operand (the other half's parts read other rows); tflag 2.
// 2. Once all of T is stored and A_kk is final: tiles 5 h .. of the quarter of tile-rows g0, g1
//    (5 and 4 of its 9), each over all of T as eight 16-column slices, one per wave (20 or 16
//    MFMAs per wave against 36), summed with A_kk through LDS into the S buffer; tflag 3.  (A
//    split of the quarter by T's column halves halved the staging too, but DIAGX then summed two
//    S buffers: its copy went 1.9 -> 3.5 us.)
// Same tickets and waits as the four-part form (order_tparts: TPART(k, 7) .. (k, 0); P >= 8).
template <typename T, bool DIST>
__device__ __noinline__ bool tpart_run8(const TpCtx<T>* ap, T* __restrict__ Akm, const T* __restrict__ Akk, int64_t ld,
                                        const T* __restrict__ Lp, T* __restrict__ sb, int* tf, int k, const int p,
                                        T* smem, int& s_ok, const int t) {
    typedef TpL<T> Q;
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    typedef typename Tr::vec_t vec_t;
    const TpCtx<T> a = *ap;
    const int lane = t & 63, w = t >> 6, lr = lane & 15, lk = lane >> 4;
    const int C = p & 3, h = p >> 2;
    const int g0 = C, g1 = 7 - C;
    long long* xs = (a.xt && h == 0) ? a.xt + 4 * (4 * (int64_t)k + C) : nullptr;  // (trace: the h = 0 parts)
    // ---- phase 1 ---------------------------------------------------------------------------
    {
        const int rt = w & 3, gi = w >> 2, g = gi ? g1 : g0, nk = 4 * (g + 1);  // k-steps of 4 (<= 32)
        const int row0 = 64 * h + 16 * rt;
        T* Ls = smem;
        T af[32];  // A fragments: row row0 + lr, k = 4 kq + lk, kq < nk
        {
            const T* ar = Akm + row0 + lr + (int64_t)lk * ld;
#pragma unroll
            for (int kq = 0; kq < 32; kq++)
                if (kq < nk) af[kq] = ar[(int64_t)(4 * kq) * ld];
        }
        if (w == 0) {
            bool remote = false;
            const bool ok = tpart_wait_linv<T, DIST>(a, k - 1, remote);
            if (ok) {
                if (remote) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
            s_ok = ok ? 1 : 0;
        }
        __syncthreads();
        if (!__builtin_amdgcn_readfirstlane(s_ok)) return false;
        if (xs && w == 0) xs[0] = wall_clock64();  // Linv_{k-1} seen
        // Linv_{k-1} rows 16 g0 + r (r < 16) and 16 g1 + r - 16 (r >= 16), all columns, as
        // Ls[r + col LSB] (the four-part form's staging)
        {
            constexpr int VPC = 32 / Q::E, NV = 32 * DB / Q::E / NT;
            vec_t lv[NV];
#pragma unroll
            for (int u = 0; u < NV; u++) {
                const int e = u * NT + t, r = Q::E * (e % VPC), col = e / VPC;
                const int row = (r < 16) ? 16 * g0 + r : 16 * g1 + r - 16;
                lv[u] = *reinterpret_cast<const vec_t*>(Lp + row + (int64_t)col * DB);
            }
#pragma unroll
            for (int u = 0; u < NV; u++) {
                const int e = u * NT + t;
                *reinterpret_cast<vec_t*>(Ls + Q::E * (e % VPC) + (e / VPC) * Q::LSB) = lv[u];
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (w == 0) st_agent(tf + p, 1);  // "A read"
        acc_t acc = acc_t{0};  // T(row0 + lr, 16 g + orow(lk, reg))
#pragma unroll
        for (int kq = 0; kq < 32; kq++) {
            if (kq < nk) {
                const int kc = 4 * kq + lk;
                acc = Tr::mma(Ls[(16 * gi + lr) + kc * Q::LSB], af[kq], acc);
            }
        }
        if (xs && w == 0) xs[1] = wall_clock64();  // T computed
        if (w == 0) s_ok = tpart_wait_flags<T>(a, tf + 4 * h, 4, 1) ? 1 : 0;  // this half's readers
        __syncthreads();
        if (!__builtin_amdgcn_readfirstlane(s_ok)) return false;
#pragma unroll
        for (int reg = 0; reg < 4; reg++) st_sc1(Akm + row0 + lr + (int64_t)(16 * g + Tr::orow(lk, reg)) * ld, acc[reg]);
        publish(tf + p, 2, false);
        if (xs && w == 0) xs[2] = wall_clock64();
    }
    // ---- phase 2 ---------------------------------------------------------------------------
    if (w == 0) {
        bool ok = tpart_wait_flags<T>(a, tf, 8, 2);                           // all of T
        if (ok) ok = tpart_wait_ver<T>(a, a.ver + (int64_t)k * a.nv + k, k - 1);  // A_kk final
        if (ok) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(s_ok)) return false;
    // all of T (column c at smem + tcol(c)) by LDS-DMA
    {
        constexpr int LPC = 64 / Q::CPI;
        for (int q = w; q < DB / Q::CPI; q += NT / 64)
            __builtin_amdgcn_global_load_lds(
                (const void*)(Akm + Q::E * (lane % LPC) + (int64_t)(Q::CPI * q + lane / LPC) * ld),
                (__attribute__((address_space(3))) void*)(smem + q * Q::TQ), 16, 0, 0);
    }
    // the quarter's tiles tau (tau <= g0: (g0, tau), else (g1, tau - g0 - 1)); this part takes
    // tau = 5 h .. 5 h + nt - 1 (5 and 4 of them), each as eight 16-column slices, slice w on
    // wave w; the slices are summed with A_kk in a fixed order through LDS
    auto tile_of = [&](int tau, int& R, int& Cc) {
        R = (tau <= g0) ? g0 : g1;
        Cc = (tau <= g0) ? tau : tau - g0 - 1;
    };
    const int tau0 = 5 * h, nt = h ? 4 : 5;
    // this thread's output elements (e = t, t + 512, t + 1024 < 256 nt) and their A_kk values,
    // loaded while T lands
    T av[3];
#pragma unroll
    for (int u = 0; u < 3; u++) {
        const int e = t + u * NT;
        av[u] = T(0);
        if (e < 256 * nt) {
            int R, Cc;
            tile_of(tau0 + (e >> 8), R, Cc);
            const int ln = (e & 255) >> 2, reg = e & 3;
            av[u] = Akk[(16 * R + (ln & 15)) + (int64_t)(16 * Cc + Tr::orow(ln >> 4, reg)) * ld];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    acc_t sl[5];
#pragma unroll
    for (int i = 0; i < 5; i++) {
        sl[i] = acc_t{0};
        if (i < nt) {
            int R, Cc;
            tile_of(tau0 + i, R, Cc);
#pragma unroll
            for (int kq = 4 * w; kq < 4 * w + 4; kq++) {
                const int kc = 4 * kq + lk;
                sl[i] = Tr::mma(-smem[Q::tcol(kc) + 16 * Cc + lr], smem[Q::tcol(kc) + 16 * R + lr], sl[i]);
            }
        }
    }
    __syncthreads();  // every wave done reading T: its area takes the slices
#pragma unroll
    for (int i = 0; i < 5; i++)
        if (i < nt)
#pragma unroll
            for (int reg = 0; reg < 4; reg++) smem[(i * 8 + w) * 256 + lane * 4 + reg] = sl[i][reg];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 3; u++) {
        const int e = t + u * NT;
        if (e < 256 * nt) {
            const int i = e >> 8, el = e & 255;
            int R, Cc;
            tile_of(tau0 + i, R, Cc);
            const int ln = el >> 2, reg = el & 3;
            T v = av[u];
#pragma unroll
            for (int w8 = 0; w8 < 8; w8++) v += smem[(i * 8 + w8) * 256 + el];
            st_sc1(sb + (16 * R + (ln & 15)) + (int64_t)(16 * Cc + Tr::orow(ln >> 4, reg)) * DB, v);
        }
    }
    if (xs && w == 0) xs[3] = wall_clock64();  // the part's S tiles computed (their stores in flight)
    publish(tf + p, 3, false);
    return true;
}

// Lkk: L_{k-1,k-1} (ld) when DIAGX(k-1) publishes its panels where these parts can read them
// (one GPU, or DIAGX(k-1) on this rank): the progressive phase 1; null: the Linv_{k-1} form
template <typename T, bool DIST>
__device__ __forceinline__ bool tpart_task(const TpCtx<T>* ap, T* Akm, T* Akk, int64_t ld, const T* Lp, int k, int c,
                                           T* smem, int& s_ok, const int t, const T* Lkk) {
    // S's quarters: f64 into the S buffer (DIAGX copies it into the look-ahead factor's LDS
    // image); f32 in place into A_kk (the rank-8 factor reads its block from memory)
    constexpr bool img = std::is_same<T, double>::value && DIAG_LA;
    if constexpr (img && tp_parts(true) == 8)
        return tpart_run8<T, DIST>(ap, Akm, Akk, ld, Lp, ap->pbuf, ap->tflag + TP_STRIDE * k, k, c, smem, s_ok, t);
    else
        return tpart_run<T, DIST>(ap, Akm, Akk, ld, Lp, img ? ap->pbuf : Akk, img ? (int64_t)DB : ld,
                                  ap->tflag + TP_STRIDE * k, k, c, smem, s_ok, t, img ? Lkk : nullptr);
}

// DIAGX(k > 0) of the split step, f32 (the parts wrote S into A_kk): wait for the four
// quarters, then L_{k,k-1} is final (lcnt[k] = k)
template <typename T>
__device__ __forceinline__ bool diagx_split_wait(const TpCtx<T>* ap, int k, int& s_ok) {
    const int w = threadIdx.x >> 6;
    if (w == 0) {
        const bool ok = tpart_wait_flags<T>(*ap, ap->tflag + TP_STRIDE * k, 4, 3);
        if (ok) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            st_agent(ap->lcnt + k, k);
        }
        s_ok = ok ? 1 : 0;
    }
    __syncthreads();
    return __builtin_amdgcn_readfirstlane(s_ok) != 0;
}

// DIAGX(k > 0) of the split step: S (the 36 lower 16 x 16 tiles, assembled in the shared S
// buffer by the parts) into the factor's LDS image, then L_{k,k-1} is final (lcnt[k] =
// k).  Each wave waits for the parts itself and copies 576 element pairs, 9 per lane
// (lower tile tau = q / 128, pair q % 8 of its column (q % 128) / 8), one batch of loads.
template <typename T>
__device__ __noinline__ bool diagx_split(const TpCtx<T>* ap, int k, T* smem, int& s_ok, const int t) {
    typedef typename Mfma<T>::vec_t vec_t;
    const TpCtx<T> a = *ap;
    const int lane = t & 63, w = t >> 6;
    const int* tf = a.tflag + TP_STRIDE * k;
    long long* xs = a.xt ? a.xt + 4 * (4 * (int64_t)a.nc + k) : nullptr;
    int rr[9], cc[9];
#pragma unroll
    for (int u = 0; u < 9; u++) {
        const int q = 576 * w + 64 * u + lane, tau = q >> 7, e = q & 127;
        int R = 0;  // lower tile tau = R (R + 1) / 2 + C
        while ((R + 1) * (R + 2) / 2 <= tau) R++;
        const int C = tau - R * (R + 1) / 2;
        rr[u] = 16 * R + 2 * (e & 7);
        cc[u] = 16 * C + (e >> 3);
    }
    constexpr int NP = tp_parts(std::is_same<T, double>::value);
    const bool ok = tpart_wait_flags<T>(a, tf, NP, 3);  // this wave polls the parts itself
    if (ok) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (xs && w == 0) xs[2] = wall_clock64();  // every quarter seen
        vec_t v[9];
#pragma unroll
        for (int u = 0; u < 9; u++) v[u] = *reinterpret_cast<const vec_t*>(a.pbuf + rr[u] + cc[u] * DB);
#pragma unroll
        for (int u = 0; u < 9; u++) {
            smem[rr[u] + cc[u] * SIL] = v[u][0];
            smem[rr[u] + 1 + cc[u] * SIL] = v[u][1];
        }
    }
    if (w == 0) s_ok = ok ? 1 : 0;
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(s_ok)) return false;
    // every column block of L_{k,k-1} is stored (each part's flag came after its stores)
    if (w == 0) st_agent(a.lcnt + k, k);
    if (xs && w == 0) xs[3] = wall_clock64();  // S in the image
    return true;
}

template <typename T>
__device__ __forceinline__ TpCtx<T> tp_ctx(const Args<T>& a) {
    return TpCtx<T>{a.ctl, a.lcnt, a.tflag, a.pbuf, a.dist, a.tlimit, a.xt, a.nc, a.ver, a.nv};
}
// the split step's context lives in LDS after the ticket words (written once per launch):
// the out-of-line calls take one pointer (by value, its ten fields cost the task loop spills)
template <typename T>
constexpr size_t pt_lds_ctx_off() {
    return pt_lds_bytes<T>() + 16;
}
template <typename T>
constexpr size_t pt_lds_total() {
    return pt_lds_ctx_off<T>() + sizeof(TpCtx<T>);
}

template <typename T, bool DIST>
__global__ __launch_bounds__(NT) void potrf_tiles_kernel(Args<T> a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    // ONE __shared__ array (a second __shared__ object can make hipcc drain the LDS-DMA
    // pipeline with vmcnt(0)); the ticket word sits after the largest per-task image
    int& s_q = *reinterpret_cast<int*>(smem_raw + pt_lds_bytes<T>());
    int& s_ok = *reinterpret_cast<int*>(smem_raw + pt_lds_bytes<T>() + sizeof(int));
    TpCtx<T>* tpc = reinterpret_cast<TpCtx<T>*>(smem_raw + pt_lds_ctx_off<T>());
    if (threadIdx.x == 0) *tpc = tp_ctx(a);  // (visible after the task loop's first barrier)
    T* smem = reinterpret_cast<T*>(smem_raw);
    const int t = threadIdx.x;
    const int wv = wave_id();
    const int64_t ld = a.ld;
    for (;;) {
        if (wv == 0) {  // one ticket per workgroup: lane 0 adds 1, the other lanes 0
            // (not taken ahead of time: a ticket claimed while the previous task still runs
            // delays critical-path tasks behind long updates -- measured 28.8 -> 33.2 ms)
            const int v = __hip_atomic_fetch_add(a.ctl + C_TICKET, (t == 0) ? 1 : 0, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
            s_q = __builtin_amdgcn_readfirstlane(v);
        }
        __syncthreads();
        // everything below is wave-uniform: keep it in SGPRs so the task dispatch is scalar
        const int q = __builtin_amdgcn_readfirstlane(s_q);
        if (q >= a.ntasks) break;
        const long long tr0 = a.trace ? wall_clock64() : 0;
        const int4 tk = a.tasks[q];
        const int type = __builtin_amdgcn_readfirstlane(tk.x & 0xff), nb = __builtin_amdgcn_readfirstlane(tk.x >> 8);
        const int i = __builtin_amdgcn_readfirstlane(tk.y), j = __builtin_amdgcn_readfirstlane(tk.z),
                  b0 = __builtin_amdgcn_readfirstlane(tk.w);
        dbg_mark(a.dbg, q, 1 + 10 * type, i, j);
        // wave 0 alone polls the task's counters (the other waves sleep in the barrier: eight
        // times fewer loads on the counters -- hundreds of workgroups polling the transport's
        // uncached words measured 10x slower distributed fits), then acquires for the
        // workgroup (invalidates this CU's L1).  All of wave 0's lanes store the same word.
        if (wv == 0) {
            const bool ok0 = wait_inputs<T, DIST>(a, type, i, j, b0, nb);
            if (ok0 && !(a.variant & 32)) {
                bool remote = false;  // DIST: an input pushed by another rank (system-scope acquire)
                if constexpr (DIST) {
                    const PtDist<T>& D = *a.dist;
                    const int dep = (type == T_DIAGX) ? i - 1 : ((type == T_BUILD || type == T_TPART) ? -1 : j);
                    remote = dep >= 0 && __builtin_amdgcn_readfirstlane(D.loc[dep]) < 0 &&
                             !__builtin_amdgcn_readfirstlane(D.acq_agent);
                }
                if (remote) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            s_ok = ok0 ? 1 : 0;
        }
        __syncthreads();
        if (!__builtin_amdgcn_readfirstlane(s_ok)) break;
        const long long tr1 = a.trace ? wall_clock64() : 0;
        const long long tc1 = a.trace ? (long long)__builtin_amdgcn_s_memtime() : 0;
        dbg_mark(a.dbg, q, 2 + 10 * type, i, j);
        // opaque copy of the thread index: keeps the per-task address arithmetic inside the
        // task instead of hoisted (and held in registers) across the whole task loop
        int tid = t;
        asm volatile("" : "+v"(tid));
        if constexpr (DIST) {
            // ---- one rank of the distributed factorisation: packed own rows (ld DB), remote
            // rows from the window, final tiles pushed to their consumers' mailboxes ----------
            const PtDist<T>& D = *a.dist;
            bool ok = true;
            if (type == T_TPART) {
                if constexpr (SPLIT_CODE)
                    ok = tpart_task<T, true>(tpc, dist_tile(a.A, D, i, i - 1), dist_tile(a.A, D, i, i), DB,
                                             a.Linv + (int64_t)(i - 1) * DB * DB, i, j, smem, s_ok, tid,
                                             __builtin_amdgcn_readfirstlane(D.loc[i - 1]) >= 0 && !tp_linv_form()
                                                 ? dist_tile(a.A, D, i - 1, i - 1) : nullptr);
            } else if (type == T_BUILD) {
                T* tij = dist_tile(a.A, D, i, j);
                // build_tile_sum addresses element (gi, gj) at base + gi + gj ld (global indices)
                const TileBuild<T>& b = *a.tb;
                const bool bad = pr::build_tile_sum<T, 1, true>(
                    b.Kd, b.FU, b.FV, b.nf, b.Kr, b.Kp, b.hd, tij - (int64_t)i * GT - (int64_t)j * GT * DB, DB, b.n,
                    b.sigma2, (int64_t)i * GT, (int64_t)j * GT, smem, tid);
                if (__builtin_amdgcn_readfirstlane(__any(bad))) atomicOr(a.tb->flag, 1);
                publish(a.ver + (int64_t)i * a.nv + j, 0, false);
            } else if (type == T_UPD) {
                // row j of this rank: its stored tiles; of another rank: the window, one tile per
                // panel (one call site: two inlined mainloops crashed hipcc 7.2)
                const int lj = __builtin_amdgcn_readfirstlane(D.loc[j]);
                const bool loc = lj >= 0;
                const T* Bop = loc ? dist_tile(a.A, D, j, b0) : nullptr;
                const uint64_t* bp = loc ? nullptr : D.tptr + (int64_t)j * D.nc + b0;
                if (D.check && !loc && wv == 0) dist_check_tags(D, j, b0, nb, 0);
                tile_gemm<T, true>(dist_tile(a.A, D, i, j), DB, dist_tile(a.A, D, i, b0), DB, Bop, DB, nb * GT, i == j,
                                   smem, tid, false, bp);
                publish(a.ver + (int64_t)i * a.nv + dist_col(D.nc, j), b0 + nb, false);
                if (D.check && !loc && wv == 0) dist_check_tags(D, j, b0, nb, 1);
                if (!loc && wv == 0) dist_release(D, b0, nb);  // this chunk's window reads are done
            } else if (type == T_TRSM) {
                T* Cik = dist_tile(a.A, D, i, j);
                tile_trsm<T>(Cik, DB, Cik, DB, a.Linv + (int64_t)j * DB * DB, DB, smem, tid);
                publish(a.lcnt + i, j + 1, false);
                if (i == D.nc) {  // the label rows z^T: every other rank's z area (the solves read it)
                    const unsigned all = ((1u << D.g) - 1u) & ~(1u << D.r);
                    dist_push(Cik, D, all, D.o_z + (int64_t)j * DB * DB * (int64_t)sizeof(T),
                              dist_f_tile() + (int64_t)i * D.nc + j, tid);
                } else {
                    const unsigned cm = dist_consumers(D, i);
                    if (wv == 0) ok = dist_wait_release(a, D, cm, j - D.ww);
                    if (wv == 0) s_ok = ok ? 1 : 0;
                    __syncthreads();
                    ok = __builtin_amdgcn_readfirstlane(s_ok) != 0;
                    if (ok)
                        dist_push(Cik, D, cm, -1, dist_f_tile() + (int64_t)i * D.nc + j, tid,
                                  (int64_t)(j % D.ww) * D.nr + i, (D.ep << 16) | (unsigned)(j + 1));
                }
            } else {  // DIAGX(k = i)
                const int k = i;
                T* Akk = dist_tile(a.A, D, k, k);
                T* Akm = k > 0 ? dist_tile(a.A, D, k, k - 1) : nullptr;
                constexpr bool fused_ts = std::is_same<T, double>::value && DIAG_LA;
                if (SPLIT_CODE && k > 0 && a.split) {
                    if constexpr (fused_ts) ok = diagx_split<T>(tpc, k, smem, s_ok, tid);
                    else ok = diagx_split_wait<T>(tpc, k, s_ok);
                    if (!ok) break;
                } else if (fused_ts && k > 0) {
                    diagx_ts<T>(Akm, Akk, DB, a.Linv + (int64_t)(k - 1) * DB * DB, a.lcnt + k, k, smem, tid, false);
                } else if (k > 0) {
                    tile_trsm<T>(Akm, DB, Akm, DB, a.Linv + (int64_t)(k - 1) * DB * DB, DB, smem, tid);
                    publish(a.lcnt + k, k, false);
                    tile_gemm<T, true, 2, GPRX_SHORT_FEED>(Akk, DB, Akm, DB, Akm, DB, GT, true, smem, tid);
                    local_sync();
                }
                diag_factor<T>(Akk, DB, a.Linv + (int64_t)k * DB * DB, a.info, (int64_t)k * DB, smem_raw, tid, a.dbg,
                               nullptr, fused_ts && k > 0, a.lcnt + k, k + 1,  // (publishes Linv_k locally)
                               (a.split && !tp_linv_form()) ? a.tflag + TP_STRIDE * k + TP_DPAN : nullptr);  // (its panels)
                // pushes after the local publication (this rank's chain goes on meanwhile): the
                // next diagonal step's rank first, L_{k,k-1} before Linv_k
                const unsigned cm = k > 0 ? dist_consumers(D, k) : 0u;
                const unsigned all = ((1u << D.g) - 1u) & ~(1u << D.r);
                const int nx = (k + 1 < D.nc) ? __builtin_amdgcn_readfirstlane(D.own[k + 1]) : D.r;
                const unsigned first = (nx != D.r) ? (1u << nx) : 0u;
                if (k > 0) {
                    if (wv == 0) ok = dist_wait_release(a, D, cm, k - 1 - D.ww);
                    if (wv == 0) s_ok = ok ? 1 : 0;
                    __syncthreads();
                    ok = __builtin_amdgcn_readfirstlane(s_ok) != 0;
                }
                const int64_t owin = -1;  // the window slot tix
                const int64_t olinv = D.o_linv + (int64_t)k * DB * DB * (int64_t)sizeof(T);
                const int64_t tix = (int64_t)((k - 1 + D.ww) % D.ww) * D.nr + k;
                const unsigned tgv = (D.ep << 16) | (unsigned)k;
                if (ok && k > 0)
                    dist_push(Akm, D, cm & first, owin, dist_f_tile() + (int64_t)k * D.nc + (k - 1), tid, tix, tgv);
                if (ok) dist_push(a.Linv + (int64_t)k * DB * DB, D, all & first, olinv, dist_f_linv(D.nr, D.nc) + k, tid);
                if (ok && k > 0)
                    dist_push(Akm, D, cm & ~first, owin, dist_f_tile() + (int64_t)k * D.nc + (k - 1), tid, tix, tgv);
                if (ok) dist_push(a.Linv + (int64_t)k * DB * DB, D, all & ~first, olinv, dist_f_linv(D.nr, D.nc) + k, tid);
            }
            if (!ok) break;
        } else {
        T* Ci = a.A + (int64_t)i * GT;  // row block i, column 0
        constexpr bool fused_ts = std::is_same<T, double>::value && DIAG_LA;
        // (a failed wait inside a task has raised C_ERR: the task ends on garbage, which the
        // launch reports as info = -1, and the next wait_inputs drains the workgroup)
        if (type == T_TPART) {
            if constexpr (SPLIT_CODE)
                (void)tpart_task<T, false>(tpc, Ci + (int64_t)(i - 1) * GT * ld, Ci + (int64_t)i * GT * ld, ld,
                                           a.Linv + (int64_t)(i - 1) * DB * DB, i, j, smem, s_ok, tid,
                                           tp_linv_form() ? nullptr
                                                          : a.A + (int64_t)(i - 1) * GT + (int64_t)(i - 1) * GT * ld);
        } else if (type == T_BUILD) {
            // ver[i][j] goes from -1 (not built) to 0; the tile's values go out write-through
            // one instantiation for every mode: an absent statistic has a zero-depth product
            // (its accumulators stay 0) and no leaves of its class
            // (inline: out of line, its register saves cost the C3 fit 0.35 ms and the sharded
            // fit 1%, more than the task loop's few spills at task level, none in a mainloop)
            const TileBuild<T>& b = *a.tb;
            const bool bad = pr::build_tile_sum<T, 1, true>(b.Kd, b.FU, b.FV, b.nf, b.Kr, b.Kp, b.hd, a.A, ld, b.n,
                                                            b.sigma2, (int64_t)i * GT, (int64_t)j * GT, smem, tid);
            if (__builtin_amdgcn_readfirstlane(__any(bad))) atomicOr(a.tb->flag, 1);  // wave-uniform branch
            publish(a.ver + (int64_t)i * a.nv + j, 0, false);
        } else if (type == T_UPD) {
            // variant 64 (timing experiment, wrong results): every update streams the same
            // L2-resident operands, to separate memory-feed from MFMA limits
            const int64_t oa = (a.variant & 64) ? 0 : (int64_t)i * GT + (int64_t)b0 * GT * ld;
            const int64_t ob = (a.variant & 64) ? GT : (int64_t)j * GT + (int64_t)b0 * GT * ld;
            // variant 128 (timing experiment, wrong results): operand stride 0 along k, every
            // k-slice of the update re-reads the same 1 KB column -- a truly cache-resident feed
            const int64_t lop = (a.variant & 128) ? 0 : ld;
            if (!(a.variant & 2))
                tile_gemm<T, true>(Ci + (int64_t)j * GT * ld, ld, a.A + oa, lop, a.A + ob, lop, nb * GT, i == j, smem,
                                   tid);
            publish(a.ver + (int64_t)i * a.nv + j, b0 + nb, false);
        } else if (type == T_UPD2) {  // tiles (i, j) and (i + 1, j): one 256 x 128 update
            if (!(a.variant & 2))
                tile_gemm_tall<T>(Ci + (int64_t)j * GT * ld, ld, a.A + (int64_t)i * GT + (int64_t)b0 * GT * ld, ld,
                                  a.A + (int64_t)j * GT + (int64_t)b0 * GT * ld, ld, nb * GT, smem, tid);
            publish2(a.ver + (int64_t)i * a.nv + j, a.ver + (int64_t)(i + 1) * a.nv + j, b0 + nb);
        } else if (type == T_TRSM) {
            T* Cik = Ci + (int64_t)j * GT * ld;
            if (!(a.variant & 1))
                tile_trsm<T>(Cik, ld, Cik, ld, a.Linv + (int64_t)j * DB * DB, DB, smem, tid);
            publish(a.lcnt + i, j + 1, false);
        } else {  // DIAGX(k = i)
            const int k = i;
            T* Akk = Ci + (int64_t)k * GT * ld;
            long long dt[4] = {0, 0, 0, 0};
            if (SPLIT_CODE && k > 0 && a.split) {
                if constexpr (fused_ts) (void)diagx_split<T>(tpc, k, smem, s_ok, tid);
                else (void)diagx_split_wait<T>(tpc, k, s_ok);
                if (a.trace) dt[0] = dt[1] = wall_clock64();
            } else if (fused_ts && k > 0) {
                T* Akm = Ci + (int64_t)(k - 1) * GT * ld;
                dt[0] = diagx_ts<T>(Akm, Akk, ld, a.Linv + (int64_t)(k - 1) * DB * DB, a.lcnt + k, k, smem, tid,
                                    a.trace != nullptr);
                dt[1] = dt[0];
            } else if (k > 0) {
                T* Akm = Ci + (int64_t)(k - 1) * GT * ld;
                tile_trsm<T>(Akm, ld, Akm, ld, a.Linv + (int64_t)(k - 1) * DB * DB, DB, smem, tid);
                if (a.trace) dt[0] = wall_clock64();
                publish(a.lcnt + k, k, false);  // L_{k,k-1} final: unblocks the updates of column k
                if (a.trace) dt[1] = wall_clock64();
                tile_gemm<T, true, 2, GPRX_SHORT_FEED>(Akk, ld, Akm, ld, Akm, ld, GT, true, smem, tid);
                local_sync();
            }
            if (a.trace) dt[2] = wall_clock64();
            diag_factor<T>(Akk, ld, a.Linv + (int64_t)k * DB * DB, a.info, (int64_t)k * DB, smem_raw, tid, a.dbg,
                           a.trace ? a.trace + 4 * (int64_t)(a.ntasks + a.nc) + 4 * (int64_t)k : nullptr,
                           fused_ts && k > 0, a.lcnt + k, k + 1,  // (publishes Linv_k: lcnt[k] = k + 1)
                           (a.split && !tp_linv_form()) ? a.tflag + TP_STRIDE * k + TP_DPAN : nullptr);  // (its panels)
            if (a.trace) dt[3] = wall_clock64();
            if (a.trace && wv == 0) {
                long long* dp = a.trace + 4 * (int64_t)a.ntasks + 4 * (int64_t)k;
                for (int u = 0; u < 4; u++) dp[u] = dt[u];
            }
        }
        }
        if (a.trace && wv == 0) {
            long long* tp = a.trace + 4 * (int64_t)q;
            tp[0] = tr0;
            tp[1] = tr1;
            tp[2] = wall_clock64();
            tp[3] = (long long)blockIdx.x | (((long long)__builtin_amdgcn_s_memtime() - tc1) << 16);
        }
    }
    dbg_mark(a.dbg, -1, 9, 0, 0);
    // the error flag of a timed-out wait ends up in info (reported by the caller)
    if (wv == 0 && ld_agent(a.ctl + C_ERR)) atomicMin(a.info, -1);
}

// ==========================================================================================
// Host: task list + list-schedule simulation
// ==========================================================================================
struct Cost {  // per-task durations (us, one CU), calibrated from GPRX_PT_TRACE timelines
    double k128 = 17.1;  // per 128-deep slice of a full tile update
    double ovh = 6.5;    // per update task: ticket, waits, fences, C read-modify-write
    double trsm = 16.0;  // TRSM tile (r01i trace: 15.9)
    double diagx = 70.0;   // DIAGX(k > 0): trsm + syrk tile + 128x128 factor/inverse (r02f trace, f64)
    double diag0 = 40.0;   // DIAGX(0): factor/inverse only
    double early = 31.0;   // DIAGX(k) publishes L_{k,k-1} after its trsm and syrk phases
    double diagf = 0.97;   // diagonal-tile update relative to a full one (2 of 8 waves idle)
    double build = 28.0;   // BUILD tile (pair statistics + kernel values + stores)
    // the split diagonal step (f64): TPART(k, c) takes tpart + tpart_c (c + 1); DIAGX(k) then
    // sums the products and factors (diagx_s), publishing L_{k,k-1} early_s into it
    // (r03w trace, N = 4096: the parts publish S ~12 us after Linv_{k-1}, DIAGX copies it in
    // 2 us and factors; step 54.4 us)
    double tpart = 11.5, tpart_c = 0.0;
    double diagx_s = 44.0, early_s = 2.0;
    // the progressive parts (f64, tpart_prog; DIAGX(k-1) on the same rank): they follow DIAGX(k-1)'s
    // panels and publish S this long after its end (X_3, T and S remain after its last fact32,
    // ~8 us before its end)
    double tpart_prog = 2.5;
    bool prog = false;  // this schedule is for the progressive form (set by the callers)
    int np = 4;         // TPART tasks per split step (tp_parts; set by the callers)
    // a paired update (T_UPD2) per panel, relative to two single-tile panels (the 256 x 128
    // mainloop's probe rate against the 128 x 128 tile's: 0.877 / 0.901)
    double tall = 0.975;
    // which chunks pair (make_schedule pair > 0): at least pair_nbmin panels wide, in the columns
    // before the last pair_tail (GPRX_PT_PAIR_NBMIN / GPRX_PT_PAIR_TAIL)
    int pair_nbmin = 1, pair_tail = 0;
};

// TPART tickets of one k in the order TPART(k, np-1), .., (k, 0): each part waits for
// the reads of the parts with a larger c, so those must hold the earlier tickets (the parts
// have the same inputs and one consumer, DIAGX(k): permuting them over their slots keeps
// every other order of the list)
static void order_tparts(std::vector<int4>& list) {
    std::map<int, std::vector<int>> pos;
    for (size_t q = 0; q < list.size(); q++)
        if ((list[q].x & 0xff) == T_TPART) pos[list[q].y].push_back((int)q);
    for (auto& kv : pos) {
        std::vector<int>& v = kv.second;
        std::sort(v.begin(), v.end());
        for (size_t u = 0; u < v.size(); u++) list[v[u]].z = (int)v.size() - 1 - (int)u;
    }
}

struct Task {
    int type, i, j, b0, nb;
    double dur;
    std::vector<int> succ, esucc;  // esucc: released at the early publication (DIAGX)
    int ndep = 0;
    double bl = 0;  // bottom level (longest path to the end, inclusive)
};

struct Schedule {
    std::vector<int4> list;
    double est_us = 0;
    int64_t ntasks = 0;
    // identity rows paired (make_schedule): an odd identity row block 2s + 1 starts its updates at
    // panel 2s with its partner -- its counters start there and its tile at column 2s is zeroed
    bool ident_even = false;
};

// Chunks of the updates of tile (i, j): b in [0, e), e = j (i > j) or j - 1 (diagonal tile:
// the last one is applied inside DIAGX(j)).  Aligned W-chunks up to the last multiple of W
// at or before column j, then the remainder before the last `near` panels in power-of-two
// pieces (W/2, W/4, ..., 1), then single panels -- few tasks (each costs a fixed ~6 us of
// ticket, waits, fences and C read-modify-write), while the last panels of a tile, the ones
// the diagonal chain waits for, still go one at a time.
// s > 0 (an identity row block of the inverse, whose panels before s are zero): the same
// rule on the panels [s, e), shifted.
// ratio > 0 (chosen per shape by the simulated makespan, potrf_tiles): greedy from the first
// panel, the widest power-of-two piece p <= W (W-aligned when p == W) that ends at least `near`
// panels before e and is at most ratio x the panels left after it.  A piece can start only
// when its last panel is final, so a wide piece close to the tile's last panel holds up the
// tile's consumer: at N = 4096 the [0, 16) piece of tiles (18, 17) and (18, 18) became ready
// with panel 15 and ran 280 us, and DIAGX(18) waited 184 us for it (r03 trace).
static void tile_chunks(int i, int j, int W, int near, std::vector<std::pair<int, int>>& out, int s = 0,
                        int ratio = 0) {
    out.clear();
    const int e = ((i == j) ? j - 1 : j) - s;
    if (e <= 0) return;
    if (ratio > 0) {
        for (int b = 0; b < e;) {
            int p = W;
            for (; p > 1; p /= 2) {
                if (p == W && b % W) continue;
                const int end = b + p;
                if (end > e - near || p > ratio * (e - end)) continue;
                break;
            }
            out.push_back({s + b, p});
            b += p;
        }
        return;
    }
    int hb = std::max(0, std::min(W * ((j - s) / W), e));
    hb -= hb % W;
    int b = 0;
    for (; b + W <= hb; b += W) out.push_back({s + b, W});
    for (int p = W / 2; p >= 1; p /= 2)
        if (b + p <= e - near) {
            out.push_back({s + b, p});
            b += p;
        }
    for (; b < e; b++) out.push_back({s + b, 1});
}

// ni > 0: the last ni row blocks are the identity (the inverse L^{-1} riding along as
// L^{-T} rows): identity block a = i - (nr - ni) has zero L blocks before column block a.
// tail > 0: the capped rule (ratio) only for the tiles of the last `tail` column blocks, the
// fixed rule before them
// pair > 0 (round 6): the off-diagonal tiles of column j from row j + pair down to the last label
// row go in vertical pairs (j + pair, j + pair + 1), ..., each pair's identical chunks as ONE
// T_UPD2 task (a 256 x 128 update: tile_gemm_tall); the `pair` - 1 tiles right below the
// diagonal -- the diagonal chain's inputs -- and the identity rows stay single
static Schedule make_schedule(int nc, int nr, int W, int near, int P, const Cost& cm0, bool build, int ni = 0,
                              int ratio = 0, bool split = false, int tail = 0, int pair = 0) {
    Cost cm = cm0;
    if (split) cm.early = cm.early_s;
    const int nr0 = nr - ni;
    auto start_of = [&](int i) { return i >= nr0 ? i - nr0 : 0; };
    // identity rows in pairs (E_2s, E_2s+1): both update from panel 2s -- the bottom row's block at
    // column 2s is a stored zero (potrf_tiles zeroes it and starts its counters at 2s), so its
    // one extra panel subtracts nothing and the two rows' chunk lists are identical
    static const bool id_pair = [] {
        const char* e = std::getenv("GPRX_PT_IDPAIR");  // 0: identity rows single (A/B)
        return !(e && std::atoi(e) == 0);
    }();
    const bool ident_even = id_pair && pair > 0 && ni > 1;
    // identity pairs in the last pair_tail columns too (the tail rule spares the factor's
    // chain-bound last columns; the identity rows' updates there are bulk work): LML N = 8192
    // 73.66 -> 73.05 ms with both (profiles/r06z_idpair_ab.txt); GPRX_PT_IDTAIL=0 restricts them
    static const bool id_tail = [] {
        const char* e = std::getenv("GPRX_PT_IDTAIL");
        return !(e && std::atoi(e) == 0);
    }();
    auto cstart = [&](int i) {
        const int a = start_of(i);
        return (ident_even && i >= nr0) ? a - (a & 1) : a;
    };
    // row i of column j: 1 the top of a pair, 2 its bottom, 0 single
    auto pair_role = [&](int i, int j) {
        if (pair <= 0) return 0;
        if (i >= nr0) {  // identity rows: (E_2s, E_2s+1)
            const int a = i - nr0;
            if (!ident_even) return 0;
            if ((a & 1) == 0) return a + 1 < ni ? 1 : 0;
            return 2;
        }
        const int r0 = j + pair;
        if (i >= r0 && (i - r0) % 2 == 0 && i + 1 < nr0) return 1;
        if (i - 1 >= r0 && (i - 1 - r0) % 2 == 0) return 2;
        return 0;
    };
    std::vector<Task> tasks;
    tasks.reserve((size_t)nr * nc * 2);
    auto add = [&](int type, int i, int j, int b0, int nb, double dur) {
        Task tk;
        tk.type = type;
        tk.i = i;
        tk.j = j;
        tk.b0 = b0;
        tk.nb = nb;
        tk.dur = dur;
        tasks.push_back(std::move(tk));
        return (int)tasks.size() - 1;
    };
    std::vector<int> diagx(nc, -1);
    std::vector<int> trsm((size_t)nr * nc, -1);
    std::vector<int> last_upd((size_t)nr * nc, -1);
    std::vector<std::vector<int>> deps, edeps;  // edeps: on L_{k,k-1}, published early by DIAGX(k)
    auto dep = [&](int tsk, int on, bool early = false) {
        if (on < 0) return;
        auto& d = early ? edeps : deps;
        if ((int)d.size() <= tsk) d.resize(tsk + 1);
        d[tsk].push_back(on);
    };
    // producer of L_{i,b} (early: the trsm phase of DIAGX(i) already published it)
    auto prodL = [&](int i, int b, bool& early) -> int {
        early = i < nc && b == i - 1;
        if (i < nc && (b == i || b == i - 1)) return diagx[i];
        return trsm[(size_t)i * nc + b];
    };
    // update chunks bucketed by their last block
    struct Chunk {
        int i, j, b0, nb;
    };
    std::vector<std::vector<Chunk>> by_last(nc);
    {
        std::vector<std::pair<int, int>> ch;
        for (int j = 1; j < nc; j++)
            for (int i = j; i < nr; i++) {
                tile_chunks(i, j, W, near, ch, cstart(i), (tail <= 0 || j >= nc - tail) ? ratio : 0);
                for (auto& c : ch) by_last[c.first + c.second - 1].push_back(Chunk{i, j, c.first, c.second});
            }
    }
    auto make_diagx = [&](int k) {
        if (split && k >= 1) {  // TPART(k, np-1..0), then DIAGX(k) on their products
            int tp[8];
            for (int c = cm.np - 1; c >= 0; c--) {
                tp[c] = add(T_TPART, k, c, 0, 0, cm.prog ? cm.tpart_prog : cm.tpart + cm.tpart_c * (c + 1));
                dep(tp[c], diagx[k - 1]);
                dep(tp[c], last_upd[(size_t)k * nc + (k - 1)]);
                dep(tp[c], last_upd[(size_t)k * nc + k]);  // phase 2 starts from A_kk
            }
            const int id = add(T_DIAGX, k, k, 0, 0, cm.diagx_s);
            diagx[k] = id;
            for (int c = 0; c < cm.np; c++) dep(id, tp[c]);
            dep(id, last_upd[(size_t)k * nc + k]);
            return;
        }
        const double dur = (k == 0) ? cm.diag0 : cm.diagx;
        const int id = add(T_DIAGX, k, k, 0, 0, dur);
        diagx[k] = id;
        if (k >= 1) {
            dep(id, diagx[k - 1]);
            dep(id, last_upd[(size_t)k * nc + (k - 1)]);
            dep(id, last_upd[(size_t)k * nc + k]);
        }
    };
    // Creation order (checked below) puts every producer before its consumers:
    // [BUILD(i, j) for the lower tiles], DIAGX(0); per k: TRSM(., k), DIAGX(k+1), the update
    // chunks ending at block k.  A tile's BUILD is its first "update".
    if (build)
        for (int i = 0; i < nc; i++)
            for (int j = 0; j <= i; j++) last_upd[(size_t)i * nc + j] = add(T_BUILD, i, j, 0, 0, cm.build);
    make_diagx(0);
    dep(diagx[0], last_upd[0]);
    for (int k = 0; k < nc; k++) {
        for (int i = k + 1; i < nr; i++) {
            if (i == k + 1 && i < nc) continue;  // inside DIAGX(k+1)
            if (k < start_of(i)) continue;        // zero block of an identity row
            const int id = add(T_TRSM, i, k, 0, 0, cm.trsm);
            trsm[(size_t)i * nc + k] = id;
            dep(id, diagx[k]);
            dep(id, last_upd[(size_t)i * nc + k]);
        }
        if (k + 1 < nc) make_diagx(k + 1);
        for (const Chunk& c : by_last[k]) {
            const bool pairable = c.nb >= cm.pair_nbmin && (c.j < nc - cm.pair_tail || (c.i >= nr0 && id_tail));
            const int role = pairable ? pair_role(c.i, c.j) : 0;
            if (role == 2) continue;  // (the pair's top row made the task: identical chunks)
            if (role == 1) {
                const int id = add(T_UPD2, c.i, c.j, c.b0, c.nb, cm.ovh + 2.0 * c.nb * cm.k128 * cm.tall);
                bool e1, e2, e3;
                for (int r = c.i; r <= c.i + 1; r++) dep(id, last_upd[(size_t)r * nc + c.j]);
                const int p1 = prodL(c.i, k, e1), p3 = prodL(c.i + 1, k, e3), p2 = prodL(c.j, k, e2);
                dep(id, p1, e1);
                dep(id, p3, e3);
                dep(id, p2, e2);
                last_upd[(size_t)c.i * nc + c.j] = id;
                last_upd[(size_t)(c.i + 1) * nc + c.j] = id;
                continue;
            }
            const double dur = cm.ovh + c.nb * cm.k128 * (c.i == c.j ? cm.diagf : 1.0);
            const int id = add(T_UPD, c.i, c.j, c.b0, c.nb, dur);
            dep(id, last_upd[(size_t)c.i * nc + c.j]);
            bool e1, e2;
            const int p1 = prodL(c.i, k, e1), p2 = prodL(c.j, k, e2);
            dep(id, p1, e1);
            dep(id, p2, e2);
            last_upd[(size_t)c.i * nc + c.j] = id;
        }
    }
    const int nt = (int)tasks.size();
    deps.resize(nt);
    edeps.resize(nt);
    for (int id = 0; id < nt; id++) {
        auto& d = deps[id];
        auto& ed = edeps[id];
        std::sort(d.begin(), d.end());
        d.erase(std::unique(d.begin(), d.end()), d.end());
        std::sort(ed.begin(), ed.end());
        ed.erase(std::unique(ed.begin(), ed.end()), ed.end());
        for (int on : d) {
            if (on >= id) throw Error{GPRX_ERR_ARG, "potrf tile schedule: producer created after consumer"};
            tasks[on].succ.push_back(id);
        }
        int ne = 0;
        for (int on : ed) {
            if (on >= id) throw Error{GPRX_ERR_ARG, "potrf tile schedule: producer created after consumer"};
            if (std::binary_search(d.begin(), d.end(), on)) continue;  // full dependency already
            tasks[on].esucc.push_back(id);
            ne++;
        }
        tasks[id].ndep = (int)d.size() + ne;
    }
    // creation order is topological: bottom levels in reverse
    for (int id = nt - 1; id >= 0; id--) {
        double m = 0;
        for (int s : tasks[id].succ) m = std::max(m, tasks[s].bl);
        for (int s : tasks[id].esucc) m = std::max(m, tasks[s].bl - (tasks[id].dur - cm.early));
        tasks[id].bl = tasks[id].dur + m;
    }
    // list scheduling on P workers, highest bottom level first
    typedef std::pair<double, int> PQ;
    std::priority_queue<PQ> ready;
    // events: (time, task) finishing, or (time, -1 - task) for an early publication
    std::priority_queue<PQ, std::vector<PQ>, std::greater<PQ>> running;
    std::vector<int> indeg(nt);
    for (int id = 0; id < nt; id++) {
        indeg[id] = tasks[id].ndep;
        if (indeg[id] == 0) ready.push({tasks[id].bl, id});
    }
    Schedule S;
    S.list.reserve(nt);
    double now = 0;
    int freew = P;
    while ((int)S.list.size() < nt || !running.empty()) {
        while (freew > 0 && !ready.empty()) {
            const int id = ready.top().second;
            ready.pop();
            const Task& tk = tasks[id];
            S.list.push_back(make_int4(tk.type | (tk.nb << 8), tk.i, tk.j, tk.b0));
            running.push({now + tk.dur, id});
            if (!tk.esucc.empty()) running.push({now + std::min(cm.early, tk.dur), -1 - id});
            freew--;
        }
        if (running.empty()) throw Error{GPRX_ERR_ARG, "potrf tile schedule: dependency cycle"};
        const PQ f = running.top();
        running.pop();
        now = f.first;
        if (f.second < 0) {
            for (int s : tasks[-1 - f.second].esucc)
                if (--indeg[s] == 0) ready.push({tasks[s].bl, s});
            continue;
        }
        freew++;
        for (int s : tasks[f.second].succ)
            if (--indeg[s] == 0) ready.push({tasks[s].bl, s});
    }
    S.est_us = now;
    S.ntasks = nt;
    S.ident_even = ident_even;
    if (split) order_tparts(S.list);
    return S;
}

// ------------------------------------------------------------------------------------------
// Distributed schedule (gprx_dist.cpp): the single-GPU task DAG with row block i on rank
// own(i) = (i / gb) mod g (identity row E_a with row a), plus, as timed nodes that occupy no
// worker:
//   push(i, b)   tile L_ib from its rank into the window of every rank that reads row i
//   pushL(k)     Linv_k from DIAGX(k)'s rank into every other rank's Linv array
//   rel(q, p)    rank q's last window-reading update chunk covering panel p is done: the window
//                slot p mod ww may be refilled on q
// A task whose input lives on another rank depends on its push node; a task that pushes a tile
// of panel b into a window depends on rel(q, b - ww) of every consumer q (flow control: chunks
// are at most ww / 2 panels wide, so a release never waits on the panel being pushed).
// Simulated on g x P workers; each rank's ticket list is its tasks in start order.  The
// simulation order is one topological order of the whole DAG, flow control included, so the
// unfinished task that started first in the simulation always has its inputs and a worker:
// the single-GPU deadlock argument, extended to the ranks and their windows.
//
// inv (LML mode): nc identity row blocks E_a = nc + 1 + a ride along (U = L^{-T}, tiles
// (E_a, b), b >= a) and the lower C = U U^T accumulates in tiles (E_a, E_c), c <= a, as
// update chunks over the panels b >= a (C_ac = -sum_b U_ab U_cb^T, stored negated).
// ------------------------------------------------------------------------------------------
static void c_chunks(int a, int W, int nc, std::vector<std::pair<int, int>>& out) {
    out.clear();
    for (int b = a; b < nc;) {
        const int e = std::min(nc, (b / W + 1) * W);
        out.push_back({b, e - b});
        b = e;
    }
}

static DistSched make_schedule_dist(int nc, bool inv, int W, int near, int P, int g, int gb, int ww, const Cost& cm0,
                                    bool build, double push_us, double rel_us, int ratio = 0, bool split = false,
                                    int tail = 0) {
    Cost cm = cm0;
    if (split) cm.early = cm.early_s;
    const int nr = nc + 1 + (inv ? nc : 0), nci = inv ? 2 * nc : nc;
    auto own = [&](int i) { return i <= nc ? (i / gb) % g : ((i - nc - 1) / gb) % g; };
    auto colx = [&](int j) { return j > nc ? j - 1 : j; };  // counter column of tile (., j)
    auto start_of = [&](int i) { return i > nc ? i - nc - 1 : 0; };
    std::vector<Task> tasks;
    std::vector<int> rank_of;  // -1: transport node
    auto add = [&](int type, int i, int j, int b0, int nb, double dur, int rk) {
        Task tk;
        tk.type = type;
        tk.i = i;
        tk.j = j;
        tk.b0 = b0;
        tk.nb = nb;
        tk.dur = dur;
        tasks.push_back(std::move(tk));
        rank_of.push_back(rk);
        return (int)tasks.size() - 1;
    };
    std::vector<int> diagx(nc, -1), pushl(nc, -1);
    std::vector<int> trsm((size_t)nr * nc, -1), push((size_t)nr * nc, -1), last_upd((size_t)nr * nci, -1);
    std::vector<std::vector<int>> deps, edeps;
    auto dep = [&](int tsk, int on, bool early = false) {
        if (on < 0) return;
        auto& d = early ? edeps : deps;
        if ((int)d.size() <= tsk) d.resize(tsk + 1);
        d[tsk].push_back(on);
    };
    auto prodL = [&](int i, int b, bool& early) -> int {
        early = i < nc && b == i - 1;
        if (i < nc && (b == i || b == i - 1)) return diagx[i];
        return trsm[(size_t)i * nc + b];
    };
    auto linv = [&](int k, int rk) { return own(k) == rk ? diagx[k] : pushl[k]; };
    // the update chunks: (i, j, b0, nb), bucketed by their last panel
    struct Chunk {
        int i, j, b0, nb;
    };
    std::vector<std::vector<Chunk>> by_last(nc);
    {
        std::vector<std::pair<int, int>> ch;
        for (int j = 1; j < nc; j++)
            for (int i = j; i < nr; i++) {
                if (i > nc && start_of(i) >= j) continue;  // identity row E_a: tiles (E_a, j > a) only
                tile_chunks(i, j, W, near, ch, start_of(i), (tail <= 0 || j >= nc - tail) ? ratio : 0);
                for (auto& c : ch) by_last[c.first + c.second - 1].push_back(Chunk{i, j, c.first, c.second});
            }
        if (inv)
            for (int aa = 0; aa < nc; aa++) {
                c_chunks(aa, W, nc, ch);
                for (int c = 0; c <= aa; c++)
                    for (auto& x : ch) by_last[x.first + x.second - 1].push_back(Chunk{nc + 1 + aa, nc + 1 + c, x.first, x.second});
            }
    }
    // who reads which row through the window, and the window-reading chunks per (rank, panel)
    DistSched S;
    S.cons.assign((size_t)g * nr, 0);
    S.need.assign((size_t)g * nc, 0);
    for (int k = 0; k < nc; k++)
        for (const Chunk& c : by_last[k]) {
            const int q = own(c.i);
            if (own(c.j) == q) continue;
            S.cons[(size_t)q * nr + c.j] = 1;
            for (int p = c.b0; p < c.b0 + c.nb; p++) S.need[(size_t)q * nc + p]++;
        }
    std::vector<int> rel((size_t)g * nc, -1);
    // producers of panel p's window tiles wait for every consumer's release of panel p - ww
    auto flow = [&](int id, int i, int p) {
        if (i == nc || p - ww < 0) return;  // the label rows go to the z area, not the window
        for (int q = 0; q < g; q++)
            if (q != own(i) && S.cons[(size_t)q * nr + i]) dep(id, rel[(size_t)q * nc + (p - ww)]);
    };
    auto make_push = [&](int i, int b, int prod) {
        bool any = false;
        for (int q = 0; q < g && !any; q++) any = q != own(i) && S.cons[(size_t)q * nr + i];
        if (!any) return;
        const int id = add(-2, i, b, 0, 0, push_us, -1);
        push[(size_t)i * nc + b] = id;
        dep(id, prod);
    };
    auto make_diagx = [&](int k) {
        int tp[8] = {-1, -1, -1, -1, -1, -1, -1, -1};
        if (split && k >= 1)  // TPART(k, np-1..0) on the owner of row block k
            for (int c = cm.np - 1; c >= 0; c--) {
                tp[c] = add(T_TPART, k, c, 0, 0,
                            (cm.prog && own(k - 1) == own(k)) ? cm.tpart_prog : cm.tpart + cm.tpart_c * (c + 1), own(k));
                dep(tp[c], linv(k - 1, own(k)));
                dep(tp[c], last_upd[(size_t)k * nci + (k - 1)]);
                dep(tp[c], last_upd[(size_t)k * nci + k]);  // phase 2 starts from A_kk
            }
        const int id = add(T_DIAGX, k, k, 0, 0, (k == 0) ? cm.diag0 : (split ? cm.diagx_s : cm.diagx), own(k));
        diagx[k] = id;
        if (k >= 1) {
            for (int c = 0; c < cm.np; c++) dep(id, tp[c]);
            dep(id, linv(k - 1, own(k)));
            dep(id, last_upd[(size_t)k * nci + (k - 1)]);
            dep(id, last_upd[(size_t)k * nci + k]);
            flow(id, k, k - 1);  // it pushes L_{k,k-1} into window slot k - 1
            make_push(k, k - 1, id);
        }
        pushl[k] = add(-3, k, k, 0, 0, push_us, -1);
        dep(pushl[k], id);
    };
    if (build)
        for (int i = 0; i < nc; i++)
            for (int j = 0; j <= i; j++) last_upd[(size_t)i * nci + j] = add(T_BUILD, i, j, 0, 0, cm.build, own(i));
    make_diagx(0);
    dep(diagx[0], last_upd[0]);
    for (int k = 0; k < nc; k++) {
        if (k - ww >= 0)  // releases of panel k - ww: every chunk covering it was created already
            for (int q = 0; q < g; q++) {
                const int p = k - ww;
                if (!S.need[(size_t)q * nc + p]) continue;
                rel[(size_t)q * nc + p] = add(-4, q, p, 0, 0, rel_us, -1);  // its chunks: wired below
            }
        for (int i = k + 1; i < nr; i++) {
            if (i == k + 1 && i < nc) continue;  // inside DIAGX(k+1)
            if (k < start_of(i)) continue;        // zero block of an identity row
            const int id = add(T_TRSM, i, k, 0, 0, cm.trsm, own(i));
            trsm[(size_t)i * nc + k] = id;
            dep(id, linv(k, own(i)));
            dep(id, last_upd[(size_t)i * nci + k]);
            flow(id, i, k);
            make_push(i, k, id);
        }
        if (k + 1 < nc) make_diagx(k + 1);
        for (const Chunk& c : by_last[k]) {
            const int rk = own(c.i);
            const double dur = cm.ovh + c.nb * cm.k128 * (c.i == c.j ? cm.diagf : 1.0);
            const int id = add(T_UPD, c.i, c.j, c.b0, c.nb, dur, rk);
            dep(id, last_upd[(size_t)c.i * nci + colx(c.j)]);
            bool e1, e2;
            dep(id, prodL(c.i, k, e1), e1);
            if (own(c.j) == rk) {
                dep(id, prodL(c.j, k, e2), e2);
            } else {
                for (int b = c.b0; b <= k; b++) dep(id, push[(size_t)c.j * nc + b]);
            }
            last_upd[(size_t)c.i * nci + colx(c.j)] = id;
        }
    }
    // the release nodes depend on the chunks that read the window (chunks are at most W <= ww
    // panels wide, so every chunk covering panel p was created before rel(., p))
    const int nt = (int)tasks.size();
    deps.resize(nt);
    edeps.resize(nt);
    for (int id = 0; id < nt; id++) {
        if (rank_of[id] >= 0 && tasks[id].type == T_UPD) {
            const Task& c = tasks[id];
            const int q = rank_of[id];
            if (own(c.j) != q)
                for (int p = c.b0; p < c.b0 + c.nb; p++) {
                    const int r = rel[(size_t)q * nc + p];
                    if (r >= 0) deps[r].push_back(id);
                }
        }
    }
    for (int id = 0; id < nt; id++) {
        auto& d = deps[id];
        auto& ed = edeps[id];
        std::sort(d.begin(), d.end());
        d.erase(std::unique(d.begin(), d.end()), d.end());
        std::sort(ed.begin(), ed.end());
        ed.erase(std::unique(ed.begin(), ed.end()), ed.end());
        for (int on : d) {
            if (on >= id) throw Error{GPRX_ERR_ARG, "potrf dist schedule: producer created after consumer"};
            tasks[on].succ.push_back(id);
        }
        int ne = 0;
        for (int on : ed) {
            if (on >= id) throw Error{GPRX_ERR_ARG, "potrf dist schedule: producer created after consumer"};
            if (std::binary_search(d.begin(), d.end(), on)) continue;
            tasks[on].esucc.push_back(id);
            ne++;
        }
        tasks[id].ndep = (int)d.size() + ne;
    }
    // bottom levels: a release node's producers may come after it in id order, so iterate the
    // longest-path recurrence to a fixed point over a topological order (Kahn)
    {
        std::vector<int> indeg(nt, 0), order;
        order.reserve(nt);
        for (int id = 0; id < nt; id++)
            for (int s2 : tasks[id].succ) indeg[s2]++;
        for (int id = 0; id < nt; id++)
            for (int s2 : tasks[id].esucc) indeg[s2]++;
        std::vector<int> st;
        for (int id = 0; id < nt; id++)
            if (!indeg[id]) st.push_back(id);
        while (!st.empty()) {
            const int id = st.back();
            st.pop_back();
            order.push_back(id);
            for (int s2 : tasks[id].succ)
                if (--indeg[s2] == 0) st.push_back(s2);
            for (int s2 : tasks[id].esucc)
                if (--indeg[s2] == 0) st.push_back(s2);
        }
        if ((int)order.size() != nt) throw Error{GPRX_ERR_ARG, "potrf dist schedule: dependency cycle"};
        for (int x = nt - 1; x >= 0; x--) {
            const int id = order[x];
            double m = 0;
            for (int s2 : tasks[id].succ) m = std::max(m, tasks[s2].bl);
            for (int s2 : tasks[id].esucc) m = std::max(m, tasks[s2].bl - (tasks[id].dur - cm.early));
            tasks[id].bl = tasks[id].dur + m;
        }
    }
    typedef std::pair<double, int> PQ;
    std::vector<std::priority_queue<PQ>> ready(g);
    std::priority_queue<PQ, std::vector<PQ>, std::greater<PQ>> running;
    std::vector<int> indeg(nt), freew(g, P);
    S.lists.assign(g, {});
    double now = 0;
    int started = 0;
    auto make_ready = [&](int id) {
        if (rank_of[id] < 0) {  // transport / release: starts at once, no worker
            running.push({now + tasks[id].dur, id});
            started++;
        } else {
            ready[rank_of[id]].push({tasks[id].bl, id});
        }
    };
    for (int id = 0; id < nt; id++) {
        indeg[id] = tasks[id].ndep;
        if (indeg[id] == 0) make_ready(id);
    }
    while (started < nt || !running.empty()) {
        for (int rk = 0; rk < g; rk++)
            while (freew[rk] > 0 && !ready[rk].empty()) {
                const int id = ready[rk].top().second;
                ready[rk].pop();
                const Task& tk = tasks[id];
                S.lists[rk].push_back(make_int4(tk.type | (tk.nb << 8), tk.i, tk.j, tk.b0));
                running.push({now + tk.dur, id});
                if (!tk.esucc.empty()) running.push({now + std::min(cm.early, tk.dur), -1 - id});
                freew[rk]--;
                started++;
            }
        if (running.empty()) throw Error{GPRX_ERR_ARG, "potrf dist schedule: dependency cycle"};
        const PQ f = running.top();
        running.pop();
        now = f.first;
        if (f.second < 0) {
            for (int s2 : tasks[-1 - f.second].esucc)
                if (--indeg[s2] == 0) make_ready(s2);
            continue;
        }
        if (rank_of[f.second] >= 0) freew[rank_of[f.second]]++;
        for (int s2 : tasks[f.second].succ)
            if (--indeg[s2] == 0) make_ready(s2);
    }
    S.est_us = now;
    S.W = W;
    if (split)
        for (auto& l : S.lists) order_tparts(l);
    return S;
}

struct Params {
    // r01i sweep (scripts/sched_sweep.sh): at N = 16384 W = 64 with no single-panel tail is
    // 1.6-2.0% faster than W = 32, near = 1; at N = 4096 (chain-bound) near = 1 stays 6% faster
    int W = 64, near = -1;  // near < 0: by size (near_for)
    int ratio = -1;         // chunk-width rule of tile_chunks: < 0 picked per shape by the simulation
    int split = 1;          // f64: the split diagonal step (TPART tasks); GPRX_PT_SPLIT=0 turns it off
    int tail = 0;           // > 0: the capped chunk rule only in the last `tail` column blocks
    int pair = -1;          // paired updates (make_schedule): < 0 the precision's default (default_pair),
                            // 0 off, n > 0 pairs from row j + n (GPRX_PT_PAIR)
    Cost cm;
    int near_for(int nc) const { return near >= 0 ? near : (nc <= 64 ? 1 : 0); }
    Params() {
        if (const char* e = std::getenv("GPRX_PT_W")) W = std::max(1, std::atoi(e));
        if (const char* e = std::getenv("GPRX_PT_NEAR")) near = std::max(0, std::atoi(e));
        if (const char* e = std::getenv("GPRX_PT_RATIO")) ratio = std::max(0, std::atoi(e));
        if (const char* e = std::getenv("GPRX_PT_DIAGX_US")) cm.diagx = std::atof(e);
        if (const char* e = std::getenv("GPRX_PT_TRSM_US")) cm.trsm = std::atof(e);
        if (const char* e = std::getenv("GPRX_PT_K128_US")) cm.k128 = std::atof(e);
        if (const char* e = std::getenv("GPRX_PT_OVH_US")) cm.ovh = std::atof(e);
        if (const char* e = std::getenv("GPRX_PT_BUILD_US")) cm.build = std::atof(e);
        if (const char* e = std::getenv("GPRX_PT_SPLIT")) split = std::atoi(e);
        if (const char* e = std::getenv("GPRX_PT_TAIL")) tail = std::atoi(e);
        if (const char* e = std::getenv("GPRX_PT_PAIR")) pair = std::atoi(e);
        if (const char* e = std::getenv("GPRX_PT_TALL")) cm.tall = std::atof(e);
        if (const char* e = std::getenv("GPRX_PT_PAIR_NBMIN")) cm.pair_nbmin = std::max(1, std::atoi(e));
        if (const char* e = std::getenv("GPRX_PT_PAIR_TAIL")) cm.pair_tail = std::max(0, std::atoi(e));
        if (const char* e = std::getenv("GPRX_PT_TPART_US")) cm.tpart = std::atof(e);
        if (const char* e = std::getenv("GPRX_PT_DIAGXS_US")) cm.diagx_s = std::atof(e);
        if (const char* e = std::getenv("GPRX_PT_TPARTP_US")) cm.tpart_prog = std::atof(e);
    }
    // the cost model for a precision: the progressive parts are the f64 look-ahead factor's
    Cost cost(bool f64) const {
        Cost c = cm;
        c.prog = f64 && DIAG_LA && !tp_linv_form();
        c.np = tp_parts(f64 && DIAG_LA);
        return c;
    }
};
static const Params& params() {
    static Params p;
    return p;
}

// the chunk rule with the shortest simulated makespan: the fixed rule (ratio 0), or a capped
// rule (ratio 8, 4, 2: width capped by the distance to the tile's last panel) on every tile or
// only on the last 16 / 32 column blocks -- where the chain-bound tail waits for the diagonal
// tiles' last wide chunks (N = 16384: ratio 2 on the last 16 blocks 25.46 -> 25.15 ms, the
// simulation ranks it first too) -- unless GPRX_PT_RATIO fixes it (GPRX_PT_TAIL its reach)
static const int kRatios[] = {0, 8, 4, 2};
static const int kTails[] = {0, 16, 32};
// Paired updates (T_UPD2) by precision, from same-box A/Bs (profiles/r06f_pair_ab.txt,
// r06lno_pair_sweep.txt, r06uv_pair_tune.txt): rows from j + 4 (f64) / j + 2 (f32), chunks of at
// least 4 panels, not in the last 32 (f64) / 16 (f32) columns -- C3's launch 25.49-25.63 ->
// 24.68-24.85 ms (pairing every chunk: 25.77; every chunk of >= 16 panels before the last 64
// columns: 25.01-25.07; rows from j + 3 or j + 6, >= 2 panels, the last 24 or 40 columns: within
// 0.3% of the default), C4's f32 factor 99.26 -> 95.23-95.26 ms (rows from j + 4: 95.5).  Pairs delay their consumers (both rows wait for the later one), which the
// narrow pieces near a tile's last panel and the chain-bound last columns cannot afford; the bulk
// gains the wider mainloop.  GPRX_PT_PAIR / _NBMIN / _TAIL override.
struct PairRule {
    int pair, nbmin, tail;
};
static PairRule default_pair(bool f64) { return f64 ? PairRule{4, 4, 32} : PairRule{2, 4, 16}; }
static Schedule best_schedule(int nc, int nr, const Params& pr, int P, bool build, int ni, bool split, bool f64) {
    Cost cm = pr.cost(f64);
    const PairRule pd = default_pair(f64);
    if (!std::getenv("GPRX_PT_PAIR_NBMIN")) cm.pair_nbmin = pd.nbmin;
    // with the inverse riding along (ni > 0, the LML) the factor's last columns are not the end of
    // the launch -- the identity rows' updates follow them -- so they pair too: the LML's factor
    // launch 46.83-47.00 -> 46.42-46.57 ms (last 16 columns spared: 46.49-46.60; same box,
    // profiles/r06ls_lml_pair_sweep.txt)
    if (!std::getenv("GPRX_PT_PAIR_TAIL")) cm.pair_tail = ni > 0 ? 0 : pd.tail;
    Schedule best;
    bool have = false;
    const int want = pr.pair >= 0 ? pr.pair : pd.pair;
    for (int pq : {want}) {
        auto consider = [&](Schedule&& S) {
            // a rule with more tasks (or the paired form) must win by > 0.5%
            if (!have || S.est_us < best.est_us * 0.995) {
                best = std::move(S);
                have = true;
            }
        };
        if (pr.ratio >= 0) {
            consider(make_schedule(nc, nr, pr.W, pr.near_for(nc), P, cm, build, ni, pr.ratio, split, pr.tail, pq));
            continue;
        }
        for (int r : kRatios)
            for (int tl : kTails) {
                if ((r == 0 && tl) || (tl && tl >= nc)) continue;
                consider(make_schedule(nc, nr, pr.W, pr.near_for(nc), P, cm, build, ni, r, split, tl, pq));
            }
    }
    return best;
}

// the split diagonal step runs for both precisions (f64: S through the look-ahead factor's LDS
// image; f32: S in place for the rank-8 factor), unless GPRX_PT_SPLIT=0
static bool split_for(bool f64) { (void)f64; return SPLIT_CODE && params().split != 0; }
// (the parts of a step wait for each other: at least tp_parts workgroups)
static bool split_for(bool f64, int P) { return P >= tp_parts(f64 && DIAG_LA) && split_for(f64); }

}  // namespace pt

// Per-context state: cached schedules (host + device copies) and the counter block.
struct PtState {
    struct Dev {
        int4* list = nullptr;
        int64_t n = 0;
        double est_us = 0;
        bool ident_even = false;  // (Schedule::ident_even)
        std::vector<int4> host;
    };
    std::map<std::tuple<int, int, bool, int, bool, int>, Dev> sched;  // (nc, nr, fused, ni, split, sizeof(T))
    int* ctr = nullptr;
    void* pbuf = nullptr;  // the split diagonal step's four TPART products (DB x DB each)
    size_t ctr_ints = 0;
    int ncu = 0;
    int* dbg = nullptr;  // pinned host status words (GPRX_PT_DEBUG)
    long long* trace = nullptr;  // GPRX_PT_TRACE timeline of the last launch (+ DIAGX phases)
    int64_t trace_n = 0, trace_nc = 0;
    const std::vector<int4>* last_list = nullptr;
    void* tb = nullptr;  // device copy of the launch's TileBuild
    std::vector<unsigned char> tb_last;  // its bytes (re-uploaded only when they change)
    ~PtState() {
        if (tb) (void)hipFree(tb);
        if (pbuf) (void)hipFree(pbuf);
        if (trace) (void)hipFree(trace);
        if (dbg) (void)hipHostFree(dbg);
        for (auto& kv : sched) (void)hipFree(kv.second.list);
        if (ctr) (void)hipFree(ctr);
    }
};

void pt_state_free(PtState* p) { delete p; }

// timeline of the last traced launch (GPRX_PT_TRACE): per ticket {type|nb<<8, i, j, b0} and
// {taken, ready, published, workgroup} (100 MHz wall clock)
static PtState* g_pt_state = nullptr;
int64_t pt_trace_copy(int32_t* tasks, long long* times, int64_t max) {
    if (!g_pt_state || !g_pt_state->trace || !g_pt_state->last_list) return 0;
    // rows: one per ticket, then nc DIAGX phase rows, nc diagonal-factor rows, 4 nc TPART stamp rows,
    // nc split-DIAGX stamp rows
    const int64_t n = std::min<int64_t>(max, g_pt_state->trace_n + 7 * g_pt_state->trace_nc);
    GPRX_HIP(hipDeviceSynchronize());
    GPRX_HIP(hipMemcpy(times, g_pt_state->trace, sizeof(long long) * 4 * n, hipMemcpyDeviceToHost));
    const int64_t nl = std::min<int64_t>(n, (int64_t)g_pt_state->last_list->size());
    std::memcpy(tasks, g_pt_state->last_list->data(), sizeof(int4) * nl);
    return n;
}

// debug snapshot of the last launch's per-workgroup status (GPRX_PT_DEBUG)
static int* g_pt_dbg = nullptr;
static int g_pt_dbg_n = 0;
static std::mutex g_pt_dbg_mu;
int pt_debug_snapshot(int* out, int max_wg) {
    std::lock_guard<std::mutex> lk(g_pt_dbg_mu);
    if (!g_pt_dbg) return 0;
    const int n = std::min(max_wg, g_pt_dbg_n);
    for (int k = 0; k < 4 * n; k++) out[k] = __atomic_load_n(g_pt_dbg + k, __ATOMIC_RELAXED);
    return n;
}
// a distributed rank's launch (GPRX_PT_DEBUG, one rank per process): its status words, owned by
// the engine; n = 0 unregisters `dbg` if it is the registered buffer (the engine's teardown)
void pt_debug_register(int* dbg, int n) {
    std::lock_guard<std::mutex> lk(g_pt_dbg_mu);
    if (n > 0) {
        g_pt_dbg = dbg;
        g_pt_dbg_n = n;
    } else if (g_pt_dbg == dbg) {
        g_pt_dbg = nullptr;
        g_pt_dbg_n = 0;
    }
}

// ctr[i] = -1 for i in [v0, v1), 0 elsewhere (i < n)
__global__ void pt_init_counters(int* __restrict__ ctr, int64_t n, int64_t v0, int64_t v1) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) ctr[i] = (i >= v0 && i < v1) ? -1 : 0;
}

// counters of the identity row blocks (the inverse riding along): block a = i - nr0 has its
// first a panels "applied" (they are zero) and its first a L blocks "final"
// (even: the schedule pairs the identity rows, Schedule::ident_even -- an odd block's updates,
// and so its ver counters, start one panel early)
__global__ void pt_init_identity_counters(int* __restrict__ lcnt, int* __restrict__ ver, int nc, int nr0, int ni,
                                          int even) {
    const int a = blockIdx.x, j = threadIdx.x;
    if (a >= ni) return;
    if (j == 0) lcnt[nr0 + a] = a;
    const int v = even ? a - (a & 1) : a;
    for (int c = j; c < nc; c += blockDim.x) ver[(int64_t)(nr0 + a) * nc + c] = v;
}

// identity rows: A[row0 + r][c] = (r == c) for the columns at or right of r's block (even: an
// odd block from the block left of its own, a zero tile its paired updates read)
template <typename T>
__global__ void pt_init_identity_rows(T* __restrict__ A, int64_t ld, int64_t row0, int64_t nid, int64_t ncol,
                                      int even) {
    const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t c = blockIdx.y;
    const int64_t rb = r / GT, c0 = (even ? rb - (rb & 1) : rb) * GT;
    if (r >= nid || c >= ncol || c < c0) return;
    A[row0 + r + c * ld] = (r == c) ? T(1) : T(0);
}

template <typename T>
void potrf_tiles(T* A, int64_t ld, int64_t np, int64_t nrows, T* Linv, int* info, Exec& ex, const TileBuild<T>* build,
                 int ni, bool build_only) {
    using namespace pt;
    if (!ex.pt) ex.pt = new PtState();
    PtState& st = *ex.pt;
    if (st.ncu == 0) {
        int dev = 0;
        GPRX_HIP(hipGetDevice(&dev));
        hipDeviceProp_t prop;
        GPRX_HIP(hipGetDeviceProperties(&prop, dev));
        st.ncu = prop.multiProcessorCount;
    }
    GPRX_REQUIRE(np % DB == 0 && nrows % GT == 0 && nrows >= np, GPRX_ERR_ARG, "potrf_tiles: bad sizes");
    const int nc = (int)(np / DB), nr = (int)(nrows / GT);
    const bool fused = build && build->mode != 0;
    GPRX_REQUIRE(ni >= 0 && ni <= nr - nc, GPRX_ERR_ARG, "potrf_tiles: bad identity row blocks");
    GPRX_REQUIRE(!build_only || fused, GPRX_ERR_ARG, "potrf_tiles: build_only needs a fused build");
    // build_only (a parity hook, gprx_dev_build_matrix): the ticket list holds the BUILD tasks
    // alone, so the launch writes exactly the covariance tiles the fused factorisation starts from
    const bool split = split_for(std::is_same<T, double>::value, st.ncu);
    auto key = std::make_tuple(nc, nr, fused, build_only ? -1 : ni, split, (int)sizeof(T));
    auto it = st.sched.find(key);
    if (it == st.sched.end()) {
        const Params& pr = params();
        Schedule S;
        if (build_only) {
            for (int i = 0; i < nc; i++)
                for (int j = 0; j <= i; j++) S.list.push_back(make_int4(T_BUILD, i, j, 0));
        } else {
            S = best_schedule(nc, nr, pr, st.ncu, fused, ni, split, std::is_same<T, double>::value);
        }
        PtState::Dev d;
        d.n = (int64_t)S.list.size();
        d.est_us = S.est_us;
        d.ident_even = S.ident_even;
        GPRX_HIP(hipMalloc(&d.list, sizeof(int4) * std::max<int64_t>(1, d.n)));
        GPRX_HIP(hipMemcpy(d.list, S.list.data(), sizeof(int4) * d.n, hipMemcpyHostToDevice));
        d.host = S.list;
        it = st.sched.emplace(key, d).first;
    }
    const PtState::Dev& sd = it->second;
    const size_t need = (size_t)C_NCTL + nr + (size_t)nr * nc + TP_STRIDE * (size_t)nc;  // + the split step's states
    if (st.ctr_ints < need) {
        if (st.ctr) GPRX_HIP(hipFree(st.ctr));
        st.ctr = nullptr;
        GPRX_HIP(hipMalloc(&st.ctr, sizeof(int) * need));
        st.ctr_ints = need;
    }
    hipStream_t s = ex.s0;
    // counters zeroed, and (fused build) ver = -1 (not built) for the tiles of the leading
    // block (the label rows are built): one launch (the two memsets of odd sizes were five
    // fill kernels, each with its dispatch gap, on every fit)
    {
        const int64_t v0 = fused ? (int64_t)C_NCTL + nr : 0, v1 = fused ? v0 + (int64_t)nc * nc : 0;
        hipLaunchKernelGGL(pt_init_counters, dim3((unsigned)((need + 255) / 256)), dim3(256), 0, s, st.ctr,
                           (int64_t)need, v0, v1);
        GPRX_HIP(hipGetLastError());
    }
    if (ni > 0) {
        hipLaunchKernelGGL(pt_init_identity_counters, dim3((unsigned)ni), dim3(128), 0, s, st.ctr + C_NCTL,
                           st.ctr + C_NCTL + nr, nc, nr - ni, ni, sd.ident_even ? 1 : 0);
        hipLaunchKernelGGL(pt_init_identity_rows<T>, dim3((unsigned)((ni * (int64_t)GT + 255) / 256), (unsigned)np),
                           dim3(256), 0, s, A, ld, (int64_t)(nr - ni) * GT, (int64_t)ni * GT, np, sd.ident_even ? 1 : 0);
    }
    Args<T> a;
    a.A = A;
    a.ld = ld;
    a.Linv = Linv;
    a.tasks = sd.list;
    a.ntasks = (int)sd.n;
    a.nc = nc;
    a.nv = nc;
    a.ctl = st.ctr;
    a.lcnt = st.ctr + C_NCTL;
    a.ver = st.ctr + C_NCTL + nr;
    a.info = info;
    a.tb = nullptr;
    a.dist = nullptr;
    a.split = split ? 1 : 0;
    a.tflag = st.ctr + C_NCTL + nr + (size_t)nr * nc;
    if (split && !st.pbuf) GPRX_HIP(hipMalloc(&st.pbuf, sizeof(T) * 4 * DB * DB));
    a.pbuf = static_cast<T*>(st.pbuf);
    if (fused) {
        GPRX_REQUIRE(build->nf == np, GPRX_ERR_ARG, "potrf_tiles: build features must have np rows");
        if (!st.tb) GPRX_HIP(hipMalloc(&st.tb, sizeof(TileBuild<double>)));
        // (a pageable copy blocks the host until the stream reaches it: skipped when unchanged)
        const unsigned char* tbb = reinterpret_cast<const unsigned char*>(build);
        if (st.tb_last.size() != sizeof(TileBuild<T>) || std::memcmp(st.tb_last.data(), tbb, sizeof(TileBuild<T>)) != 0) {
            GPRX_HIP(hipMemcpyAsync(st.tb, build, sizeof(TileBuild<T>), hipMemcpyHostToDevice, s));
            st.tb_last.assign(tbb, tbb + sizeof(TileBuild<T>));
        }
        a.tb = reinterpret_cast<const TileBuild<T>*>(st.tb);
    }
    a.dbg = nullptr;
    a.trace = nullptr;
    a.xt = nullptr;
    static const bool tracing = std::getenv("GPRX_PT_TRACE") != nullptr;
    if (tracing) {
        if (st.trace_n + 7 * st.trace_nc < sd.n + 7 * nc) {  // + the split step's 5 nc stamp rows
            if (st.trace) GPRX_HIP(hipFree(st.trace));
            GPRX_HIP(hipMalloc(&st.trace, sizeof(long long) * 4 * (sd.n + 7 * nc)));
        }
        st.trace_n = sd.n;
        st.trace_nc = nc;
        a.trace = st.trace;
        a.xt = st.trace + 4 * (sd.n + 2 * nc);
        GPRX_HIP(hipMemsetAsync(a.xt, 0, sizeof(long long) * 4 * 5 * nc, s));
        g_pt_state = &st;
        st.last_list = &sd.host;
    }
    static const int variant = std::getenv("GPRX_PT_VARIANT") ? std::atoi(std::getenv("GPRX_PT_VARIANT")) : 0;
    a.variant = variant;
    static const bool debug = std::getenv("GPRX_PT_DEBUG") != nullptr;
    if (debug) {
        if (!st.dbg) GPRX_HIP(hipHostMalloc((void**)&st.dbg, sizeof(int) * 4 * st.ncu, hipHostMallocCoherent));
        std::memset(st.dbg, 0xff, sizeof(int) * 4 * st.ncu);
        g_pt_dbg = st.dbg;
        g_pt_dbg_n = st.ncu;
        a.dbg = st.dbg;
    }
    // one wait may take at most 2 s + 20x the whole predicted factorisation
    a.tlimit = (long long)(1e8 * (2.0 + 20.0 * sd.est_us * 1e-6));
    // + the ticket word; at least 96 KB so the launch stays at one workgroup per CU
    auto lds_of = [](size_t b) { return std::max<size_t>(b, 96 * 1024); };
    const size_t lds = lds_of(pt_lds_total<T>());
    static bool attr = false;
    if (!attr) {
        GPRX_HIP(hipFuncSetAttribute((const void*)potrf_tiles_kernel<double, false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_of(pt_lds_total<double>())));
        GPRX_HIP(hipFuncSetAttribute((const void*)potrf_tiles_kernel<float, false>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_of(pt_lds_total<float>())));
        attr = true;
    }
    const double nn = (double)np;
    ProfScope ps(KC_TILES, s,
                 nn * nn * nn / 3.0 + (double)(nrows - np - (int64_t)ni * GT) * nn * nn + (ni ? nn * nn * nn / 3.0 : 0.0),
                 0.0);
    hipLaunchKernelGGL((potrf_tiles_kernel<T, false>), dim3((unsigned)st.ncu), dim3(NT), lds, s, a);
    GPRX_HIP(hipGetLastError());
}

// ---- distributed factorisation: per-rank ticket lists and one rank's launch ------------------
DistSched potrf_dist_schedule(int nc, int g, int gb, int ww, int P, bool build, bool inv, int ratio, bool f64, int tail) {
    const pt::Params& pr = pt::params();
    // a push: one tile's stores over xGMI plus the flag (measured on one GPU as a same-device
    // copy; GPRX_DIST_PUSH_US / GPRX_DIST_REL_US override)
    double push_us = 4.0, rel_us = 2.0;
    if (const char* e = std::getenv("GPRX_DIST_PUSH_US")) push_us = std::atof(e);
    if (const char* e = std::getenv("GPRX_DIST_REL_US")) rel_us = std::atof(e);
    ww = std::max(2, std::min(ww, nc));
    // update chunks at most half a window wide (flow control, make_schedule_dist), powers of two
    int W = 1;
    while (2 * W <= std::min(pr.W, std::max(1, ww / 2))) W *= 2;
    return pt::make_schedule_dist(nc, inv, W, pr.near_for(nc), P, g, std::max(1, gb), ww, pr.cost(f64), build, push_us, rel_us,
                                  pr.ratio >= 0 ? pr.ratio : ratio, pt::split_for(f64, P), pr.ratio >= 0 ? pr.tail : tail);
}

template <typename T>
void potrf_tiles_dist_launch(const DistLaunch<T>& L) {
    using namespace pt;
    Args<T> a;
    std::memset(&a, 0, sizeof(a));
    a.A = L.A;
    a.ld = DB;
    a.Linv = L.Linv;
    a.tasks = L.list;
    a.ntasks = L.ntasks;
    a.nc = L.nc;
    a.nv = L.nci;
    a.ctl = L.ctr;
    a.lcnt = L.ctr + C_NCTL;
    a.ver = L.ctr + C_NCTL + L.nr;
    a.info = L.info;
    a.tlimit = L.tlimit;
    a.tb = L.tb_dev;
    a.dist = L.dist_dev;
    a.dbg = L.dbg;
    a.trace = L.trace;
    a.xt = nullptr;
    a.split = L.split;
    a.pbuf = L.pbuf;
    a.tflag = L.tflag;
    auto lds_of = [](size_t b) { return std::max<size_t>(b, 96 * 1024); };
    const size_t lds = lds_of(pt_lds_total<T>());
    static bool attr = false;
    if (!attr) {
        GPRX_HIP(hipFuncSetAttribute((const void*)potrf_tiles_kernel<double, true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_of(pt_lds_total<double>())));
        GPRX_HIP(hipFuncSetAttribute((const void*)potrf_tiles_kernel<float, true>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_of(pt_lds_total<float>())));
        attr = true;
    }
    hipLaunchKernelGGL((potrf_tiles_kernel<T, true>), dim3((unsigned)L.P), dim3(NT), lds, L.s, a);
    GPRX_HIP(hipGetLastError());
}
template void potrf_tiles_dist_launch<double>(const DistLaunch<double>&);
template void potrf_tiles_dist_launch<float>(const DistLaunch<float>&);

// Host-only schedule statistics (no device work): tasks, predicted makespan, and a check
// that every task's producers come earlier in the ticket order.
int64_t potrf_tiles_schedule_stats(int nc, int nr, int P, bool build, double* est_us, int ni, int ratio,
                                   int32_t* list_out, int64_t list_max, int pair) {
    if (nc < 1 || nr < nc || P < 1 || ni < 0 || ni > nr - nc)
        throw Error{GPRX_ERR_ARG, "potrf tile schedule: need nc >= 1, nr >= nc + ni, P >= 1"};
    pt::Params pr = pt::params();
    if (pair >= 0) pr.pair = pair;
    const bool split = pt::split_for(true, P);  // the f64 schedule
    pt::Schedule S = ratio >= 0 ? pt::make_schedule(nc, nr, pr.W, pr.near_for(nc), P, pr.cost(true), build, ni, ratio, split,
                                                    pr.tail, pr.pair > 0 ? pr.pair : 0)
                                : pt::best_schedule(nc, nr, pr, P, build, ni, split, true);
    if (est_us) *est_us = S.est_us;
    if (list_out)  // the ticket list: {type | nb << 8, i, j, b0} per ticket
        for (int64_t q = 0; q < (int64_t)S.list.size() && q < list_max; q++) {
            const int4 t = S.list[q];
            list_out[4 * q] = t.x, list_out[4 * q + 1] = t.y, list_out[4 * q + 2] = t.z, list_out[4 * q + 3] = t.w;
        }
    return S.ntasks;
}

bool potrf_split_for(bool f64, int P) { return pt::split_for(f64, P); }

template void potrf_tiles<double>(double*, int64_t, int64_t, int64_t, double*, int*, Exec&, const TileBuild<double>*,
                                  int, bool);
template void potrf_tiles<float>(float*, int64_t, int64_t, int64_t, float*, int*, Exec&, const TileBuild<float>*, int,
                                 bool);

}  // namespace gprx
