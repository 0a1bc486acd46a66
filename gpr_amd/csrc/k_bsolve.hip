// k_bsolve.hip — back substitution alpha = L^{-T} z in ONE launch (gfx950).
//
// Replaces the second half of the regression-vector solve (alpha = C Y with C = (K+s^2 I)^{-1},
// lib/GaussianProcess.cpp:642-672, ComputeRegressionVectors; the reference forms C explicitly
// with lapack::lu_invert, include/LAPACKUtils.h:38-56).  Here z = L^{-1} Y is already in the
// augmented rows of the factor (potrf), and
//     alpha_k = Linv_k^T ( z_k - sum_{j > k} L_jk^T alpha_j )        (128-row blocks k)
// is a chain over the blocks from the last to the first.  The stream version launched two
// kernels per block (~18 us each, 2.2 ms at N = 16384); here one workgroup per block streams
// its column panel L_{k+1..,k} (contiguous in the column-major factor) as the alpha_j it needs
// are published, and publishes alpha_k when done: the critical path per block is one
// 128 x 128 tile GEMV, the diagonal-block solve and one hand-off.
//
// Blocks are claimed through a ticket counter (last block first), so every workgroup waits
// only on blocks claimed by workgroups already running: no deadlock whatever the dispatch
// order.  alpha is handed off with sc1 (write-through) stores and sc1 loads and a relaxed
// agent-scope flag per block after every storing wave drained its stores
// (MI355X_MICROARCH.md, inter-workgroup visibility, "Valid forms"); the factor itself was
// written by the previous kernel.  Waits are bounded in wall-clock time; a timeout sets the
// error word, drains every workgroup and is reported by the caller.
#include "gprx_internal.h"

#include <algorithm>

namespace gprx {

namespace bs {

constexpr int NT = 256;   // 4 waves; wave w owns columns 32w..32w+31 of the block
constexpr int CPW = DB / 4;
enum { C_TICKET = 0, C_ERR = 1, C_NCTL = 4 };

__device__ __forceinline__ int ld_uni(const int* p) {
    return __builtin_amdgcn_readfirstlane(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
template <typename T>
__device__ __forceinline__ T ld_sc1(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <typename T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// partial[c] += sum over the 128 rows of tile (column-major, ld) of tile[r][c] * v[r], for the
// wave's 32 columns: lane l covers rows 2l, 2l+1 (one 16-byte load per column, coalesced).
template <typename T>
__device__ __forceinline__ void tile_gemv(const T* __restrict__ tile, int64_t ld, int w, int lane, T v0, T v1,
                                          T (&p)[CPW]) {
#pragma unroll
    for (int cc = 0; cc < CPW; cc++) {
        typedef T v2 __attribute__((ext_vector_type(2)));
        const v2 c2 = *reinterpret_cast<const v2*>(tile + (int64_t)(w * CPW + cc) * ld + 2 * lane);
        p[cc] = fma(c2[0], v0, fma(c2[1], v1, p[cc]));
    }
}

// sum the 64 lane partials of each of the wave's 32 columns into out[32w + cc] (LDS), in two
// passes of 16 columns (34 KB of LDS)
constexpr int RH = CPW / 2;
template <typename T>
__device__ __forceinline__ void reduce_cols(const T (&p)[CPW], int w, int lane, T (*red)[RH + 1], T* out) {
#pragma unroll
    for (int half = 0; half < 2; half++) {
#pragma unroll
        for (int cc = 0; cc < RH; cc++) red[w * 64 + lane][cc] = p[half * RH + cc];
        __syncthreads();
        // 4 lanes per column: each sums 16 of the 64 partials, then two shuffles
        const int cc = lane & (RH - 1), qd = lane >> 4;
        T s = 0;
#pragma unroll
        for (int q = 0; q < 16; q++) s += red[w * 64 + qd * 16 + q][cc];
        s += __shfl_xor(s, 16);
        s += __shfl_xor(s, 32);
        if (qd == 0) out[w * CPW + half * RH + cc] = s;
        __syncthreads();
    }
}

template <typename T>
struct Args {
    const T* A;       // factor, column-major, ld; label rows at np..np+m-1 hold z^T
    int64_t ld, np;
    int m;
    const T* Linv;    // DB x DB inverse of each diagonal block
    T* alpha;         // np x m, row-major
    int* ctl;         // [C_NCTL] then one flag per (block, rhs pass)
    int* info;        // set to -1 (atomicMin) when a wait timed out
    long long tlimit; // wall-clock ticks (100 MHz) per wait
};

template <typename T>
__global__ __launch_bounds__(NT) void backsolve_chain_kernel(Args<T> a) {
    __shared__ T red[NT][RH + 1];
    __shared__ int s_fail;
    __shared__ T svec[DB];
    __shared__ int s_k;
    const int t = threadIdx.x, w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    const int nb = (int)(a.np / DB);
    int* flags = a.ctl + C_NCTL;
    if (w == 0) {
        const int v = __hip_atomic_fetch_add(a.ctl + C_TICKET, (t == 0) ? 1 : 0, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        s_k = __builtin_amdgcn_readfirstlane(v);
    }
    __syncthreads();
    const int tk = __builtin_amdgcn_readfirstlane(s_k);
    if (tk >= nb) return;
    const int k = nb - 1 - tk;
    const int64_t r0 = (int64_t)k * DB;
    const T* Lk = a.Linv + (int64_t)k * DB * DB;
    bool ok = true;
    for (int r = 0; r < a.m && ok; r++) {
        int* fl = flags + (int64_t)r * nb;
        T p[CPW];
#pragma unroll
        for (int cc = 0; cc < CPW; cc++) p[cc] = 0;
        // s_k = sum_{j>k} L_jk^T alpha_j, tiles in the order their alpha_j appear
        const long long t0 = wall_clock64();
        for (int j = nb - 1; j > k && ok; j--) {
            while (ld_uni(fl + j) == 0) {
                if (ld_uni(a.ctl + C_ERR)) {
                    ok = false;
                    break;
                }
                if (wall_clock64() - t0 > a.tlimit) {
                    __hip_atomic_store(a.ctl + C_ERR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            if (!ok) break;
            const int64_t rj = (int64_t)j * DB + 2 * lane;
            const T v0 = ld_sc1(a.alpha + rj * a.m + r), v1 = ld_sc1(a.alpha + (rj + 1) * a.m + r);
            tile_gemv<T>(a.A + (int64_t)j * DB + r0 * a.ld, a.ld, w, lane, v0, v1, p);
        }
        // the waves poll on their own: agree before the workgroup barriers
        if (t == 0) s_fail = 0;
        __syncthreads();
        if (!ok && lane == 0) s_fail = 1;
        __syncthreads();
        if (s_fail) break;
        reduce_cols<T>(p, w, lane, red, svec);
        // v = z_k - s_k;  alpha_k = Linv_k^T v
        if (t < DB) svec[t] = a.A[a.np + r + (r0 + t) * a.ld] - svec[t];
        __syncthreads();
#pragma unroll
        for (int cc = 0; cc < CPW; cc++) p[cc] = 0;
        tile_gemv<T>(Lk, DB, w, lane, svec[2 * lane], svec[2 * lane + 1], p);
        __syncthreads();
        reduce_cols<T>(p, w, lane, red, svec);
        if (t < DB) st_sc1(a.alpha + (r0 + t) * a.m + r, svec[t]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (w == 0) __hip_atomic_store(fl + k, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 0 && ld_uni(a.ctl + C_ERR)) atomicMin(a.info, -1);
}

}  // namespace bs

template <typename T>
void launch_backsolve_chain(const T* A, int64_t ld, int64_t np, int m, const T* Linv, T* alpha, int* info,
                            Exec& ex, hipStream_t s) {
    using namespace bs;
    const int nb = (int)(np / DB);
    const size_t need = (size_t)C_NCTL + (size_t)nb * m;
    GPRX_REQUIRE(np % DB == 0, GPRX_ERR_ARG, "launch_backsolve_chain: bad sizes");
    int* scratch = ex.scratch_ints(need);
    ProfScope ps(KC_BACKSOLVE, s, 2.0 * (double)np * np * m / 2.0, (double)sizeof(T) * np * (np + 1) / 2.0);
    GPRX_HIP(hipMemsetAsync(scratch, 0, sizeof(int) * need, s));
    Args<T> a;
    a.A = A;
    a.ld = ld;
    a.np = np;
    a.m = m;
    a.Linv = Linv;
    a.alpha = alpha;
    a.ctl = scratch;
    a.info = info;
    a.tlimit = (long long)(1e8 * 4.0);
    hipLaunchKernelGGL(backsolve_chain_kernel<T>, dim3((unsigned)nb), dim3(NT), 0, s, a);
    GPRX_HIP(hipGetLastError());
}

template void launch_backsolve_chain<double>(const double*, int64_t, int64_t, int, const double*, double*, int*,
                                             Exec&, hipStream_t);
template void launch_backsolve_chain<float>(const float*, int64_t, int64_t, int, const float*, float*, int*, Exec&,
                                            hipStream_t);

}  // namespace gprx
