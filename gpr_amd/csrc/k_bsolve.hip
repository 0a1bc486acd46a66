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
#include <cstring>

namespace gprx {

namespace bs {

constexpr int NT = 512;        // 8 waves
constexpr int QR = DB / 4;     // rows per thread in the column layout: thread t -> column
                               // c = t & 127, rows QR q .. QR q + QR - 1, q = t >> 7
constexpr int CPW = DB / 8;    // streamed tiles: wave w sums columns CPW w .. CPW w + CPW - 1
enum { C_TICKET = 0, C_ERR = 1, C_NCTL = 4 };
constexpr int LDL = DB + 1;    // padded LDS column of Linv_k (2-way bank conflicts at most)
template <typename T>
constexpr size_t bs_lds() {
    return sizeof(T) * (size_t)DB * LDL;
}

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

// A streamed tile's share of one lane: rows 2l, 2l+1 of the wave's CPW columns (one 16-byte
// load per column, coalesced across the wave).  Loaded before the tile's alpha_j is waited
// for, so the load latency hides under the wait.
template <typename T>
struct TileRows {
    typedef T v2 __attribute__((ext_vector_type(2)));
    v2 x[CPW];
    __device__ __forceinline__ void load(const T* __restrict__ tile, int64_t ld, int w, int lane) {
#pragma unroll
        for (int cc = 0; cc < CPW; cc++)
            x[cc] = *reinterpret_cast<const v2*>(tile + (int64_t)(w * CPW + cc) * ld + 2 * lane);
    }
    // p[cc] += tile[2l][CPW w + cc] v0 + tile[2l + 1][CPW w + cc] v1
    __device__ __forceinline__ void apply(T v0, T v1, T (&p)[CPW]) const {
#pragma unroll
        for (int cc = 0; cc < CPW; cc++) p[cc] = fma(x[cc][0], v0, fma(x[cc][1], v1, p[cc]));
    }
};

// Sum the 64 lane partials of each of the wave's CPW = 16 columns without LDS or barriers:
// four halving exchanges (xor 32, 16, 8, 4) leave lane l with column
// 8 b5 + 4 b4 + 2 b3 + b2 (b_i = bit i of l) summed over its 16 lanes' worth, two more
// (xor 2, 1) finish the sum.  Returns that column's sum and sets col.
template <typename T>
__device__ __forceinline__ T wave_reduce_cols(T (&p)[CPW], int lane, int& col) {
    T q8[8], q4[4], q2[2], q1;
    const bool u5 = lane & 32, u4 = lane & 16, u3 = lane & 8, u2 = lane & 4;
#pragma unroll
    for (int i = 0; i < 8; i++) q8[i] = (u5 ? p[i + 8] : p[i]) + __shfl_xor(u5 ? p[i] : p[i + 8], 32);
#pragma unroll
    for (int i = 0; i < 4; i++) q4[i] = (u4 ? q8[i + 4] : q8[i]) + __shfl_xor(u4 ? q8[i] : q8[i + 4], 16);
#pragma unroll
    for (int i = 0; i < 2; i++) q2[i] = (u3 ? q4[i + 2] : q4[i]) + __shfl_xor(u3 ? q4[i] : q4[i + 2], 8);
    q1 = (u2 ? q2[1] : q2[0]) + __shfl_xor(u2 ? q2[0] : q2[1], 4);
    q1 += __shfl_xor(q1, 2);
    q1 += __shfl_xor(q1, 1);
    col = (u5 ? 8 : 0) + (u4 ? 4 : 0) + (u3 ? 2 : 0) + (u2 ? 1 : 0);
    return q1;
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
    long long* trace; // GPRX_BS_TRACE: per block {start, non-critical done, alpha_{k+1} seen, published}
    // distributed factor (optional): tile (j, k) of the factor at tiles[j * nb + k] with leading
    // dimension tld[j] (j = nb: the label rows z^T); A and ld are then unused
    const uint64_t* tiles;
    const int64_t* tld;
};

// tile (j, k) of the factor (j = nb: the label rows) and its leading dimension
template <typename T>
__device__ __forceinline__ const T* bs_tile(const Args<T>& a, int j, int k, int nb, int64_t& ld) {
    if (a.tiles) {
        ld = a.tld[j];
        return reinterpret_cast<const T*>(a.tiles[(int64_t)j * nb + k]);
    }
    ld = a.ld;
    return a.A + (int64_t)j * DB + (int64_t)k * DB * a.ld;
}

// Wait until *f != 0; false on timeout or another workgroup's error (every wave polls on its
// own: the caller agrees through LDS before the next barrier).
__device__ __forceinline__ bool wait_flag(const int* f, int* ctl, long long t0, long long tlimit) {
    while (ld_uni(f) == 0) {
        if (ld_uni(ctl + C_ERR)) return false;
        if (wall_clock64() - t0 > tlimit) {
            __hip_atomic_store(ctl + C_ERR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

// alpha is pre-filled with a NaN of a fixed payload (bs_init_kernel): a consumer polls the
// values of alpha_{k+1} themselves on the critical path -- one global round trip per block
// instead of two (poll the flag, then load the values).  No computed value has this payload.
__device__ __forceinline__ bool unset(double v) {
    return __builtin_bit_cast(unsigned long long, v) == 0x7ff4deadbeef1234ull;
}
__device__ __forceinline__ bool unset(float v) { return __builtin_bit_cast(unsigned, v) == 0x7fa5deadu; }
template <typename T>
__device__ __forceinline__ T unset_value();
template <>
__device__ __forceinline__ double unset_value<double>() {
    return __builtin_bit_cast(double, 0x7ff4deadbeef1234ull);
}
template <>
__device__ __forceinline__ float unset_value<float>() {
    return __builtin_bit_cast(float, 0x7fa5deadu);
}
// the chain's counters zeroed and alpha set to the "not yet solved" value, in one launch
template <typename T>
__global__ void bs_init_kernel(int* __restrict__ ctl, int64_t nctl, T* __restrict__ alpha, int64_t nalpha) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nctl) ctl[i] = 0;
    if (alpha && i < nalpha) alpha[i] = unset_value<T>();
}

// Load QR consecutive values starting at p (16-byte aligned) into registers.
template <typename T>
__device__ __forceinline__ void load_run(const T* __restrict__ p, T (&x)[QR]) {
    typedef T v2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int i = 0; i < QR; i += 2) {
        const v2 y = *reinterpret_cast<const v2*>(p + i);
        x[i] = y[0];
        x[i + 1] = y[1];
    }
}

// Block k = nb - 1 - ticket.  While the later blocks are still being solved (off the
// critical path) the workgroup loads Linv_k into LDS and the critical tile L_{k+1,k} into
// registers in the column layout (thread: column c, rows QR q ..), and it streams the tiles
// L_{j,k}, j >= k + 2 (coalesced, lanes over rows; each tile's loads issued before its
// alpha_j is waited for), reducing them in-wave.  The critical path once alpha_{k+1} is
// published (its values polled directly, bs_init_kernel): 32 FMAs per thread, a 4-way
// combine through LDS, 32 FMAs against Linv_k, a combine, the alpha_k stores.
template <typename T>
__global__ __launch_bounds__(NT) void backsolve_chain_kernel(Args<T> a) {
    __shared__ T s_alpha[DB];     // alpha_j being applied
    __shared__ T s_part[4][DB];   // per-quarter partial sums
    __shared__ T s_other[DB];     // sum over j >= k + 2 of L_jk^T alpha_j
    __shared__ T s_v[DB];         // v = z_k - sum_{j > k} L_jk^T alpha_j
    __shared__ int s_int[2];      // ticket, fail
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* s_linv = reinterpret_cast<T*>(smem_raw);  // column c of Linv_k at c * LDL (padded)
    const int t = threadIdx.x, w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    const int c = t & (DB - 1), q = t >> 7;
    const int nb = (int)(a.np / DB);
    int* flags = a.ctl + C_NCTL;
    if (w == 0) {
        const int v = __hip_atomic_fetch_add(a.ctl + C_TICKET, (t == 0) ? 1 : 0, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        s_int[0] = __builtin_amdgcn_readfirstlane(v);
    }
    __syncthreads();
    const int tk = __builtin_amdgcn_readfirstlane(s_int[0]);
    if (tk >= nb) return;
    const int k = nb - 1 - tk;
    const int64_t r0 = (int64_t)k * DB;
    const bool has1 = k + 1 < nb;
    if (a.trace && t == 0) a.trace[4 * k] = wall_clock64();
    // (Linv_k^T v)_c = sum_r Linv_k[r][c] v[r] from LDS; (L_jk^T x)_c likewise from registers
    {
        const T* Lk = a.Linv + (int64_t)k * DB * DB;
        for (int e = t; e < DB * DB; e += NT) s_linv[(e / DB) * LDL + (e % DB)] = Lk[e];
    }
    T t1[QR];
    if (has1) {
        int64_t l1;
        const T* p1 = bs_tile<T>(a, k + 1, k, nb, l1);
        load_run<T>(p1 + (int64_t)c * l1 + QR * q, t1);
    }
    // agree on a failed wait (waves poll on their own) before using the barriers' results
    auto agree = [&](bool ok) {
        if (t == 0) s_int[1] = 0;
        __syncthreads();
        if (!ok) s_int[1] = 1;  // (any lane: the alpha poll fails per lane)
        __syncthreads();
        return s_int[1] == 0;
    };
    bool ok = true;
    for (int r = 0; r < a.m && ok; r++) {
        int* fl = flags + (int64_t)r * nb;
        const long long t0 = wall_clock64();
        T zc;  // label row r of block k (z^T; final before the launch: loaded first, off the chain)
        {
            int64_t lz;
            const T* pz = bs_tile<T>(a, nb, k, nb, lz);
            zc = pz[r + (int64_t)c * lz];
        }
        T p[CPW];
#pragma unroll
        for (int cc = 0; cc < CPW; cc++) p[cc] = 0;
        for (int j = nb - 1; j > k + 1 && ok; j--) {
            TileRows<T> tr;
            int64_t lj;
            const T* pj = bs_tile<T>(a, j, k, nb, lj);
            tr.load(pj, lj, w, lane);
            // alpha_j's two values of this lane, polled directly (no flag round trip first: the
            // loop follows the chain front, and its last tile j = k + 2 was late for alpha_{k+1})
            const int64_t rj = (int64_t)j * DB + 2 * lane;
            const T* p0 = a.alpha + rj * a.m + r;
            const T* p1 = a.alpha + (rj + 1) * a.m + r;
            T v0 = ld_sc1(p0), v1 = ld_sc1(p1);
            while (unset(v0) || unset(v1)) {
                if (__hip_atomic_load(a.ctl + C_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                    ok = false;
                    break;
                }
                if (wall_clock64() - t0 > a.tlimit) {
                    __hip_atomic_store(a.ctl + C_ERR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
                v0 = ld_sc1(p0);
                v1 = ld_sc1(p1);
            }
            // (a lane that failed leaves the loop at once; the others find the error word set)
            if (!__builtin_amdgcn_readfirstlane(__ballot(ok) == __ballot(1))) {
                ok = false;
                break;
            }
            tr.apply(v0, v1, p);
        }
        if (!agree(ok)) break;
        {
            int col;
            const T sum = wave_reduce_cols<T>(p, lane, col);
            if ((lane & 3) == 0) s_other[CPW * w + col] = sum;
        }
        if (a.trace && r == 0 && t == 0) a.trace[4 * k + 1] = wall_clock64();
        // ---- critical path ----
        T crit = 0;
        if (has1) {
            // alpha_{k+1} polled value by value (lanes of waves 0-1), straight into s_alpha
            if (t < DB) {
                const T* ap = a.alpha + ((int64_t)(k + 1) * DB + t) * a.m + r;
                T v = ld_sc1(ap);
                while (unset(v)) {
                    if (__hip_atomic_load(a.ctl + C_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
                        ok = false;
                        break;
                    }
                    if (wall_clock64() - t0 > a.tlimit) {
                        __hip_atomic_store(a.ctl + C_ERR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                    v = ld_sc1(ap);
                }
                s_alpha[t] = v;
            }
            if (a.trace && r == 0 && t == 0) a.trace[4 * k + 2] = wall_clock64();
            if (!agree(ok)) break;  // (its barriers also publish s_alpha)
            {
                T sp = 0;
#pragma unroll
                for (int i = 0; i < QR; i++) sp = fma(t1[i], s_alpha[QR * q + i], sp);
                s_part[q][c] = sp;
            }
            __syncthreads();
            if (t < DB) crit = s_part[0][t] + s_part[1][t] + s_part[2][t] + s_part[3][t];
        } else {
            __syncthreads();  // s_other complete
        }
        if (t < DB) s_v[t] = zc - s_other[t] - crit;
        __syncthreads();
        {
            T s = 0;
#pragma unroll
            for (int i = 0; i < QR; i++) s = fma(s_linv[c * LDL + QR * q + i], s_v[QR * q + i], s);
            s_part[q][c] = s;
        }
        __syncthreads();
        if (t < DB) st_sc1(a.alpha + (r0 + t) * a.m + r, s_part[0][t] + s_part[1][t] + s_part[2][t] + s_part[3][t]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (w == 0) __hip_atomic_store(fl + k, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (a.trace && r == 0 && t == 0) a.trace[4 * k + 3] = wall_clock64();
    }
    if (t == 0 && ld_uni(a.ctl + C_ERR)) atomicMin(a.info, -1);
}

// ---------------------------------------------------------------------------------------
// Forward substitution z = L^{-1} r in ONE launch, in place in the label rows of the factor
// (rows np .. np + m - 1 hold r^T, then z^T): the correction solve of the fp32 refinement
// (gprx_api.cpp refine_f32; the reference inverts fp32 GPs in double, LAPACKUtils.h:85-97).
//     z_k = Linv_k ( r_k - sum_{j < k} L_kj z_j )                (128-row blocks k)
// Block k = ticket (first block first): it waits only on blocks claimed before it.  Lanes own
// rows (2 per lane), wave w columns 16 w .. 16 w + 15 of each tile: a tile's loads go out
// before its z_j is waited for, z_j comes in as wave-uniform sc1 loads, and the eight waves'
// row partials meet in LDS once per block.  Replaces 2 GEMM launches per block (trsm_rows).
template <typename T>
__global__ __launch_bounds__(NT) void forward_chain_kernel(Args<T> a) {
    __shared__ T s_part[8][DB];
    __shared__ T s_v[DB];
    __shared__ int s_int[2];
    const int t = threadIdx.x, w = __builtin_amdgcn_readfirstlane(t >> 6), lane = t & 63;
    const int nb = (int)(a.np / DB);
    int* flags = a.ctl + C_NCTL;
    if (w == 0) {
        const int v = __hip_atomic_fetch_add(a.ctl + C_TICKET, (t == 0) ? 1 : 0, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        s_int[0] = __builtin_amdgcn_readfirstlane(v);
    }
    __syncthreads();
    const int k = __builtin_amdgcn_readfirstlane(s_int[0]);
    if (k >= nb) return;
    T* zrows = const_cast<T*>(a.A) + a.np;  // label rows: element (rhs r, sample i) at zrows[r + i ld]
    typedef T v2 __attribute__((ext_vector_type(2)));
    bool ok = true;
    for (int r = 0; r < a.m && ok; r++) {
        int* fl = flags + (int64_t)r * nb;
        const long long t0 = wall_clock64();
        T p0 = 0, p1 = 0;  // rows 2 lane, 2 lane + 1 of block k
        for (int j = 0; j < k && ok; j++) {
            const T* tile = a.A + (int64_t)k * DB + (int64_t)j * DB * a.ld;  // L_kj
            v2 x[CPW];
#pragma unroll
            for (int cc = 0; cc < CPW; cc++)
                x[cc] = *reinterpret_cast<const v2*>(tile + (int64_t)(w * CPW + cc) * a.ld + 2 * lane);
            ok = wait_flag(fl + j, a.ctl, t0, a.tlimit);
            if (!ok) break;
#pragma unroll
            for (int cc = 0; cc < CPW; cc++) {
                const T zc = ld_sc1(zrows + r + ((int64_t)j * DB + w * CPW + cc) * a.ld);
                p0 = fma(x[cc][0], zc, p0);
                p1 = fma(x[cc][1], zc, p1);
            }
        }
        // agree on a failed wait (each wave polled on its own)
        if (t == 0) s_int[1] = 0;
        __syncthreads();
        if (!ok) s_int[1] = 1;  // (any lane: the alpha poll fails per lane)
        s_part[w][2 * lane] = p0;
        s_part[w][2 * lane + 1] = p1;
        __syncthreads();
        if (s_int[1]) {
            ok = false;
            break;
        }
        if (t < DB) {
            T acc = 0;
#pragma unroll
            for (int ww = 0; ww < 8; ww++) acc += s_part[ww][t];
            s_v[t] = zrows[r + ((int64_t)k * DB + t) * a.ld] - acc;
        }
        __syncthreads();
        // z_k = Linv_k v
        {
            const T* Lk = a.Linv + (int64_t)k * DB * DB;
            T q0 = 0, q1 = 0;
#pragma unroll
            for (int cc = 0; cc < CPW; cc++) {
                const v2 x = *reinterpret_cast<const v2*>(Lk + (int64_t)(w * CPW + cc) * DB + 2 * lane);
                const T vc = s_v[w * CPW + cc];
                q0 = fma(x[0], vc, q0);
                q1 = fma(x[1], vc, q1);
            }
            s_part[w][2 * lane] = q0;
            s_part[w][2 * lane + 1] = q1;
        }
        __syncthreads();
        if (t < DB) {
            T acc = 0;
#pragma unroll
            for (int ww = 0; ww < 8; ww++) acc += s_part[ww][t];
            st_sc1(zrows + r + ((int64_t)k * DB + t) * a.ld, acc);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (w == 0) __hip_atomic_store(fl + k, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (t == 0 && ld_uni(a.ctl + C_ERR)) atomicMin(a.info, -1);
}

}  // namespace bs

// GPRX_BS_TRACE timeline of the last launch (per block, 100 MHz wall clock)
static long long* g_bs_trace = nullptr;
static int g_bs_trace_n = 0;
int64_t bs_trace_copy(long long* out, int64_t max_blocks) {
    if (!g_bs_trace) return 0;
    const int64_t n = std::min<int64_t>(max_blocks, g_bs_trace_n);
    GPRX_HIP(hipDeviceSynchronize());
    GPRX_HIP(hipMemcpy(out, g_bs_trace, sizeof(long long) * 4 * n, hipMemcpyDeviceToHost));
    return n;
}

template <typename T>
void launch_backsolve_chain(const T* A, int64_t ld, int64_t np, int m, const T* Linv, T* alpha, int* info,
                            Exec& ex, hipStream_t s, const uint64_t* tiles, const int64_t* tld) {
    using namespace bs;
    const int nb = (int)(np / DB);
    const size_t need = (size_t)C_NCTL + (size_t)nb * m;
    GPRX_REQUIRE(np % DB == 0, GPRX_ERR_ARG, "launch_backsolve_chain: bad sizes");
    int* scratch = ex.scratch_ints(need);
    ProfScope ps(KC_BACKSOLVE, s, 2.0 * (double)np * np * m / 2.0, (double)sizeof(T) * np * (np + 1) / 2.0);
    {
        const int64_t na = np * (int64_t)m, nmax = std::max<int64_t>((int64_t)need, na);
        hipLaunchKernelGGL(bs_init_kernel<T>, dim3((unsigned)((nmax + 255) / 256)), dim3(256), 0, s, scratch,
                           (int64_t)need, alpha, na);
        GPRX_HIP(hipGetLastError());
    }
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
    a.trace = nullptr;
    a.tiles = tiles;
    a.tld = tld;
    static const bool tracing = std::getenv("GPRX_BS_TRACE") != nullptr;
    if (tracing) {
        if (g_bs_trace_n < nb) {
            if (g_bs_trace) GPRX_HIP(hipFree(g_bs_trace));
            GPRX_HIP(hipMalloc(&g_bs_trace, sizeof(long long) * 4 * nb));
        }
        g_bs_trace_n = nb;
        a.trace = g_bs_trace;
    }
    static bool attr = false;
    if (!attr) {
        GPRX_HIP(hipFuncSetAttribute((const void*)backsolve_chain_kernel<double>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)bs_lds<double>()));
        GPRX_HIP(hipFuncSetAttribute((const void*)backsolve_chain_kernel<float>,
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)bs_lds<float>()));
        attr = true;
    }
    hipLaunchKernelGGL(backsolve_chain_kernel<T>, dim3((unsigned)nb), dim3(NT), bs_lds<T>(), s, a);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void launch_forward_chain(T* A, int64_t ld, int64_t np, int m, const T* Linv, int* info, Exec& ex, hipStream_t s) {
    using namespace bs;
    const int nb = (int)(np / DB);
    const size_t need = (size_t)C_NCTL + (size_t)nb * m;
    GPRX_REQUIRE(np % DB == 0 && ld % 2 == 0, GPRX_ERR_ARG, "launch_forward_chain: bad sizes");
    int* scratch = ex.scratch_ints(need);
    ProfScope ps(KC_BACKSOLVE, s, 2.0 * (double)np * np * m / 2.0, (double)sizeof(T) * np * (np + 1) / 2.0);
    GPRX_HIP(hipMemsetAsync(scratch, 0, sizeof(int) * need, s));
    Args<T> a;
    std::memset(&a, 0, sizeof(a));
    a.A = A;
    a.ld = ld;
    a.np = np;
    a.m = m;
    a.Linv = Linv;
    a.ctl = scratch;
    a.info = info;
    a.tlimit = (long long)(1e8 * 4.0);
    hipLaunchKernelGGL(forward_chain_kernel<T>, dim3((unsigned)nb), dim3(NT), 0, s, a);
    GPRX_HIP(hipGetLastError());
}
template void launch_forward_chain<double>(double*, int64_t, int64_t, int, const double*, int*, Exec&, hipStream_t);
template void launch_forward_chain<float>(float*, int64_t, int64_t, int, const float*, int*, Exec&, hipStream_t);

template void launch_backsolve_chain<double>(const double*, int64_t, int64_t, int, const double*, double*, int*,
                                             Exec&, hipStream_t, const uint64_t*, const int64_t*);
template void launch_backsolve_chain<float>(const float*, int64_t, int64_t, int, const float*, float*, int*, Exec&,
                                            hipStream_t, const uint64_t*, const int64_t*);

}  // namespace gprx
