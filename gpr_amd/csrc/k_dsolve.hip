// k_dsolve.hip — the triangular solves and small kernels of the storage-sharded fit (gfx950).
//
// Replaces, for a factor whose row blocks are dealt over g ranks (gprx_dist.cpp), the same
// reference steps as k_bsolve.hip: alpha = (K + s^2 I)^{-1} Y (ComputeRegressionVectors,
// lib/GaussianProcess.cpp:642-672, C from lapack::lu_invert, include/LAPACKUtils.h:38-56), and
// the correction solve of the fp32 refinement (the reference inverts fp32 GPs in double,
// LAPACKUtils.h:85-97).  No rank holds the whole factor: rank q stores only the row blocks i it
// owns, tiles L_ik for k <= i.
//
// Back substitution (SURVEY.md 8(e) potrs row):
//     alpha_k = Linv_k^T ( z_k - sum_{i > k} L_ik^T alpha_i )
// The sum runs over rows owned by several ranks, so it is split by owner: rank q forms its
// partial w_qk = sum_{i > k, i on q} L_ik^T alpha_i (alpha_i of its own rows, solved by itself)
// and pushes it into the mailbox of own(k); own(k) adds the partials, solves alpha_k and pushes
// alpha_k into every rank's alpha area.  The chain's cross-rank hop is one DB x m partial per
// group boundary of the row ownership; everything else is local.
// Forward substitution:
//     z_i = Linv_i ( r_i - sum_{k < i} L_ik z_k )
// is row-local: own(i) holds row i; each solved z_k is pushed into every rank's z area.
//
// One launch per rank, one workgroup per 128-block (tickets: last block first for the back
// substitution, first block first for the forward one, so a workgroup waits only on blocks
// claimed before it, on every rank).  A block no rank of this launch works on is still
// waited for (its alpha / z arrives by push), so the launch ends with the whole vector here.
// Hand-off: every data store to a mailbox is a system-scope relaxed store (`sc0 sc1`: written
// through, the line dropped from this XCD's L2) and every read of pushed data a system-scope load,
// so a flag needs only each storing wave's s_waitcnt vmcnt(0) and a barrier before it -- no L2
// write-back fence per block (MI355X_MICROARCH.md, inter-workgroup visibility, the {sc0 sc1
// stores and loads both sides} form; a buffer_wbl2 costs 1.7-6.5 us, on the chain once per
// block).  The diagonal inverse of the block sits in LDS (loaded before any wait); waits are
// bounded in wall-clock time.
#include "gprx_dist.h"
#include "k_mma.h"

#include <algorithm>
#include <climits>
#include <cstring>

namespace gprx {
namespace ds {

constexpr int NT = 512;     // 8 waves
constexpr int QR = DB / 4;  // rows per thread in the column layout (thread: column t & 127, quarter t >> 7)
enum { C_TICKET = 0, C_ERR = 1, C_NCTL = 4 };

__device__ __forceinline__ unsigned ld_sys(const unsigned* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(unsigned* p, unsigned v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ T ld_nc(const T* p) {  // data another rank pushed (bypass stale lines)
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
__device__ __forceinline__ void st_nc(T* p, T v) {  // data for another workgroup or rank (written through)
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
constexpr int LSL = DB + 1;  // LDS column stride of the diagonal inverse (conflict-free row and column reads)
// Linv block (column-major, DB x DB) into LDS with stride LSL: coalesced global reads
template <typename T>
__device__ __forceinline__ void load_linv_lds(const T* __restrict__ Lb, T* __restrict__ sL, int t) {
#pragma unroll 8
    for (int v = 0; v < DB * DB / NT; v++) {
        const int e = t + v * NT, row = e & (DB - 1), col = e >> 7;
        sL[row + col * LSL] = Lb[e];
    }
}
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// Wait (every wave on its own) until *f == ep; false on timeout or another workgroup's error.
__device__ bool wait_eq(const unsigned* f, unsigned ep, int* ctl, long long t0, long long tlimit) {
    while (__builtin_amdgcn_readfirstlane(ld_sys(f)) != ep) {
        if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(ctl + C_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)))
            return false;
        if (wall_clock64() - t0 > tlimit) {
            __hip_atomic_store(ctl + C_ERR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return false;
        }
        __builtin_amdgcn_s_sleep(1);
    }
    return true;
}

template <typename T>
__device__ __forceinline__ const T* tile_of(const DSArgs<T>& a, int i, int k) {  // own row block i, column k
    return a.store + a.roff[a.loc[i]] + (int64_t)k * DB * DB;
}
template <typename T>
__device__ __forceinline__ T* mb_ptr(const DSArgs<T>& a, int q, int64_t off) {
    return reinterpret_cast<T*>(uni64(a.mb[q] + (uint64_t)off));
}
__device__ __forceinline__ unsigned* mb_flag(const uint64_t* mb, int q, int64_t off) {
    return reinterpret_cast<unsigned*>(uni64(mb[q] + (uint64_t)off));
}

// every wave's (written-through) stores drained, then (wave 0) flag word `fo` (byte offset in
// the mailboxes) = ep at every rank in mask
template <typename T>
__device__ void signal(const DSArgs<T>& a, unsigned mask, int64_t fo, unsigned ep) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if ((threadIdx.x >> 6) == 0) {
        for (int q = 0; q < a.g; q++)
            if ((mask >> q) & 1) st_sys(mb_flag(a.mb, q, fo), ep);
    }
}

// z(rhs r, column c) of block k as the back substitution's right-hand side
template <typename T>
__device__ __forceinline__ T z_of(const DSArgs<T>& a, const T* zb, int r, int c) {
    return a.zmode == 0 ? ld_nc(zb + r + (int64_t)c * DB) : ld_nc(zb + (int64_t)c * a.m + r);
}

template <typename T>
__global__ __launch_bounds__(NT) void dist_back_kernel(DSArgs<T> a) {
    __shared__ T s_part[4][DB];
    __shared__ T s_v[DB];
    __shared__ int s_int[2];
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
    T* sL = reinterpret_cast<T*>(s_dyn);  // Linv_k, stride LSL
    const int t = threadIdx.x, lane = t & 63;
    const int c = t & (DB - 1), qq = t >> 7;
    if ((t >> 6) == 0) {
        const int v = __hip_atomic_fetch_add(a.ctl + C_TICKET, (t == 0) ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_int[0] = __builtin_amdgcn_readfirstlane(v);
        // no line of an earlier solve's mailbox traffic (or right-hand side) left in this CU's
        // or this XCD's caches: the plain loads below (Linv, rhs, own tiles) see this solve's data
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    const int tk = __builtin_amdgcn_readfirstlane(s_int[0]);
    if (tk >= a.nc) return;
    const int k = a.nc - 1 - tk;
    const int ok_ = a.own[k];
    if (ok_ == a.r) {
        load_linv_lds(a.Linv + (int64_t)k * DB * DB, sL, t);
        __syncthreads();
    }
    const long long t0 = wall_clock64();
    const unsigned all = ((1u << a.g) - 1u);
    T* my_alpha = mb_ptr<T>(a, a.r, a.o_alpha);
    // does this rank own a row block above k (it then has a partial for block k)?
    const bool mine = ok_ == a.r;
    const bool has = a.last_own > k;
    bool ok = true;
    auto agree = [&](bool good) {
        __syncthreads();  // every thread has read the previous verdict
        if (t == 0) s_int[1] = 0;
        __syncthreads();
        if (!good && lane == 0) s_int[1] = 1;
        __syncthreads();
        return s_int[1] == 0;
    };
    if (mine || has) {
        // z block k (the label tiles or the forward solve's z area), waited for once
        const T* zb = nullptr;
        if (mine) {
            if (a.zmode == 0) {
                if (a.own[a.nc] == a.r) {
                    zb = tile_of(a, a.nc, k);
                } else {
                    zb = mb_ptr<T>(a, a.r, a.o_ztile) + (int64_t)k * DB * DB;
                    ok = wait_eq(mb_flag(a.mb, a.r, a.o_fflags + 4 * ((int64_t)a.nc * a.nc + k)), a.fit_ep, a.ctl, t0, a.tlimit);
                }
            } else {
                zb = mb_ptr<T>(a, a.r, a.o_zf) + (int64_t)k * DB * a.m;
                ok = wait_eq(mb_flag(a.mb, a.r, a.o_sflags + 4 * ((int64_t)a.nc + k)), a.sep, a.ctl, t0, a.tlimit);
            }
        }
        if (!agree(ok)) goto done;
        for (int r = 0; r < a.m && ok; r++) {
            T s = 0;
            for (int x = a.nown - 1; x >= 0 && ok; x--) {  // own row blocks above k, last first
                const int i = a.orows[x];
                if (i <= k) break;
                T L[QR];
                {
                    const T* p = tile_of(a, i, k) + (int64_t)c * DB + QR * qq;
#pragma unroll
                    for (int u = 0; u < QR; u++) L[u] = p[u];
                }
                ok = wait_eq(mb_flag(a.mb, a.r, a.o_sflags + 4 * (int64_t)i), a.sep, a.ctl, t0, a.tlimit);
                if (!ok) break;
                const T* ai = my_alpha + (int64_t)i * DB * a.m;
#pragma unroll
                for (int u = 0; u < QR; u++) s = fma(L[u], ld_nc(ai + (int64_t)(QR * qq + u) * a.m + r), s);
            }
            __syncthreads();  // every thread done reading the previous right-hand side's s_part
            s_part[qq][c] = s;
            if (!agree(ok)) break;
            const T w = (t < DB) ? s_part[0][t] + s_part[1][t] + s_part[2][t] + s_part[3][t] : T(0);
            if (!mine) {  // push this rank's partial for block k to its owner
                if (t < DB)
                    st_nc(mb_ptr<T>(a, ok_, a.o_part) + ((int64_t)a.r * a.nc + k) * DB * a.m + (int64_t)t * a.m + r, w);
                continue;
            }
            // the owner: the other ranks' partials (ranks owning a row block above k)
            if (r == 0) {
                for (int q = 0; q < a.g && ok; q++)
                    if (q != a.r && a.last_of[q] > k)
                        ok = wait_eq(mb_flag(a.mb, a.r, a.o_sflags + 4 * ((int64_t)2 * a.nc + (int64_t)q * a.nc + k)), a.sep,
                                     a.ctl, t0, a.tlimit);
                if (!agree(ok)) break;
            }
            if (t < DB) {
                T v = z_of(a, zb, r, t) - w;
                for (int q = 0; q < a.g; q++)
                    if (q != a.r && a.last_of[q] > k)
                        v -= ld_nc(mb_ptr<T>(a, a.r, a.o_part) + ((int64_t)q * a.nc + k) * DB * a.m + (int64_t)t * a.m + r);
                s_v[t] = v;
            }
            __syncthreads();
            {  // alpha_k = Linv_k^T v: column c, rows of quarter qq
                const T* Lk = sL + c * LSL + QR * qq;
                T acc = 0;
#pragma unroll
                for (int u = 0; u < QR; u++) acc = fma(Lk[u], s_v[QR * qq + u], acc);
                s_part[qq][c] = acc;
            }
            __syncthreads();
            if (t < DB) {
                const T al = s_part[0][t] + s_part[1][t] + s_part[2][t] + s_part[3][t];
                for (int q = 0; q < a.g; q++) st_nc(mb_ptr<T>(a, q, a.o_alpha) + ((int64_t)k * DB + t) * a.m + r, al);
            }
            __syncthreads();
        }
        if (!agree(ok)) goto done;
        if (mine) signal(a, all, a.o_sflags + 4 * (int64_t)k, a.sep);
        else signal(a, 1u << ok_, a.o_sflags + 4 * ((int64_t)2 * a.nc + (int64_t)a.r * a.nc + k), a.sep);
    }
    // alpha_k here before the launch ends (pushed by its owner)
    if (!mine) {
        ok = wait_eq(mb_flag(a.mb, a.r, a.o_sflags + 4 * (int64_t)k), a.sep, a.ctl, t0, a.tlimit);
    }
done:
    if (t == 0 && __hip_atomic_load(a.ctl + C_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(a.info, -1);
}

// z_i = Linv_i (rhs_i - sum_{k < i} L_ik z_k) on own(i); thread: row (t & 127) of block i,
// column quarter t >> 7 (the tile loads coalesce along the rows)
template <typename T>
__global__ __launch_bounds__(NT) void dist_forward_kernel(DSArgs<T> a) {
    __shared__ T s_part[4][DB];
    __shared__ T s_v[DB];
    __shared__ int s_int[2];
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
    T* sL = reinterpret_cast<T*>(s_dyn);  // Linv_i, stride LSL
    const int t = threadIdx.x, lane = t & 63;
    const int row = t & (DB - 1), cq = t >> 7;
    if ((t >> 6) == 0) {
        const int v = __hip_atomic_fetch_add(a.ctl + C_TICKET, (t == 0) ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_int[0] = __builtin_amdgcn_readfirstlane(v);
        // no line of an earlier solve's mailbox traffic (or right-hand side) left in this CU's
        // or this XCD's caches: the plain loads below (Linv, rhs, own tiles) see this solve's data
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    __syncthreads();
    const int i = __builtin_amdgcn_readfirstlane(s_int[0]);
    if (i >= a.nc) return;
    const long long t0 = wall_clock64();
    const unsigned all = ((1u << a.g) - 1u);
    T* my_z = mb_ptr<T>(a, a.r, a.o_zf);
    bool ok = true;
    auto agree = [&](bool good) {
        __syncthreads();  // every thread has read the previous verdict
        if (t == 0) s_int[1] = 0;
        __syncthreads();
        if (!good && lane == 0) s_int[1] = 1;
        __syncthreads();
        return s_int[1] == 0;
    };
    if (a.own[i] == a.r) {
        load_linv_lds(a.Linv + (int64_t)i * DB * DB, sL, t);
        __syncthreads();
        for (int r = 0; r < a.m && ok; r++) {
            T s = 0;
            for (int k = 0; k < i && ok; k++) {
                T L[QR];
                const T* p = tile_of(a, i, k) + row + (int64_t)(QR * cq) * DB;
#pragma unroll
                for (int u = 0; u < QR; u++) L[u] = p[(int64_t)u * DB];
                if (r == 0) ok = wait_eq(mb_flag(a.mb, a.r, a.o_sflags + 4 * ((int64_t)a.nc + k)), a.sep, a.ctl, t0, a.tlimit);
                if (!ok) break;
                const T* zk = my_z + (int64_t)k * DB * a.m + r;
#pragma unroll
                for (int u = 0; u < QR; u++) s = fma(L[u], ld_nc(zk + (int64_t)(QR * cq + u) * a.m), s);
            }
            __syncthreads();
            s_part[cq][row] = s;
            if (!agree(ok)) break;
            if (t < DB) s_v[t] = a.rhs[((int64_t)i * DB + t) * a.m + r] - (s_part[0][t] + s_part[1][t] + s_part[2][t] + s_part[3][t]);
            __syncthreads();
            {
                const T* Li = sL + row + QR * cq * LSL;
                T acc = 0;
#pragma unroll
                for (int u = 0; u < QR; u++) acc = fma(Li[u * LSL], s_v[QR * cq + u], acc);
                s_part[cq][row] = acc;
            }
            __syncthreads();
            if (t < DB) {
                const T zi = s_part[0][t] + s_part[1][t] + s_part[2][t] + s_part[3][t];
                for (int q = 0; q < a.g; q++) st_nc(mb_ptr<T>(a, q, a.o_zf) + ((int64_t)i * DB + t) * a.m + r, zi);
            }
            __syncthreads();
        }
        if (agree(ok)) signal(a, all, a.o_sflags + 4 * ((int64_t)a.nc + i), a.sep);
    } else {
        ok = wait_eq(mb_flag(a.mb, a.r, a.o_sflags + 4 * ((int64_t)a.nc + i)), a.sep, a.ctl, t0, a.tlimit);
    }
    if (t == 0 && __hip_atomic_load(a.ctl + C_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(a.info, -1);
}

// out[0] = 2 sum log L_ii over this rank's diagonal blocks (global index < n); out[1] = sum of
// z^2 over the label tiles when this rank owns them (else 0)
template <typename T>
__global__ __launch_bounds__(256) void dist_reduce_kernel(DSArgs<T> a, int64_t n, double* __restrict__ out) {
    __shared__ double s0[256], s1[256];
    const int t = threadIdx.x;
    double x = 0, y = 0;
    for (int xi = 0; xi < a.nown; xi++) {
        const int i = a.orows[xi];
        if (i >= a.nc) continue;
        const int64_t gi = (int64_t)i * DB + (t & (DB - 1));
        if (t < DB && gi < n) x += 2.0 * log((double)tile_of(a, i, i)[t + (int64_t)t * DB]);
    }
    if (a.own[a.nc] == a.r)
        for (int k = 0; k < a.nc; k++) {
            const T* z = tile_of(a, a.nc, k);
            for (int e = t; e < a.m * DB; e += 256) {
                const int r = e % a.m, c = e / a.m;
                if ((int64_t)k * DB + c < n) {
                    const double v = (double)z[r + (int64_t)c * DB];
                    y += v * v;
                }
            }
        }
    s0[t] = x;
    s1[t] = y;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) {
            s0[t] += s0[t + o];
            s1[t] += s1[t + o];
        }
        __syncthreads();
    }
    if (t == 0) {
        out[0] = s0[0];
        out[1] = s1[0];
    }
}

// ---- the sharded posterior covariance ---------------------------------------------------------
// One workgroup per CU of the rank's slice, tasks (own row block i, chunk c) claimed in i-major
// order: a task waits only on V_k(c), k < i, produced by tasks of smaller i on every rank, each
// rank claims its tickets in i order, so the smallest unfinished i always runs (no deadlock).
template <typename T>
__global__ __launch_bounds__(NT) void dist_pvar_kernel(PVArgs<T> a) {
    typedef mm::Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
    T* smem = reinterpret_cast<T*>(s_dyn);
    __shared__ int s_int[4];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6, lr = lane & 15, lk = lane >> 4;
    const int wr = w & 1, wc = w >> 1;
    const int64_t ldr = (int64_t)a.nch * DB;
    constexpr int VS = DB + 16 / (int)sizeof(T);  // LDS stride of the V tile (rows of 16-B vectors, fewer conflicts)
    const unsigned* vf0 = nullptr;
    bool ok = true;
    for (;;) {
        if (w == 0) {
            const int v = __hip_atomic_fetch_add(a.ctl + C_TICKET, (t == 0) ? 1 : 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_int[0] = __builtin_amdgcn_readfirstlane(v);
        }
        __syncthreads();
        const int tk = __builtin_amdgcn_readfirstlane(s_int[0]);
        if (tk >= a.nown * a.nch || !ok) break;
        const int li = tk / a.nch, c = tk - li * a.nch;
        const int i = __builtin_amdgcn_readfirstlane(a.orows[li]);
        const T* Li = a.store + a.roff[__builtin_amdgcn_readfirstlane(a.loc[i])];  // 128 x 128 i, ld DB
        vf0 = mb_flag(a.mb, a.r, a.o_vflags + 4 * (int64_t)c * a.nc);
        // acc(m, q) = sum_{k < i} L_ik V_k(c)(row, q): the ready V_k in runs of at most 64 panels
        acc_t acc[2][4];
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 4; y++) acc[x][y] = acc_t{0};
        for (int k0 = 0; k0 < i && ok;) {
            if (w == 0) {
                const int nmax = min(64, i - k0);
                const long long t0 = wall_clock64();
                int nk = 0;
                for (;;) {
                    const bool good = lane >= nmax || ld_sys(vf0 + k0 + (lane < nmax ? lane : 0)) == a.ep;
                    const unsigned long long bad = __ballot(!good);
                    nk = bad ? (int)__builtin_ctzll(bad) : nmax;  // the ready prefix
                    nk = __builtin_amdgcn_readfirstlane(nk);
                    if (nk > 0) break;
                    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(a.ctl + C_ERR, __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_AGENT))) break;
                    if (wall_clock64() - t0 > a.tlimit) {
                        __hip_atomic_store(a.ctl + C_ERR, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
                // pushed data: no stale line of an earlier use of the window in this CU's or XCD's caches
                if (nk > 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                s_int[1] = nk;
            }
            __syncthreads();
            const int nk = __builtin_amdgcn_readfirstlane(s_int[1]);
            if (nk <= 0) {
                ok = false;
                break;
            }
            // (B unused with Bpan; a null B crashed hipcc 7.2's optimizer)
            mm::tile_mma<T, 0, true>(acc, Li + (int64_t)k0 * DB * DB, DB, Li, DB, DB * nk, DB * nk, smem, t,
                                     a.vslot + ((int64_t)a.r * a.vstride + c) * a.nc + k0);
            __syncthreads();  // the staging ring is reused
            k0 += nk;
        }
        if (!ok) break;
        // W(q, m) = K(z_q, x_m) - acc(m, q), in place in R (chunk c's rows, block i's columns)
        T* Wt = a.R + (int64_t)c * DB + (int64_t)li * DB * ldr;
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 4; y++)
#pragma unroll
                for (int reg = 0; reg < 4; reg++) {
                    const int m = 64 * wr + 16 * y + lr, q = 32 * wc + 16 * x + Tr::orow(lk, reg);
                    T* p = Wt + q + (int64_t)m * ldr;
                    *p = *p - acc[x][y][reg];
                }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // V_i(c)(r, q) = sum_m Linv_i(r, m) W(q, m)
        mm::tile_mma<T>(acc, a.Linv + (int64_t)i * DB * DB, DB, Wt, ldr, DB, DB, smem, t);
        __syncthreads();  // ring done: the LDS takes V (q + r VS)
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 4; y++)
#pragma unroll
                for (int reg = 0; reg < 4; reg++) {
                    const int rr = 64 * wr + 16 * y + lr, q = 32 * wc + 16 * x + Tr::orow(lk, reg);
                    smem[q + rr * VS] = acc[x][y][reg];
                }
        __syncthreads();
        // this block's share of |L^{-1} k|^2 (or of (L^{-1} k_a) . (L^{-1} k_b)) per query column
        if (t < (a.pairs ? 64 : DB)) {
            const int j2 = a.pairs ? 64 + t : t;
            double sum = 0;
            for (int rr = 0; rr < DB; rr++) sum += (double)smem[t + rr * VS] * (double)smem[j2 + rr * VS];
            a.part[(int64_t)li * ldr + (int64_t)c * DB + t] = sum;
        }
        // V_i(c) into every rank's window slot (c, i): 16-B written-through stores, then the flags
        {
            constexpr int E = 16 / (int)sizeof(T), VPR = DB / E;  // elements per vector, vectors per row
            constexpr int NV = DB * VPR / NT;
            u4 v[NV];
#pragma unroll
            for (int u = 0; u < NV; u++) {
                const int e = t + u * NT, rr = e / VPR, q = (e % VPR) * E;
                v[u] = *reinterpret_cast<const u4*>(smem + q + rr * VS);
            }
            for (int q = 0; q < a.g; q++) {
                u4* d4 = reinterpret_cast<u4*>(uni64(a.vslot[((int64_t)q * a.vstride + c) * a.nc + i]));
#pragma unroll
                for (int u = 0; u < NV; u++)
                    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(d4 + t + u * NT), "v"(v[u]) : "memory");
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (w == 0)
            for (int q = 0; q < a.g; q++) st_sys(mb_flag(a.mb, q, a.o_vflags + 4 * ((int64_t)c * a.nc + i)), a.ep);
    }
    if (t == 0 && __hip_atomic_load(a.ctl + C_ERR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMin(a.info, -1);
}

}  // namespace ds

template <typename T>
void launch_dist_pvar(const PVArgs<T>& a, int P, hipStream_t s) {
    GPRX_REQUIRE(a.g <= 32 && a.nch >= 1 && a.nc >= 1 && P >= 1, GPRX_ERR_ARG, "dist posterior covariance: bad sizes");
    const size_t lds = std::max(mm::gemm_lds<T>(), sizeof(T) * (size_t)DB * (DB + 16 / sizeof(T)));
    static bool attr = false;
    if (!attr) {
        GPRX_HIP(hipFuncSetAttribute((const void*)ds::dist_pvar_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
        attr = true;
    }
    hipLaunchKernelGGL(ds::dist_pvar_kernel<T>, dim3((unsigned)P), dim3(ds::NT), lds, s, a);
    GPRX_HIP(hipGetLastError());
}

// dynamic LDS of the two solve kernels (the diagonal inverse, padded), set once per type
template <typename T>
static size_t dsolve_lds() {
    const size_t lds = sizeof(T) * (size_t)DB * ds::LSL;
    static bool attr = false;
    if (!attr) {
        GPRX_HIP(hipFuncSetAttribute((const void*)ds::dist_back_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
        GPRX_HIP(hipFuncSetAttribute((const void*)ds::dist_forward_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)lds));
        attr = true;
    }
    return lds;
}

template <typename T>
void launch_dist_back(const DSArgs<T>& a, hipStream_t s) {
    GPRX_REQUIRE(a.g <= 32 && a.m >= 1 && a.nc >= 1, GPRX_ERR_ARG, "dist back substitution: bad sizes");
    const size_t lds = dsolve_lds<T>();
    hipLaunchKernelGGL(ds::dist_back_kernel<T>, dim3((unsigned)a.nc), dim3(ds::NT), lds, s, a);
    GPRX_HIP(hipGetLastError());
}
template <typename T>
void launch_dist_forward(const DSArgs<T>& a, hipStream_t s) {
    GPRX_REQUIRE(a.g <= 32 && a.m >= 1 && a.nc >= 1 && a.rhs, GPRX_ERR_ARG, "dist forward substitution: bad sizes");
    const size_t lds = dsolve_lds<T>();
    hipLaunchKernelGGL(ds::dist_forward_kernel<T>, dim3((unsigned)a.nc), dim3(ds::NT), lds, s, a);
    GPRX_HIP(hipGetLastError());
}
template <typename T>
void launch_dist_reduce(const DSArgs<T>& a, int64_t n, double* out, hipStream_t s) {
    hipLaunchKernelGGL(ds::dist_reduce_kernel<T>, dim3(1), dim3(256), 0, s, a, n, out);
    GPRX_HIP(hipGetLastError());
}

#define GPRX_INST(T)                                                          \
    template void launch_dist_back<T>(const DSArgs<T>&, hipStream_t);         \
    template void launch_dist_forward<T>(const DSArgs<T>&, hipStream_t);      \
    template void launch_dist_reduce<T>(const DSArgs<T>&, int64_t, double*, hipStream_t);  \
    template void launch_dist_pvar<T>(const PVArgs<T>&, int, hipStream_t);
GPRX_INST(double)
GPRX_INST(float)
#undef GPRX_INST

}  // namespace gprx
