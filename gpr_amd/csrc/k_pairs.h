// k_pairs.h — pair statistics of the covariance on the MFMA units: the device pieces shared
// by the stand-alone build/predict kernels (k_pairs.hip) and the tile-dataflow factorisation,
// which builds each covariance tile as a task of its own (k_ptiles.hip, BUILD).  The feature
// layout and the formulas are described at the top of k_pairs.hip.
#pragma once
#include "gprx_internal.h"
#include "k_mma.h"

#include <type_traits>

namespace gprx {
namespace pr {

using namespace mm;

constexpr int KG = 16;  // feature-column granule (the tile kernel's k-stage)

static inline int64_t rup(int64_t x, int64_t g) { return (x + g - 1) / g * g; }

template <typename T>
static inline int kr_of(const KCanon<T>& K, int d) {  // MFMA depth of the r2 product
    return K.need_r2 ? (int)rup(d, KG) : 0;
}
template <typename T>
static inline int kp_of(const KCanon<T>& K, int d) {  // MFMA depth of the periodic product
    return K.nper ? (int)rup(2 * d, KG) : 0;
}

// Kernel values of E pairs from their (r2, S) for the trees this file accepts (no White
// leaf, one periodic table).  Same formulas and products/sums as kernel_value/leaf_value
// (0 + x and 1 * x are exact, so the results are bit-identical), but organised leaf-outer:
// the loops over leaves and terms are wave-uniform (leaf constants come in through scalar
// loads, the type test is a uniform branch) and the per-pair work is an unrolled,
// statically indexed loop over E registers.  The generic kernel_value reached from 32
// unrolled call sites per thread was emitted as an out-of-line call per pair.
// FOLD (f64 predict): exp leaves with fold set take fexp_fold(f1 x + f0), which also carries
// the leaf's scale; SET: the first leaf of a sum writes p (0 + x and 1 x are exact: the same
// bits as adding to 0 / multiplying 1, one instruction less per pair).
template <typename T, int E, bool MUL, bool FOLD = false, bool SET = false>
__device__ __forceinline__ void leaf_into(const KLeaf<T>* __restrict__ L, const T (&r2)[E], const T (&s)[E],
                                          T (&p)[E]) {
    const int ty = L->type;
    const T c0 = L->c0, c1 = L->c1, c2 = L->c2;
    if constexpr (FOLD && std::is_same<T, double>::value) {
        if (L->fold) {
            const T f1 = L->f1, f0 = L->f0;
            const bool per = ty == L_PERIODIC;
#pragma unroll
            for (int e = 0; e < E; e++) {
                const T f = fexp_fold(fma(f1, per ? s[e] : r2[e], f0));
                p[e] = SET ? f : (MUL ? p[e] * f : p[e] + f);
            }
            return;
        }
    }
    if constexpr (SET) {
#pragma unroll
        for (int e = 0; e < E; e++) p[e] = MUL ? T(1) : T(0);
    }
    if (ty == L_PERIODIC) {
#pragma unroll
        for (int e = 0; e < E; e++) {
            const T f = c0 * fexp(c1 * s[e]);
            p[e] = MUL ? p[e] * f : p[e] + f;
        }
    } else if (ty == L_RQ) {
        if (c2 == T(1)) {  // alpha = 1: pow(b, -1) is 1 / b (the reference's std::pow, :794-797)
#pragma unroll
            for (int e = 0; e < E; e++) {
                const T f = c0 / (T(1) + c1 * r2[e]);
                p[e] = MUL ? p[e] * f : p[e] + f;
            }
        } else {
#pragma unroll
            for (int e = 0; e < E; e++) {
                const T f = c0 * fexp(-c2 * log1p(c1 * r2[e]));
                p[e] = MUL ? p[e] * f : p[e] + f;
            }
        }
    } else {  // L_GAUSS, L_GAUSS_EXP
#pragma unroll
        for (int e = 0; e < E; e++) {
            const T f = c0 * fexp(c1 * r2[e]);
            p[e] = MUL ? p[e] * f : p[e] + f;
        }
    }
}

template <typename T, int E, bool FOLD = false>
__device__ __forceinline__ void pair_values(const KCanon<T>* __restrict__ K, const T (&r2)[E], const T (&s)[E],
                                            T (&v)[E]) {
    const int nl = K->nleaf;
    if (FOLD && K->sum_leaves) {  // (nl >= 1: the first leaf writes v)
        leaf_into<T, E, false, true, true>(&K->leaf[0], r2, s, v);
#pragma unroll 1
        for (int l = 1; l < nl; l++) leaf_into<T, E, false, true>(&K->leaf[l], r2, s, v);
        return;
    }
#pragma unroll
    for (int e = 0; e < E; e++) v[e] = 0;
    if (K->sum_leaves) {
#pragma unroll 1
        for (int l = 0; l < nl; l++) leaf_into<T, E, false>(&K->leaf[l], r2, s, v);
        return;
    }
    const int nt = K->nterm;
#pragma unroll 1
    for (int t = 0; t < nt; t++) {
        const unsigned msk = K->term_mask[t];
        T p[E];
#pragma unroll
        for (int e = 0; e < E; e++) p[e] = 1;
#pragma unroll 1
        for (int l = 0; l < nl; l++)
            if (msk & (1u << l)) leaf_into<T, E, true>(&K->leaf[l], r2, s, p);
#pragma unroll
        for (int e = 0; e < E; e++) v[e] += p[e];
    }
}

// Statistics of the 128 x 128 pair block (rows from FU + i0, columns from FV + j0).
template <typename T, int NPER, bool R2>
__device__ __forceinline__ void block_stats(const T* FU, int64_t nu, int64_t i0, const T* FV, int64_t nv, int64_t j0,
                                            int Kr, int Kp, T* smem, int t, typename Mfma<T>::acc_t (&ar)[2][4],
                                            typename Mfma<T>::acc_t (&ap)[2][4]) {
    if (R2 && NPER) {  // adjacent column ranges: one pass of the staging ring
        tile_mma2<T>(ar, ap, FU + i0, nu, FV + j0, nv, Kr, Kp, smem, t);
        return;
    }
    if (R2) tile_mma<T, 0, false, BKS, GPRX_PAIR_FEED>(ar, FU + i0, nu, FV + j0, nv, Kr, Kr, smem, t);
    if (NPER) {
        __syncthreads();  // the second product reuses the staging ring
        tile_mma<T, 0, false, BKS, GPRX_PAIR_FEED>(ap, FU + (int64_t)Kr * nu + i0, nu, FV + (int64_t)Kr * nv + j0, nv, Kp, Kp, smem, t);
    }
}

// max(x, 0) that keeps NaN: a non-finite input sample must give a non-finite kernel value,
// as the reference's direct differences do (its (M - M) == (M - M) check then throws,
// lib/GaussianProcess.cpp:399-401); fmax(NaN, 0) would return 0, a finite value.
template <typename T>
__device__ __forceinline__ T clamp0(T x) {
    return x < T(0) ? T(0) : x;
}

// (r2, S) of one pair from the tile products and the per-sample norms (hd = d / 2)
template <typename T, int NPER, bool R2>
__device__ __forceinline__ void pair_stats(T pr2, T pper, T nu, T nv, T hd, T& r2, T& sp) {
    r2 = R2 ? clamp0(nu + nv + pr2) : T(0);
    sp = NPER ? clamp0(fma(T(-0.5), pper, hd)) : T(0);
}
// the same without the clamps (predict): a rounding-negative statistic (~1e-16 relative, a
// query on a training point) only moves a kernel value by that much in every leaf form
// (exp, 1 / (1 + c r2), log1p), and NaN propagates as before; the clamps were 3 of the ~17
// f64 VALU instructions per pair outside the exps, which bound the predict epilogue
template <typename T, int NPER, bool R2>
__device__ __forceinline__ void pair_stats_nc(T pr2, T pper, T nu, T nv, T hd, T& r2, T& sp) {
    r2 = R2 ? nu + nv + pr2 : T(0);
    sp = NPER ? fma(T(-0.5), pper, hd) : T(0);
}

// Tile (i0, j0) of K(X, X) (+ sigma2 on the diagonal, identity beyond n) into A
// (column-major), from the features FU, FV (nf rows); plain stores of the lower triangle.
// Returns whether any of this thread's values is not finite.
template <typename T, int NPER, bool R2>
__device__ __forceinline__ bool build_tile(const KCanon<T>* __restrict__ Kd, const T* __restrict__ FU,
                                           const T* __restrict__ FV, int64_t nf, int Kr, int Kp, T hd,
                                           T* __restrict__ A, int64_t ld, int64_t n, T sigma2, int64_t i0, int64_t j0,
                                           T* smem, const int t) {
    typedef Mfma<T> Tr;
    const int lane = t & 63, w = t >> 6;
    const int wr = w & 1, wc = w >> 1, lr = lane & 15, lk = lane >> 4;
    T nu[4], nv[2][4];  // squared norms of this thread's rows and columns
    auto load_norms = [&]() {
#pragma unroll
        for (int y = 0; y < 4; y++) nu[y] = R2 ? FU[(int64_t)(Kr + Kp) * nf + i0 + wr * 64 + y * 16 + lr] : T(0);
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int reg = 0; reg < 4; reg++)
                nv[x][reg] = R2 ? FV[(int64_t)(Kr + Kp) * nf + j0 + wc * 32 + x * 16 + Tr::orow(lk, reg)] : T(0);
    };
    load_norms();  // early: the latency hides under the tile products
    typename Tr::acc_t ar[2][4], ap[2][4];
    block_stats<T, NPER, R2>(FU, nf, i0, FV, nf, j0, Kr, Kp, smem, t, ar, ap);
    bool bad = false;
    // chunks of 8 pairs per thread (column group x, registers 2h, 2h + 1): statistics ->
    // values -> stores; 8 keeps the interleaved exp sequences within registers
    constexpr int G = 2;
    auto chunk = [&](auto cc) {
        constexpr int x = decltype(cc)::value / (4 / G), h = decltype(cc)::value % (4 / G);
        T r2[4 * G], sp[4 * G], v[4 * G];
#pragma unroll
        for (int reg = G * h; reg < G * h + G; reg++)
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const int64_t gj = j0 + wc * 32 + x * 16 + Tr::orow(lk, reg);
                const int64_t gi = i0 + wr * 64 + y * 16 + lr;
                T a, b;
                pair_stats<T, NPER, R2>(R2 ? ar[x][y][reg] : T(0), NPER ? ap[x][y][reg] : T(0), nu[y], nv[x][reg], hd,
                                        a, b);
                r2[(reg - G * h) * 4 + y] = gi == gj ? T(0) : a;
                sp[(reg - G * h) * 4 + y] = gi == gj ? T(0) : b;
            }
        pair_values<T, 4 * G>(Kd, r2, sp, v);
#pragma unroll
        for (int reg = G * h; reg < G * h + G; reg++) {
            const int64_t gj = j0 + wc * 32 + x * 16 + Tr::orow(lk, reg);
            T* col = A + gj * ld;
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const int64_t gi = i0 + wr * 64 + y * 16 + lr;
                T val = v[(reg - G * h) * 4 + y];
                if (gi >= n || gj >= n) {
                    val = (gi == gj) ? T(1) : T(0);
                } else {
                    if (!isfinite(val)) bad = true;
                    if (gi == gj) val += sigma2;
                }
                if (gi >= gj) col[gi] = val;
            }
        }
    };
    chunk(std::integral_constant<int, 0>{});
    chunk(std::integral_constant<int, 1>{});
    chunk(std::integral_constant<int, 2>{});
    chunk(std::integral_constant<int, 3>{});
    return bad;
}


// Tile (i0, j0) of the cross matrix K(Xa, Xb) into A (column-major, ld): rows from FU (nfu
// rows, na valid), columns from FV (nfv rows, nb valid); only valid entries are stored.  The
// sparse fit's Kmn blocks (include/SparseGaussianProcess.h:218-235).
// With Y (one label column, nb entries): also ky[r] = sum over this tile's columns j of
// K(a_{i0+r}, b_j) Y[j], r < 128 (rows >= na get 0) -- the sparse fit's Kmn Y without a
// 128-row label tile in the rank-k accumulation.
template <typename T, int NPER, bool R2>
__device__ __forceinline__ bool cross_tile(const KCanon<T>* __restrict__ Kd, const T* __restrict__ FU, int64_t nfu,
                                           int64_t na, const T* __restrict__ FV, int64_t nfv, int64_t nb, int Kr,
                                           int Kp, T hd, T* __restrict__ A, int64_t ld, int64_t i0, int64_t j0,
                                           T* smem, const int t, const T* __restrict__ Y = nullptr,
                                           T* __restrict__ ky = nullptr) {
    typedef Mfma<T> Tr;
    const int lane = t & 63, w = t >> 6;
    const int wr = w & 1, wc = w >> 1, lr = lane & 15, lk = lane >> 4;
    T nu[4], nv[2][4];
#pragma unroll
    for (int y = 0; y < 4; y++) nu[y] = R2 ? FU[(int64_t)(Kr + Kp) * nfu + i0 + wr * 64 + y * 16 + lr] : T(0);
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int reg = 0; reg < 4; reg++)
            nv[x][reg] = R2 ? FV[(int64_t)(Kr + Kp) * nfv + j0 + wc * 32 + x * 16 + Tr::orow(lk, reg)] : T(0);
    typename Tr::acc_t ar[2][4], ap[2][4];
    block_stats<T, NPER, R2>(FU, nfu, i0, FV, nfv, j0, Kr, Kp, smem, t, ar, ap);
    bool bad = false;
    T yacc[4] = {T(0), T(0), T(0), T(0)};
    constexpr int G = 2;
    auto chunk = [&](auto cc) {
        constexpr int x = decltype(cc)::value / (4 / G), h = decltype(cc)::value % (4 / G);
        T r2[4 * G], sp[4 * G], v[4 * G];
#pragma unroll
        for (int reg = G * h; reg < G * h + G; reg++)
#pragma unroll
            for (int y = 0; y < 4; y++) {
                T a, b;
                pair_stats<T, NPER, R2>(R2 ? ar[x][y][reg] : T(0), NPER ? ap[x][y][reg] : T(0), nu[y], nv[x][reg], hd,
                                        a, b);
                r2[(reg - G * h) * 4 + y] = a;
                sp[(reg - G * h) * 4 + y] = b;
            }
        pair_values<T, 4 * G>(Kd, r2, sp, v);
#pragma unroll
        for (int reg = G * h; reg < G * h + G; reg++) {
            const int64_t gj = j0 + wc * 32 + x * 16 + Tr::orow(lk, reg);
            T* col = A + gj * ld;
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const int64_t gi = i0 + wr * 64 + y * 16 + lr;
                const T val = v[(reg - G * h) * 4 + y];
                if (gi < na && gj < nb) {
                    if (!isfinite(val)) bad = true;
                    col[gi] = val;
                }
            }
            if (Y) {
                const T yj = gj < nb ? Y[gj] : T(0);
#pragma unroll
                for (int y = 0; y < 4; y++) yacc[y] = fma(v[(reg - G * h) * 4 + y], yj, yacc[y]);
            }
        }
    };
    chunk(std::integral_constant<int, 0>{});
    chunk(std::integral_constant<int, 1>{});
    chunk(std::integral_constant<int, 2>{});
    chunk(std::integral_constant<int, 3>{});
    if (Y) {
        // rows 64 wr + 16 y + lr: over the lane groups lk (shuffles), then the 4 column waves
        // wc (LDS, in a fixed order); the staging ring is free once every wave is past it
        __syncthreads();
        T* red = smem;  // [4 wc][128 rows]
#pragma unroll
        for (int y = 0; y < 4; y++) {
            T v = yacc[y];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lk == 0) red[wc * GT + wr * 64 + y * 16 + lr] = v;
        }
        __syncthreads();
        if (t < GT) ky[t] = (i0 + t < na) ? ((red[t] + red[GT + t]) + (red[2 * GT + t] + red[3 * GT + t])) : T(0);
    }
    return bad;
}

// Sum-of-leaves trees only (K.sum_leaves): the same tile as build_tile, stored whole (the
// upper half of a diagonal tile gets the symmetric values) with write-through stores for a
// hand-off to other workgroups, and with the value separated by statistic, v = sum_{r2 leaves} leaf(r2) + sum_{periodic} leaf(S).
// The r2 part is evaluated right after the first tile product, in place of its accumulators,
// so the norms and the r2 temporaries are dead before the periodic product starts: it fits
// the register budget of the factorisation kernel (which holds the loop state of its other
// task types) without spills.  Returns whether any of this thread's values is not finite.
template <typename T, int E, bool PER>
__device__ __forceinline__ void leaves_of_class(const KCanon<T>* __restrict__ K, const T (&st)[E], T (&v)[E]) {
    // exp-form leaves only (Gaussian, GaussianExp: c0 exp(c1 r2); Periodic: c0 exp(c1 S)):
    // one short code path for both classes (pairs_tile_build leaves other trees unfused)
    const int nl = K->nleaf;
#pragma unroll 1
    for (int l = 0; l < nl; l++) {
        const KLeaf<T>& L = K->leaf[l];
        if ((L.type == L_PERIODIC) != PER) continue;
        const T c0 = L.c0, c1 = L.c1;
#pragma unroll
        for (int e = 0; e < E; e++) v[e] += c0 * exp(c1 * st[e]);  // (fexp's table loads slowed this path: 1.20 -> 1.36 ms)
    }
}

template <typename T, int NPER, bool R2>
__device__ __forceinline__ bool build_tile_sum(const KCanon<T>* __restrict__ Kd, const T* __restrict__ FU,
                                               const T* __restrict__ FV, int64_t nf, int Kr, int Kp, T hd,
                                               T* __restrict__ A, int64_t ld, int64_t n, T sigma2, int64_t i0,
                                               int64_t j0, T* smem, const int t) {
    typedef Mfma<T> Tr;
    const int lane = t & 63, w = t >> 6;
    const int wr = w & 1, wc = w >> 1, lr = lane & 15, lk = lane >> 4;
    typename Tr::acc_t ar[2][4], ap[2][4];
    // per-thread work in 8 chunks of 4 pairs, column (x, reg) = (c >> 2, c & 3), rows y:
    // compile-time chunk indices keep the accumulators in registers (a loop around the
    // leaf loops would not be unrolled, and indexing them at run time puts them in scratch)
    auto each = [&](auto fn) {
        fn(std::integral_constant<int, 0>{});
        fn(std::integral_constant<int, 1>{});
        fn(std::integral_constant<int, 2>{});
        fn(std::integral_constant<int, 3>{});
        fn(std::integral_constant<int, 4>{});
        fn(std::integral_constant<int, 5>{});
        fn(std::integral_constant<int, 6>{});
        fn(std::integral_constant<int, 7>{});
    };
    if (R2) {
        tile_mma<T, 0, false, BKS, GPRX_PAIR_FEED>(ar, FU + i0, nf, FV + j0, nf, Kr, Kr, smem, t);
        T nu[4];
#pragma unroll
        for (int y = 0; y < 4; y++) nu[y] = FU[(int64_t)(Kr + Kp) * nf + i0 + wr * 64 + y * 16 + lr];
        each([&](auto cc) {
            constexpr int x = decltype(cc)::value >> 2, reg = decltype(cc)::value & 3;
            const int64_t gj = j0 + wc * 32 + x * 16 + Tr::orow(lk, reg);
            const T nv = FV[(int64_t)(Kr + Kp) * nf + gj];
            T r2[4], v[4];
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const int64_t gi = i0 + wr * 64 + y * 16 + lr;
                r2[y] = gi == gj ? T(0) : clamp0(nu[y] + nv + ar[x][y][reg]);
                v[y] = 0;
            }
            leaves_of_class<T, 4, false>(Kd, r2, v);
#pragma unroll
            for (int y = 0; y < 4; y++) ar[x][y][reg] = v[y];
        });
    }
    if (NPER) {
        if (R2) __syncthreads();  // the second product reuses the staging ring
        tile_mma<T, 0, false, BKS, GPRX_PAIR_FEED>(ap, FU + (int64_t)Kr * nf + i0, nf, FV + (int64_t)Kr * nf + j0, nf, Kp, Kp, smem, t);
    }
    bool bad = false;
    each([&](auto cc) {
        constexpr int x = decltype(cc)::value >> 2, reg = decltype(cc)::value & 3;
        const int64_t gj = j0 + wc * 32 + x * 16 + Tr::orow(lk, reg);
        T* col = A + gj * ld;
        T v[4];
#pragma unroll
        for (int y = 0; y < 4; y++) v[y] = R2 ? ar[x][y][reg] : T(0);
        if (NPER) {
            T sp[4];
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const int64_t gi = i0 + wr * 64 + y * 16 + lr;
                sp[y] = gi == gj ? T(0) : clamp0(fma(T(-0.5), ap[x][y][reg], hd));
            }
            leaves_of_class<T, 4, true>(Kd, sp, v);
        }
#pragma unroll
        for (int y = 0; y < 4; y++) {
            const int64_t gi = i0 + wr * 64 + y * 16 + lr;
            T val = v[y];
            if (gi >= n || gj >= n) {
                val = (gi == gj) ? T(1) : T(0);
            } else {
                if (!isfinite(val)) bad = true;
                if (gi == gj) val += sigma2;
            }
            st_sc1(col + gi, val);
        }
    });
    return bad;
}

}  // namespace pr
}  // namespace gprx
