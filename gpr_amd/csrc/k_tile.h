// k_tile.h — the 64x64 pair-statistics tile shared by the covariance build and the fused
// prediction kernel.  256 threads; thread (tx = t & 15, ty = t >> 4) owns rows tx*4..+3 and
// columns ty*4..+3 of the tile.  Samples are staged DC dimensions at a time in LDS,
// dimension-major, so each thread reads its 4 rows / 4 columns with two 16-byte loads.
#pragma once
#include "gprx_internal.h"

namespace gprx {

constexpr int DC = 16;  // dimensions per LDS chunk

template <typename T, int NPER, bool R2>
struct TileSmem {
    T xa[R2 ? DC : 1][BT];
    T xb[R2 ? DC : 1][BT];
    T per[NPER > 0 ? NPER * 4 : 1][DC][BT];
};

// Stage a DC-dimension chunk of 64 samples (rows r0..r0+63 of a row-major n x d matrix)
// into LDS laid out [k][row].  Rows >= n and dims >= d read as zero.
template <typename T>
__device__ __forceinline__ void stage_chunk(T (*dst)[BT], const T* __restrict__ src, int64_t r0, int64_t n, int d,
                                            int k0) {
    const int t = threadIdx.x;
#pragma unroll
    for (int u = 0; u < (BT * DC) / 256; u++) {
        const int e = t + 256 * u;
        const int row = e / DC, k = e % DC;
        const int64_t gr = r0 + row;
        T v = T(0);
        if (gr < n && k0 + k < d) v = src[gr * d + k0 + k];
        dst[k][row] = v;
    }
}

// Accumulate the pair statistics of the tile (rows i0.. of set A, columns j0.. of set B).
// tabA/tabB are the periodic sin/cos tables (slot p: sin at 2p, cos at 2p+1, each n x d).
template <typename T, int NPER, bool R2>
__device__ __forceinline__ void tile_stats(TileSmem<T, NPER, R2>& sm, const T* __restrict__ Xa,
                                           const T* __restrict__ tabA, int64_t na, int64_t i0,
                                           const T* __restrict__ Xb, const T* __restrict__ tabB, int64_t nb,
                                           int64_t j0, int d, T (&r2)[4][4], T (&s0)[4][4], T (&s1)[4][4]) {
    const int t = threadIdx.x;
    const int tx = t & 15, ty = t >> 4;
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) {
            r2[a][b] = 0;
            s0[a][b] = 0;
            s1[a][b] = 0;
        }
    const int64_t nd_a = na * (int64_t)d, nd_b = nb * (int64_t)d;
    for (int k0 = 0; k0 < d; k0 += DC) {
        if (R2) {
            stage_chunk<T>(sm.xa, Xa, i0, na, d, k0);
            stage_chunk<T>(sm.xb, Xb, j0, nb, d, k0);
        }
#pragma unroll
        for (int p = 0; p < NPER; p++) {
            stage_chunk<T>(sm.per[4 * p + 0], tabA + (2 * p) * nd_a, i0, na, d, k0);
            stage_chunk<T>(sm.per[4 * p + 1], tabA + (2 * p + 1) * nd_a, i0, na, d, k0);
            stage_chunk<T>(sm.per[4 * p + 2], tabB + (2 * p) * nd_b, j0, nb, d, k0);
            stage_chunk<T>(sm.per[4 * p + 3], tabB + (2 * p + 1) * nd_b, j0, nb, d, k0);
        }
        __syncthreads();
        const int kmax = min(DC, d - k0);
        for (int k = 0; k < kmax; k++) {
            if (R2) {
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
                        const T sn = fma(sa[a], cb[b], -ca[a] * sb[b]);  // sin(b (x_a - x_b))
                        if (p == 0) s0[a][b] = fma(sn, sn, s0[a][b]);
                        else s1[a][b] = fma(sn, sn, s1[a][b]);
                    }
            }
        }
        __syncthreads();
    }
}

// Direct (untiled) pair statistics incl. the periodic b-derivative sums F_p.
template <typename T>
__device__ inline void pair_stats(const KCanon<T>& K, const T* xa, const T* xb, int d, T& r2, T& s0, T& s1, T& f0,
                                  T& f1) {
    r2 = s0 = s1 = f0 = f1 = 0;
    for (int k = 0; k < d; k++) {
        T df = xa[k] - xb[k];
        r2 = fma(df, df, r2);
        if (K.nper > 0) {
            T sn, cs;
            gsincos(K.b[0] * df, &sn, &cs);
            s0 = fma(sn, sn, s0);
            f0 += T(2) * df * cs * sn;
        }
        if (K.nper > 1) {
            T sn, cs;
            gsincos(K.b[1] * df, &sn, &cs);
            s1 = fma(sn, sn, s1);
            f1 += T(2) * df * cs * sn;
        }
    }
}

template <typename T>
__device__ inline void kernel_grad(const KCanon<T>& K, T r2, T s0, T s1, T f0, T f1, T* out /* nparams */) {
    T lv[MAX_LEAF];
#pragma unroll
    for (int l = 0; l < MAX_LEAF; l++) lv[l] = (l < K.nleaf) ? leaf_value(K.leaf[l], r2, s0, s1) : T(0);
#pragma unroll
    for (int l = 0; l < MAX_LEAF; l++) {
        if (l >= K.nleaf) break;
        T adj = 0;  // d k / d leaf_l
        for (int t = 0; t < K.nterm; t++) {
            unsigned m = K.term_mask[t];
            if (!(m & (1u << l))) continue;
            T p = 1;
#pragma unroll
            for (int l2 = 0; l2 < MAX_LEAF; l2++)
                if (l2 != l && (m & (1u << l2))) p *= lv[l2];
            adj += p;
        }
        T g[3];
        leaf_grad(K.leaf[l], r2, s0, s1, f0, f1, g);
        const int np = (K.leaf[l].type == L_WHITE) ? 1 : ((K.leaf[l].type == L_GAUSS || K.leaf[l].type == L_GAUSS_EXP) ? 2 : 3);
        for (int q = 0; q < np; q++) out[K.param_base[l] + q] = adj * g[q];
    }
}

}  // namespace gprx
