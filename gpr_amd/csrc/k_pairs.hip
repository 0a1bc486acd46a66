// k_pairs.hip — pair statistics of the covariance on the MFMA units (gfx950).
//
// Replaces the same reference loops as k_build.hip / k_predict.hip -- the OpenMP pair loop of
// GaussianProcess::ComputeKernelMatrixInternal (lib/GaussianProcess.cpp:384-402) with
// AddNoiseToKernelMatrix (:375-381), and the per-query kernel vector of Predict
// (lib/GaussianProcess.cpp:54-61, 684-693) -- for kernel trees whose leaves are Gaussian,
// GaussianExp, RationalQuadratic and at most one Periodic frequency (no White leaf, which
// needs the exact test r2 == 0, include/Kernel.h:696).
//
// Every leaf depends on a pair only through r2 = sum_k (x_k - y_k)^2 and
// S = sum_k sin^2(b (x_k - y_k)) (gprx_internal.h).  Both are inner products of per-sample
// feature vectors plus per-sample constants, so a 128 x 128 block of pair statistics is a
// 128 x 128 x K MFMA tile (k_mma.h) instead of O(d) VALU work per pair:
//     r2 = |x~|^2 + |y~|^2 + x~ . (-2 y~)                                   (K = d)
//     S  = d/2 - 1/2 [C_x, S_x] . [C_y, S_y]                                (K = 2 d)
// (sin^2 u = (1 - cos 2u) / 2 and cos(2b(x - y)) = C_x C_y + S_x S_y) with x~ = x - x_0
// (both sets centred on the first training sample: r2 and S are translation invariant, and
// centring keeps |x~|^2 ~ r2 so the expansion loses no significant digits), C = cos(2b x~_k),
// S = sin(2b x~_k).  Feature matrices are column-major (rows padded to 128, columns to 16) so
// the tile kernel streams them with LDS-DMA like any GEMM operand; the squared norms sit in
// one more column after the MFMA operands and are added in the epilogue.
#include "k_pairs.h"

namespace gprx {

namespace pr {

// F (np x (Kr + Kp + 1), column-major, ld np): the left (U) or right (V) features of n
// samples, then their squared norms |x~|^2.  Padding rows are all zero.
// flag (may be NULL): set when a live sample has a non-finite coordinate.  Every kernel this
// path evaluates is then non-finite on that sample's row (x - x = NaN in the reference's
// direct differences), which the reference rejects (lib/GaussianProcess.cpp:399-401); the
// feature expansion alone would hide it on the diagonal, where r2 = S = 0 is exact.
template <typename T>
__global__ void features_kernel(const T* __restrict__ X, int64_t n, int d, const T* __restrict__ center, T b,
                                int need_r2, int nper, int right, T* __restrict__ F, int64_t np, int Kr, int Kp,
                                int* __restrict__ flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    const bool live = i < n;
    if (flag && live) {
        bool bad = false;
        for (int k = 0; k < d; k++) bad |= !isfinite(X[i * d + k]);
        if (bad) atomicOr(flag, 1);
    }
    T nrm = 0;
    if (need_r2) {
        for (int k = 0; k < d; k++) {
            const T xt = live ? X[i * d + k] - center[k] : T(0);
            nrm = fma(xt, xt, nrm);
            F[i + (int64_t)k * np] = right ? T(-2) * xt : xt;
        }
        for (int k = d; k < Kr; k++) F[i + (int64_t)k * np] = 0;
    }
    F[i + (int64_t)(Kr + Kp) * np] = nrm;
    if (nper) {
        T* P = F + (int64_t)Kr * np;
        const T b2 = T(2) * b;
        for (int k = 0; k < d; k++) {
            T sn = 0, cs = 0;
            if (live) gsincos(b2 * (X[i * d + k] - center[k]), &sn, &cs);
            P[i + (int64_t)k * np] = cs;
            P[i + (int64_t)(d + k) * np] = sn;
        }
        for (int k = 2 * d; k < Kp; k++) P[i + (int64_t)k * np] = 0;
    }
}

// Lower triangle of K(X, X) (+ sigma2 on the diagonal, identity padding) into A (column-major).
template <typename T, int NPER, bool R2>
__global__ __launch_bounds__(NT) void kbuild_mma_kernel(const KCanon<T>* __restrict__ Kd, const T* __restrict__ FU,
                                                        const T* __restrict__ FV,
                                                        int64_t nf, int Kr, int Kp, T hd, T* __restrict__ A,
                                                        int64_t ld, int64_t n, T sigma2, int* __restrict__ flag) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* smem = reinterpret_cast<T*>(smem_raw);
    // the kernel tree is read from device memory (scalar loads): as a by-value kernel
    // argument indexed per leaf/term, hipcc copied it to scratch
    int64_t ti, tj;
    {
        const int64_t b = blockIdx.x;
        int64_t i = (int64_t)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
        while ((i + 1) * (i + 2) / 2 <= b) i++;
        while (i * (i + 1) / 2 > b) i--;
        ti = i;
        tj = b - i * (i + 1) / 2;
    }
    const bool bad = build_tile<T, NPER, R2>(Kd, FU, FV, nf, Kr, Kp, hd, A, ld, n, sigma2, ti * GT, tj * GT, smem,
                                                    threadIdx.x);
    if (bad) atomicOr(flag, 1);
}

// Cross matrix K(Xa, Xb) (na x nb) into A, one workgroup per 128x128 tile (grid.x over the
// rows of Xa, grid.y over the rows of Xb).
template <typename T, int NPER, bool R2>
__global__ __launch_bounds__(NT) void kcross_mma_kernel(const KCanon<T>* __restrict__ Kd, const T* __restrict__ FU,
                                                        int64_t nfu, int64_t na, const T* __restrict__ FV, int64_t nfv,
                                                        int64_t nb, int Kr, int Kp, T hd, T* __restrict__ A, int64_t ld,
                                                        int* __restrict__ flag, const T* __restrict__ Y,
                                                        T* __restrict__ kyp) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* smem = reinterpret_cast<T*>(smem_raw);
    // kyp: per column tile, the tile rows' partial K Y (nfu entries per column tile)
    T* ky = Y ? kyp + (int64_t)blockIdx.y * nfu + (int64_t)blockIdx.x * GT : nullptr;
    const bool bad = cross_tile<T, NPER, R2>(Kd, FU, nfu, na, FV, nfv, nb, Kr, Kp, hd, A, ld, (int64_t)blockIdx.x * GT,
                                             (int64_t)blockIdx.y * GT, smem, threadIdx.x, Y, ky);
    if (bad) atomicOr(flag, 1);
}

// S[row0 + 0, i] += alpha sum_{c < nct} kyp[c * nfu + i] for i < na (the label row of the
// sparse normal equations).  256 threads = 16 rows x 16 column-tile groups: group q sums
// c = q, q + 16, ... (rows in consecutive lanes: coalesced), then the 16 group sums are added
// in order through LDS -- a fixed summation order, so repeated fits agree bit for bit.
template <typename T>
__global__ __launch_bounds__(256) void ky_reduce_kernel(const T* __restrict__ kyp, int64_t nfu, int nct, int64_t na,
                                                        T alpha, T* __restrict__ S, int64_t lds, int64_t row0) {
    __shared__ T sh[16][17];
    const int r = threadIdx.x & 15, q = threadIdx.x >> 4;
    const int64_t i = (int64_t)blockIdx.x * 16 + r;
    T v = 0;
    if (i < na)
        for (int c = q; c < nct; c += 16) v += kyp[(int64_t)c * nfu + i];
    sh[q][r] = v;
    __syncthreads();
    if (q == 0 && i < na) {
        T t = 0;
#pragma unroll
        for (int u = 0; u < 16; u++) t += sh[u][r];
        S[row0 + i * lds] += alpha * t;
    }
}

// mean[q][r] = sum_j k(xq_q, x_j) alpha[j][r], r < m <= PM, one workgroup per 128 queries
// streaming the training set in 128-point blocks; K(Xq, X) is never materialised.  (PM = 1:
// more outputs per query would spill next to the two accumulator sets; they take the direct
// kernel of k_predict.hip.)
constexpr int PM = 1;
template <typename T, int NPER, bool R2>
__global__ __launch_bounds__(NT) void predict_mma_kernel(const KCanon<T>* __restrict__ Kd, const T* __restrict__ FU,
                                                         int64_t nfu,
                                                         const T* __restrict__ FV, int64_t nfv, int Kr, int Kp, T hd,
                                                         const T* __restrict__ alpha, int64_t n, int m, int64_t q,
                                                         T* __restrict__ mean) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* smem = reinterpret_cast<T*>(smem_raw);
    typedef Mfma<T> Tr;
    const int64_t i0 = (int64_t)blockIdx.x * GT;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w & 1, wc = w >> 1, lr = lane & 15, lk = lane >> 4;
    T racc[PM][4];
#pragma unroll
    for (int r = 0; r < PM; r++)
#pragma unroll
        for (int y = 0; y < 4; y++) racc[r][y] = 0;
    T nu[4];
#pragma unroll
    for (int y = 0; y < 4; y++) nu[y] = R2 ? FU[(int64_t)(Kr + Kp) * nfu + i0 + wr * 64 + y * 16 + lr] : T(0);
    // ONE staging ring over all training blocks: the stage index runs on across blocks, so the
    // next block's first stages are loading while this block's exp epilogue runs (a fresh
    // ring per block exposed its fill latency 128 times per workgroup).  Column norms and alpha
    // of a block go through LDS after the ring, double-buffered by block parity: block jb + 1's
    // are loaded at the end of block jb's epilogue (alpha = 0 masks the padding columns).
    typedef Stage<T, BKS> S;
    typedef typename Tr::acc_t acc_t;
    T* nvs = smem + gemm_lds<T>() / sizeof(T);  // [2][GT]
    T* als = nvs + 2 * GT;                      // [2][GT]
    const int nblk = (int)((n + GT - 1) / GT);
    const int NS1 = __builtin_amdgcn_readfirstlane(Kr) / BKS, NS = NS1 + __builtin_amdgcn_readfirstlane(Kp) / BKS;
    const int64_t total = (int64_t)nblk * NS;
    const int lcol = lane / S::LPC, lrow = S::src_row(lane);
    auto issue = [&](int64_t gs) {  // global stage gs: block gs / NS, k-columns (gs % NS) BKS ..
        const int jb = (int)(gs / NS), sx = (int)(gs % NS);
        T* buf = smem + (gs % NBUF) * S::STG;
        const T* A = FU + i0;
        const T* B = FV + (int64_t)jb * GT;
#pragma unroll
        for (int u = 0; u < S::IPW; u++) {
            const int g = w * S::IPW + u;
            const bool isB = g >= S::GRP;
            const int gg = isB ? g - S::GRP : g;
            const int64_t col = (int64_t)sx * BKS + gg * S::CPI + lcol;
            const T* src = isB ? (B + lrow + col * nfv) : (A + lrow + col * nfu);
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (__attribute__((address_space(3))) void*)(buf + g * S::SRP), 16, 0, 0);
        }
    };
    auto load_block_consts = [&](int jb) {  // norms / alpha of block jb into parity jb & 1
        if (t < GT) {
            const int64_t j = (int64_t)jb * GT + t;
            if (R2) nvs[(jb & 1) * GT + t] = FV[(int64_t)(Kr + Kp) * nfv + j];
            als[(jb & 1) * GT + t] = (j < n) ? alpha[j * m] : T(0);
        }
    };
    load_block_consts(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the ring's counted waits see only its loads)
#pragma unroll
    for (int p = 0; p < AHEAD; p++)
        if (p < total) issue(p);
    auto stage_sync = [&](int64_t gs) {
        const int64_t ahead = total - 1 - gs;
        if (AHEAD >= 3 && ahead >= 2) wait_vm<(AHEAD >= 3 ? 2 : 0) * S::IPW>();
        else if (AHEAD >= 2 && ahead >= 1) wait_vm<S::IPW>();
        else wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (gs + AHEAD < total) issue(gs + AHEAD);
    };
    auto stages = [&](acc_t(&acc)[2][4], int64_t gbeg, int64_t gend) {
#pragma nounroll
        for (int64_t gs = gbeg; gs < gend; gs++) {
            stage_sync(gs);
            const T* a = smem + (gs % NBUF) * S::STG;
            const T* b = a + S::GRP * S::SRP;
            T fa[2][4], fb[2][2];
            auto frag = [&](int kq, int r) {
                const int kr = kq * 4 + lk;
#pragma unroll
                for (int x = 0; x < 2; x++) fb[r][x] = b[S::at(kr, wc * 32 + x * 16 + lr)];
#pragma unroll
                for (int y = 0; y < 4; y++) fa[r][y] = a[S::at(kr, wr * 64 + y * 16 + lr)];
            };
            frag(0, 0);
#pragma unroll
            for (int kq = 0; kq < BKS / 4; kq++) {
                if (kq + 1 < BKS / 4) frag(kq + 1, (kq + 1) & 1);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int x = 0; x < 2; x++)
#pragma unroll
                    for (int y = 0; y < 4; y++) acc[x][y] = Tr::mma(fb[kq & 1][x], fa[kq & 1][y], acc[x][y]);
            }
        }
    };
#pragma nounroll
    for (int jb = 0; jb < nblk; jb++) {
        acc_t ar[2][4], ap[2][4];
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 4; y++) {
                ar[x][y] = acc_t{0};
                ap[x][y] = acc_t{0};
            }
        const int64_t g0 = (int64_t)jb * NS;
        stages(ar, g0, g0 + NS1);
        stages(ap, g0 + NS1, g0 + NS);
        const T* nvb = nvs + (jb & 1) * GT;
        const T* alb = als + (jb & 1) * GT;
        // 8 pairs per thread at a time (column group x, registers 2h, 2h + 1; rows y): eight
        // independent exp chains per wave against four -- only two waves share a SIMD
        auto chunk = [&](auto cc) {
            constexpr int x = decltype(cc)::value >> 1, h = decltype(cc)::value & 1;
            T r2[8], sp[8], v[8];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const int reg = 2 * h + u;
                const int jl = wc * 32 + x * 16 + Tr::orow(lk, reg);
#pragma unroll
                for (int y = 0; y < 4; y++)
                    pair_stats_nc<T, NPER, R2>(R2 ? ar[x][y][reg] : T(0), NPER ? ap[x][y][reg] : T(0), nu[y],
                                               R2 ? nvb[jl] : T(0), hd, r2[4 * u + y], sp[4 * u + y]);
            }
            pair_values<T, 8, true>(Kd, r2, sp, v);  // (folded exp leaves: k_pairs.h leaf_into)
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const T al = alb[wc * 32 + x * 16 + Tr::orow(lk, 2 * h + u)];
#pragma unroll
                for (int y = 0; y < 4; y++) racc[0][y] = fma(v[4 * u + y], al, racc[0][y]);
            }
        };
        chunk(std::integral_constant<int, 0>{});
        chunk(std::integral_constant<int, 1>{});
        chunk(std::integral_constant<int, 2>{});
        chunk(std::integral_constant<int, 3>{});
        if (jb + 1 < nblk) {
            load_block_consts(jb + 1);  // (read after the next stage barrier)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the prefetched stages landed during the epilogue
        }
    }
    __syncthreads();  // the reduction below reuses the ring's LDS
    // rows 64 wr + 16 y + lr: sum over the lane groups lk, then over the 4 column waves (LDS)
    T* red = smem;  // [4 wc][128 rows][PM]
#pragma unroll
    for (int r = 0; r < PM; r++)
#pragma unroll
        for (int y = 0; y < 4; y++) {
            T v = racc[r][y];
            v += __shfl_xor(v, 16);
            v += __shfl_xor(v, 32);
            if (lk == 0) red[(wc * GT + wr * 64 + y * 16 + lr) * PM + r] = v;
        }
    __syncthreads();
    if (t < GT * PM) {
        const int row = t / PM, r = t % PM;
        const int64_t gi = i0 + row;
        if (r < m && gi < q) {
            T s = 0;
#pragma unroll
            for (int c = 0; c < 4; c++) s += red[(c * GT + row) * PM + r];
            mean[gi * m + r] = s;
        }
    }
}

// ---------------------------------------------------------------------------------------
// LML gradient from pair statistics (replaces lml_grad_kernel, k_lml.hip, for sum-of-leaves
// trees): sum_{i >= j} w_ij dk_l(x_i, x_j)/dp, w_ij = (alpha_i alpha_j - C_ij) (x2 off the
// diagonal), the reference's tr((alpha alpha^T - C) D_p) (include/Likelihood.h:204-229).
// The periodic derivative in b needs F = sum_k (x_k - y_k) sin(2b (x_k - y_k)), again an
// inner product of per-sample features (K = 4d):
//   F = [x~ s, -x~ c, -s, c] . [c', s', y~ c', y~ s']    (s = sin 2b x~, c = cos 2b x~)
// ---------------------------------------------------------------------------------------
template <typename T>
__global__ void grad_features_kernel(const T* __restrict__ X, int64_t n, int d, const T* __restrict__ center, T b,
                                     int right, T* __restrict__ G, int64_t np, int Kf) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= np) return;
    const bool live = i < n;
    const T b2 = T(2) * b;
    for (int k = 0; k < d; k++) {
        T sn = 0, cs = 0, xt = 0;
        if (live) {
            xt = X[i * d + k] - center[k];
            gsincos(b2 * xt, &sn, &cs);
        }
        G[i + (int64_t)k * np] = right ? cs : xt * sn;
        G[i + (int64_t)(d + k) * np] = right ? sn : -xt * cs;
        G[i + (int64_t)(2 * d + k) * np] = right ? xt * cs : -sn;
        G[i + (int64_t)(3 * d + k) * np] = right ? xt * sn : cs;
    }
    for (int k = 4 * d; k < Kf; k++) G[i + (int64_t)k * np] = 0;
}

// One workgroup per lower 128 x 128 tile; part[tile][3 l + q] = the tile's sums (reduced
// afterwards in a fixed order: deterministic).  The statistics go one at a time through one
// accumulator set: r2 (its leaves' derivatives summed at once), then S, where the periodic
// leaf's w e and w e S are summed and w e is kept in place of S, then F (sum of w e F).
// At most one periodic leaf (pairs_grad_supported).
// CROSS: every tile of a rectangular pair block (rows: the U features, nf rows, nrow live;
// columns: the V features, nfv rows, ncol live) with weights w_ij = alpha_i beta_j - C_ij and
// no diagonal (the sparse likelihood's sum over K(X, Xm), include/SparseLikelihood.h:317-340).
template <typename T, int NPER, bool R2, bool CROSS = false>
__global__ __launch_bounds__(NT) void grad_mma_kernel(const KCanon<T>* __restrict__ Kd, const T* __restrict__ FU,
                                                      const T* __restrict__ FV, const T* __restrict__ GU,
                                                      const T* __restrict__ GV, int64_t nf, int Kr, int Kp, int Kf,
                                                      T hd, const T* __restrict__ alpha, const T* __restrict__ C,
                                                      int64_t ldc, int64_t n, double* __restrict__ part,
                                                      const uint64_t* __restrict__ ctab, int64_t nfv = 0,
                                                      int64_t ncol = 0, const T* __restrict__ beta = nullptr) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* smem = reinterpret_cast<T*>(smem_raw);
    double* sacc = reinterpret_cast<double*>(smem_raw + gemm_lds<T>());  // [8 waves][MAX_LEAF * 3]
    typedef Mfma<T> Tr;
    int64_t ti, tj;
    if (CROSS) {
        ti = blockIdx.x % (nf / GT);
        tj = blockIdx.x / (nf / GT);
    } else {
        const int64_t b = blockIdx.x;
        int64_t i = (int64_t)((sqrt(8.0 * (double)b + 1.0) - 1.0) * 0.5);
        while ((i + 1) * (i + 2) / 2 <= b) i++;
        while (i * (i + 1) / 2 > b) i--;
        ti = i;
        tj = b - i * (i + 1) / 2;
    }
    const int64_t nv_ = CROSS ? nfv : nf, ncol_ = CROSS ? ncol : n;
    const T* __restrict__ bvec = CROSS ? beta : alpha;
    // a distributed context's share (gprx_dist.cpp): C tile (ti, tj) from the rank's packed
    // storage, stored negated (the C = U U^T chunks accumulate C -= U U^T), or 0 when row block
    // ti is another rank's -- that tile contributes zero here
    const T* __restrict__ ct = nullptr;
    if (!CROSS && ctab) {
        const uint64_t pv = ctab[ti * (nf / GT) + tj];
        if (!pv) {
            if (threadIdx.x < MAX_LEAF * 3) part[(int64_t)blockIdx.x * MAX_LEAF * 3 + threadIdx.x] = 0.0;
            return;
        }
        ct = reinterpret_cast<const T*>(pv);
    }
    const int64_t i0 = ti * GT, j0 = tj * GT;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int wr = w & 1, wc = w >> 1, lr = lane & 15, lk = lane >> 4;
    const int nl = Kd->nleaf;
    // compile-time (x, reg) chunks of 4 pairs (rows y): static indices keep the accumulators
    // in registers around the run-time leaf loops
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
    auto gj_of = [&](int x, int reg) { return j0 + wc * 32 + x * 16 + Tr::orow(lk, reg); };
    auto gi_of = [&](int y) { return i0 + wr * 64 + y * 16 + lr; };
    // pair weights, zero outside the lower triangle and the matrix; loaded after each tile
    // product (held across one, they pushed the kernel into spills)
    T wt[2][4][4];
    auto load_weights = [&]() {
        each([&](auto cc) {
            constexpr int x = decltype(cc)::value >> 2, reg = decltype(cc)::value & 3;
            const int64_t gj = gj_of(x, reg);
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const int64_t gi = gi_of(y);
                const bool in = gi < n && gj < ncol_ && (CROSS || gi >= gj);
                const int64_t ci = in ? gi : 0, cj = in ? gj : 0;
                const T cv = ct ? -ct[in ? (gi - i0) + (gj - j0) * DB : 0] : C[ci + cj * ldc];
                const T v = alpha[ci] * bvec[cj] - cv;
                wt[x][y][reg] = in ? (CROSS ? v : v * (gi == gj ? T(1) : T(2))) : T(0);
            }
        });
    };
    // the wave's sums into its LDS row
    auto flush = [&](int l, double a0, double a1, double a2) {
        double v[3] = {a0, a1, a2};
#pragma unroll
        for (int q = 0; q < 3; q++) {
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) v[q] += __shfl_xor(v[q], off);
            if (lane == 0) sacc[w * MAX_LEAF * 3 + l * 3 + q] += v[q];
        }
    };
    if (t < 8 * MAX_LEAF * 3) sacc[t] = 0;
    __syncthreads();
    typename Tr::acc_t ar[2][4];
    if (R2) {
        tile_mma<T, 0, false, BKS, GPRX_PAIR_FEED>(ar, FU + i0, nf, FV + j0, nv_, Kr, Kr, smem, t);
        load_weights();
        T nu[4];
#pragma unroll
        for (int y = 0; y < 4; y++) nu[y] = FU[(int64_t)(Kr + Kp) * nf + i0 + wr * 64 + y * 16 + lr];
        each([&](auto cc) {
            constexpr int x = decltype(cc)::value >> 2, reg = decltype(cc)::value & 3;
            const int64_t gj = gj_of(x, reg);
            const T nv = FV[(int64_t)(Kr + Kp) * nv_ + gj];
#pragma unroll
            for (int y = 0; y < 4; y++)
                ar[x][y][reg] = (!CROSS && gi_of(y) == gj) ? T(0) : clamp0(nu[y] + nv + ar[x][y][reg]);
        });
        // one element loop per leaf type, with the leaf's constants hoisted (the formulas of
        // leaf_grad, gprx_internal.h, rearranged: one exp per pair, no per-pair division
        // outside RQ)
#pragma unroll 1
        for (int l = 0; l < nl; l++) {
            const KLeaf<T>& L = Kd->leaf[l];
            const int ty = L.type;
            if (ty == L_PERIODIC) continue;
            double a0 = 0, a1 = 0, a2 = 0;
            if (ty == L_GAUSS) {  // p = (sigma, scale): g = (sc^2 r2 / sig^3 e, 2 sc e), e = exp(c1 r2)
                const T sig = L.p[0], sc = L.p[1], c1 = L.c1;
                const T k0 = sc * sc / (sig * sig * sig), k1 = T(2) * sc;
                each([&](auto cc) {
                    constexpr int x = decltype(cc)::value >> 2, reg = decltype(cc)::value & 3;
#pragma unroll
                    for (int y = 0; y < 4; y++) {
                        const T r2 = ar[x][y][reg], we = wt[x][y][reg] * exp(c1 * r2);
                        a0 += (double)(we * (k0 * r2));
                        a1 += (double)(we * k1);
                    }
                });
            } else if (ty == L_GAUSS_EXP) {  // p = (sigma, scale) in log space
                const T sig = L.p[0], sc = L.p[1];
                const T ke = T(-0.5) * exp(T(-2) * sig), m0 = exp(T(2) * sc - T(2) * sig), m1 = T(2) * exp(T(2) * sc);
                each([&](auto cc) {
                    constexpr int x = decltype(cc)::value >> 2, reg = decltype(cc)::value & 3;
#pragma unroll
                    for (int y = 0; y < 4; y++) {
                        const T r2 = ar[x][y][reg], we = wt[x][y][reg] * exp(ke * r2);
                        a0 += (double)(we * (m0 * r2));
                        a1 += (double)(we * m1);
                    }
                });
            } else {  // L_RQ, p = (scale, sigma, alpha)
                const T sc = L.p[0], sig = L.p[1], al = L.p[2];
                const T kq = T(0.5) / (sig * sig * al), k0 = T(2) * sc, k1 = sc * sc / (sig * sig * sig), k2 = sc * sc;
                each([&](auto cc) {
                    constexpr int x = decltype(cc)::value >> 2, reg = decltype(cc)::value & 3;
#pragma unroll
                    for (int y = 0; y < 4; y++) {
                        const T r2 = ar[x][y][reg], fq = fma(kq, r2, T(1)), lf = log(fq), inv = T(1) / fq;
                        const T wp = wt[x][y][reg] * exp(-al * lf);
                        a0 += (double)(wp * k0);
                        a1 += (double)(wp * (k1 * r2 * inv));
                        a2 += (double)(wp * (k2 * (kq * r2 * inv - lf)));
                    }
                });
            }
            flush(l, a0, a1, a2);
        }
    }
    if (NPER) {
        int lp = 0;
        for (int l = 0; l < nl; l++)
            if (Kd->leaf[l].type == L_PERIODIC) lp = l;
        const KLeaf<T>& L = Kd->leaf[lp];
        const T sc = L.p[0], sig = L.p[2], c1 = L.c1;
        if (R2) __syncthreads();  // the staging ring is reused
        tile_mma<T, 0, false, BKS, GPRX_PAIR_FEED>(ar, FU + (int64_t)Kr * nf + i0, nf, FV + (int64_t)Kr * nv_ + j0, nv_, Kp, Kp, smem, t);
        load_weights();
        double a0 = 0, a2 = 0;
        each([&](auto cc) {
            constexpr int x = decltype(cc)::value >> 2, reg = decltype(cc)::value & 3;
            const int64_t gj = gj_of(x, reg);
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const T sp = (!CROSS && gi_of(y) == gj) ? T(0) : clamp0(fma(T(-0.5), ar[x][y][reg], hd));
                T we = wt[x][y][reg] * exp(c1 * sp);
                // pinned here: sunk past the next product (to its use), S and the weights
                // stayed live across it and spilled
                asm volatile("" : "+v"(we));
                a0 += (double)we;
                a2 += (double)(we * sp);
                ar[x][y][reg] = we;
            }
        });
        __syncthreads();
        typename Tr::acc_t af[2][4];
        tile_mma<T, 0, false, BKS, GPRX_PAIR_FEED>(af, GU + i0, nf, GV + j0, nv_, Kf, Kf, smem, t);
        double a1 = 0;
        each([&](auto cc) {
            constexpr int x = decltype(cc)::value >> 2, reg = decltype(cc)::value & 3;
            const int64_t gj = gj_of(x, reg);
#pragma unroll
            for (int y = 0; y < 4; y++)
                a1 += (double)(ar[x][y][reg] * ((!CROSS && gi_of(y) == gj) ? T(0) : af[x][y][reg]));
        });
        // d/d(scale) = 2 sc e, d/db = -0.5 sc^2 e F / sigma^2, d/dsigma = sc^2 e S / sigma^3
        flush(lp, (double)(T(2) * sc) * a0, (double)(T(-0.5) * sc * sc / (sig * sig)) * a1,
              (double)(sc * sc / (sig * sig * sig)) * a2);
    }
    __syncthreads();
    if (t < MAX_LEAF * 3) {
        double v = 0;
#pragma unroll
        for (int ww = 0; ww < 8; ww++) v += sacc[ww * MAX_LEAF * 3 + t];
        part[(int64_t)blockIdx.x * MAX_LEAF * 3 + t] = v;
    }
}

// gout[p] = sum over tiles of part[tile][p], in tile order
__global__ void grad_reduce_kernel(const double* __restrict__ part, int64_t ntiles, double* __restrict__ gout) {
    __shared__ double red[256];
    const int p = blockIdx.x, t = threadIdx.x;
    double v = 0;
    for (int64_t b = t; b < ntiles; b += 256) v += part[b * MAX_LEAF * 3 + p];
    red[t] = v;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (t < o) red[t] += red[t + o];
        __syncthreads();
    }
    if (t == 0) gout[p] = red[0];
}

}  // namespace pr

template <typename T>
bool pairs_mma_supported(const KCanon<T>& K, int m) {
    if (K.nper > 1 || m > pr::PM) return false;
    for (int l = 0; l < K.nleaf; l++)
        if (K.leaf[l].type == L_WHITE) return false;
    return K.need_r2 || K.nper > 0;
}

// feature columns of one sample set (Kr + Kp operand columns + the squared norms)
template <typename T>
int64_t pairs_feature_cols(const KCanon<T>& K, int d) {
    return pr::kr_of(K, d) + pr::kp_of(K, d) + 1;
}

template <typename T>
void launch_pair_features(const KCanon<T>& K, const T* X, int64_t n, int d, const T* center, bool right, T* F,
                          int64_t np, hipStream_t s, int* flag) {
    const int Kr = pr::kr_of(K, d), Kp = pr::kp_of(K, d);
    hipLaunchKernelGGL(pr::features_kernel<T>, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, s, X, n, d, center,
                       K.nper ? K.b[0] : T(0), K.need_r2 ? 1 : 0, K.nper, right ? 1 : 0, F, np, Kr, Kp, flag);
}

template <typename T>
static size_t pairs_lds() {
    const size_t a = mm::gemm_lds<T>() + sizeof(T) * 4 * GT, b = sizeof(T) * 4 * GT * pr::PM;  // + norms, alpha (x2)
    return a > b ? a : b;
}

#define GPRX_PAIRS_DISPATCH(KERN, ...)                                                                  \
    do {                                                                                              \
        const size_t lds_ = pairs_lds<T>();                                                           \
        auto go = [&](auto kfn) {                                                                     \
            GPRX_HIP(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize,     \
                                         (int)lds_));                                                \
            hipLaunchKernelGGL(kfn, grid, dim3(mm::NT), lds_, s, __VA_ARGS__);                        \
        };                                                                                            \
        if (K.nper && K.need_r2) go(pr::KERN<T, 1, true>);                                            \
        else if (K.nper) go(pr::KERN<T, 1, false>);                                                   \
        else go(pr::KERN<T, 0, true>);                                                                \
    } while (0)

// Lower triangle of K(X, X) + sigma2 I (identity beyond n) into A, from the features FU, FV
// (nf rows, nf = npad: a multiple of 128 >= n).
template <typename T>
void launch_kbuild_mma(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, const T* FV, int64_t nf, int d, T* A,
                       int64_t ld, int64_t n, T sigma2, int* flag, hipStream_t s) {
    const int Kr = pr::kr_of(K, d), Kp = pr::kp_of(K, d);
    const int64_t nt = nf / GT;
    const dim3 grid((unsigned)(nt * (nt + 1) / 2));
    ProfScope ps(KC_BUILD, s, 2.0 * (double)GT * GT * (Kr + Kp) * nt * (nt + 1) / 2,
                 (double)sizeof(T) * (n * (double)d + (double)n * (n + 1) / 2));
    GPRX_PAIRS_DISPATCH(kbuild_mma_kernel, Kd, FU, FV, nf, Kr, Kp, T(0.5) * T(d), A, ld, n, sigma2, flag);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void launch_kcross_mma(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, int64_t nfu, int64_t na, const T* FV,
                       int64_t nfv, int64_t nb, int d, T* A, int64_t ld, int* flag, hipStream_t s, const T* Y,
                       T* kyp) {
    GPRX_REQUIRE(nfu % GT == 0 && nfv % GT == 0 && na <= nfu && nb <= nfv && ld >= nfu, GPRX_ERR_ARG,
                 "launch_kcross_mma: feature rows must be multiples of 128 covering the samples");
    const int Kr = pr::kr_of(K, d), Kp = pr::kp_of(K, d);
    const dim3 grid((unsigned)(nfu / GT), (unsigned)(nfv / GT));
    ProfScope ps(KC_BUILD, s, 2.0 * (double)nfu * nfv * (Kr + Kp), (double)sizeof(T) * (double)na * nb);
    GPRX_PAIRS_DISPATCH(kcross_mma_kernel, Kd, FU, nfu, na, FV, nfv, nb, Kr, Kp, T(0.5) * T(d), A, ld, flag, Y, kyp);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void launch_ky_reduce(const T* kyp, int64_t nfu, int nct, int64_t na, T alpha, T* S, int64_t lds, int64_t row0,
                      hipStream_t s) {
    if (na <= 0) return;
    hipLaunchKernelGGL(pr::ky_reduce_kernel<T>, dim3((unsigned)((na + 15) / 16)), dim3(256), 0, s, kyp, nfu, nct, na,
                       alpha, S, lds, row0);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
void launch_predict_mma(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, int64_t nfu, const T* FV, int64_t nfv,
                        int d, const T* alpha, int64_t n, int m, int64_t q, T* mean, hipStream_t s) {
    const int Kr = pr::kr_of(K, d), Kp = pr::kp_of(K, d);
    const dim3 grid((unsigned)(nfu / GT));
    ProfScope ps(KC_PREDICT, s, (double)q * n * (2.0 * d + 2.0 * m), (double)sizeof(T) * (double)(q + n) * d);
    GPRX_PAIRS_DISPATCH(predict_mma_kernel, Kd, FU, nfu, FV, nfv, Kr, Kp, T(0.5) * T(d), alpha, n, m, q, mean);
    GPRX_HIP(hipGetLastError());
}

// LML gradient trees: sum of Gaussian / GaussianExp / RQ / (one frequency) Periodic leaves
template <typename T>
bool pairs_grad_supported(const KCanon<T>& K) {
    if (!pairs_mma_supported<T>(K, 1) || !K.sum_leaves) return false;
    int nperleaf = 0;
    for (int l = 0; l < K.nleaf; l++) {
        const int ty = K.leaf[l].type;
        if (ty != L_GAUSS && ty != L_GAUSS_EXP && ty != L_RQ && ty != L_PERIODIC) return false;
        nperleaf += ty == L_PERIODIC;
    }
    return nperleaf <= 1;
}

template <typename T>
int64_t pairs_grad_feature_cols(const KCanon<T>& K, int d) {
    return K.nper ? pr::rup(4 * d, pr::KG) : 0;
}

// acc[3 l + q] = sum_{i >= j} w_ij d leaf_l / d p_q, from the features of launch_pair_features
// (FU, FV: nf rows) and grad features GU, GV (computed here); part: ntiles * 3 MAX_LEAF doubles
template <typename T>
void launch_lml_grad_mma(const KCanon<T>& K, const KCanon<T>* Kd, const T* X, int64_t n, int d, const T* FU,
                         const T* FV, T* GU, T* GV, int64_t nf, const T* alpha, const T* C, int64_t ldc, double* part,
                         double* acc, hipStream_t s, const uint64_t* ctab) {
    const int Kr = pr::kr_of(K, d), Kp = pr::kp_of(K, d), Kf = (int)pairs_grad_feature_cols(K, d);
    if (K.nper) {
        const dim3 g((unsigned)((nf + 255) / 256));
        hipLaunchKernelGGL(pr::grad_features_kernel<T>, g, dim3(256), 0, s, X, n, d, X, K.b[0], 0, GU, nf, Kf);
        hipLaunchKernelGGL(pr::grad_features_kernel<T>, g, dim3(256), 0, s, X, n, d, X, K.b[0], 1, GV, nf, Kf);
    }
    const int64_t nt = nf / GT, ntiles = nt * (nt + 1) / 2;
    const dim3 grid((unsigned)ntiles);
    ProfScope ps(KC_LML_GRAD, s, 2.0 * (double)GT * GT * (Kr + Kp + Kf) * ntiles,
                 (double)sizeof(T) * ((double)n * (n + 1) / 2 + (double)n * d));
    const size_t lds = mm::gemm_lds<T>() + sizeof(double) * 8 * MAX_LEAF * 3;
    auto go = [&](auto kfn) {
        GPRX_HIP(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(kfn, grid, dim3(mm::NT), lds, s, Kd, FU, FV, (const T*)GU, (const T*)GV, nf, Kr, Kp, Kf,
                           T(0.5) * T(d), alpha, C, ldc, n, part, ctab, nf, n, alpha);
    };
    if (K.nper && K.need_r2) go(pr::grad_mma_kernel<T, 1, true>);
    else if (K.nper) go(pr::grad_mma_kernel<T, 1, false>);
    else go(pr::grad_mma_kernel<T, 0, true>);
    hipLaunchKernelGGL(pr::grad_reduce_kernel, dim3(MAX_LEAF * 3), dim3(256), 0, s, (const double*)part, ntiles, acc);
    GPRX_HIP(hipGetLastError());
}

// Cross form: acc[3 l + q] = sum_{i < na, j < nb} (a_i b_j - C_ij) d leaf_l(xa_i, xb_j) / d p_q
// (no doubling, no diagonal).  FU: left features of Xa (nfu rows), FV: right features of Xb
// (nfv rows), both centred on `center`; GU, GV (nfu / nfv rows) are computed here.
template <typename T>
void launch_lml_grad_mma_cross(const KCanon<T>& K, const KCanon<T>* Kd, const T* Xa, int64_t na, const T* Xb,
                               int64_t nb, const T* center, int d, const T* FU, int64_t nfu, const T* FV, int64_t nfv,
                               T* GU, T* GV, const T* a, const T* b, const T* C, int64_t ldc, double* part, double* acc,
                               hipStream_t s) {
    GPRX_REQUIRE(nfu % GT == 0 && nfv % GT == 0 && na <= nfu && nb <= nfv && ldc >= nfu, GPRX_ERR_ARG,
                 "launch_lml_grad_mma_cross: feature rows must be multiples of 128 covering the samples");
    const int Kr = pr::kr_of(K, d), Kp = pr::kp_of(K, d), Kf = (int)pairs_grad_feature_cols(K, d);
    if (K.nper) {
        hipLaunchKernelGGL(pr::grad_features_kernel<T>, dim3((unsigned)((nfu + 255) / 256)), dim3(256), 0, s, Xa, na,
                           d, center, K.b[0], 0, GU, nfu, Kf);
        hipLaunchKernelGGL(pr::grad_features_kernel<T>, dim3((unsigned)((nfv + 255) / 256)), dim3(256), 0, s, Xb, nb,
                           d, center, K.b[0], 1, GV, nfv, Kf);
    }
    const int64_t ntiles = (nfu / GT) * (nfv / GT);
    if (ntiles == 0) {
        GPRX_HIP(hipMemsetAsync(acc, 0, sizeof(double) * MAX_LEAF * 3, s));
        return;
    }
    ProfScope ps(KC_LML_GRAD, s, 2.0 * (double)GT * GT * (Kr + Kp + Kf) * ntiles,
                 (double)sizeof(T) * ((double)na * nb + (double)(na + nb) * d));
    const size_t lds = mm::gemm_lds<T>() + sizeof(double) * 8 * MAX_LEAF * 3;
    auto go = [&](auto kfn) {
        GPRX_HIP(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
        hipLaunchKernelGGL(kfn, dim3((unsigned)ntiles), dim3(mm::NT), lds, s, Kd, FU, FV, (const T*)GU, (const T*)GV,
                           nfu, Kr, Kp, Kf, T(0.5) * T(d), a, C, ldc, na, part, (const uint64_t*)nullptr, nfv, nb, b);
    };
    if (K.nper && K.need_r2) go(pr::grad_mma_kernel<T, 1, true, true>);
    else if (K.nper) go(pr::grad_mma_kernel<T, 1, false, true>);
    else go(pr::grad_mma_kernel<T, 0, true, true>);
    hipLaunchKernelGGL(pr::grad_reduce_kernel, dim3(MAX_LEAF * 3), dim3(256), 0, s, (const double*)part, ntiles, acc);
    GPRX_HIP(hipGetLastError());
}

template <typename T>
TileBuild<T> pairs_tile_build(const KCanon<T>& K, const KCanon<T>* Kd, const T* FU, const T* FV, int64_t nf, int d,
                              int64_t n, T sigma2, int* flag) {
    TileBuild<T> b;
    b.Kd = Kd;
    b.FU = FU;
    b.FV = FV;
    b.nf = nf;
    b.Kr = pr::kr_of(K, d);
    b.Kp = pr::kp_of(K, d);
    b.hd = T(0.5) * T(d);
    b.sigma2 = sigma2;
    b.n = n;
    b.flag = flag;
    // as GPRX_PAIRS_DISPATCH.  0 (no fused build: the caller launches kbuild_mma_kernel) for
    // trees with products, which build_tile_sum does not separate, and for RationalQuadratic
    // leaves: the fused path carries exp-form leaves only, to keep the factorisation kernel
    // small (its code and register budget are shared with every other task type)
    bool expform = K.sum_leaves != 0;
    for (int l = 0; l < K.nleaf; l++)
        if (K.leaf[l].type != L_GAUSS && K.leaf[l].type != L_GAUSS_EXP && K.leaf[l].type != L_PERIODIC) expform = false;
    b.mode = !expform ? 0 : (K.nper && K.need_r2) ? 1 : (K.nper ? 3 : 2);
    return b;
}

#define GPRX_PAIRS_INST(T)                                                                                    \
    template bool pairs_grad_supported<T>(const KCanon<T>&);                                                  \
    template int64_t pairs_grad_feature_cols<T>(const KCanon<T>&, int);                                       \
    template void launch_lml_grad_mma_cross<T>(const KCanon<T>&, const KCanon<T>*, const T*, int64_t, const T*,  \
                                               int64_t, const T*, int, const T*, int64_t, const T*, int64_t, T*,  \
                                               T*, const T*, const T*, const T*, int64_t, double*, double*,        \
                                               hipStream_t);                                                      \
    template void launch_lml_grad_mma<T>(const KCanon<T>&, const KCanon<T>*, const T*, int64_t, int, const T*, \
                                         const T*, T*, T*, int64_t, const T*, const T*, int64_t, double*,     \
                                         double*, hipStream_t, const uint64_t*);                                \
    template TileBuild<T> pairs_tile_build<T>(const KCanon<T>&, const KCanon<T>*, const T*, const T*, int64_t, int, \
                                              int64_t, T, int*);                                              \
    template bool pairs_mma_supported<T>(const KCanon<T>&, int);                                              \
    template int64_t pairs_feature_cols<T>(const KCanon<T>&, int);                                            \
    template void launch_pair_features<T>(const KCanon<T>&, const T*, int64_t, int, const T*, bool, T*, int64_t, \
                                          hipStream_t, int*);                                                 \
    template void launch_kbuild_mma<T>(const KCanon<T>&, const KCanon<T>*, const T*, const T*, int64_t, int, T*,    \
                                       int64_t, int64_t, T, int*, hipStream_t);                               \
    template void launch_kcross_mma<T>(const KCanon<T>&, const KCanon<T>*, const T*, int64_t, int64_t, const T*,  \
                                       int64_t, int64_t, int, T*, int64_t, int*, hipStream_t, const T*, T*);   \
    template void launch_ky_reduce<T>(const T*, int64_t, int, int64_t, T, T*, int64_t, int64_t, hipStream_t);   \
    template void launch_predict_mma<T>(const KCanon<T>&, const KCanon<T>*, const T*, int64_t, const T*, int64_t, \
                                        int, const T*, int64_t, int, int64_t, T*, hipStream_t);
GPRX_PAIRS_INST(double)
GPRX_PAIRS_INST(float)
#undef GPRX_PAIRS_INST

}  // namespace gprx
