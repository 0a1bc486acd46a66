// k_mma.h — the 128x128 f64/f32 MFMA tile machinery shared by the tile-dataflow
// factorisation (k_ptiles.hip) and the pair-statistics kernels (k_pairs.hip).
//
// One 512-thread workgroup (8 waves of 64x32 outputs, v_mfma_f64_16x16x4f64 /
// v_mfma_f32_16x16x4f32) computes acc = A B^T for a 128x128 tile, A and B being 128-row
// column-major operand panels K deep.  Operands are staged by LDS-DMA (global_load_lds_dwordx4,
// no VGPRs) into a ring of NBUF stage buffers of BKS k-columns; loads run AHEAD stages ahead of
// the MFMAs and stay in flight across the per-stage barrier (raw s_barrier + counted vmcnt: a
// __syncthreads() would drain them, cdna_hip_programming.md §5 "Pipelining across barriers").
// One wave-instruction moves 64 x 16 B = 1 KiB = one 128-row f64 column (two f32 columns),
// written contiguously at a wave-uniform LDS base; columns (column pairs) are PAD apart.
// Accumulator layout: acc[x][y][reg] = C(row = 64 wr + 16 y + lr, col = 32 wc + 16 x +
// orow(lk, reg)) with w = wave, wr = w & 1, wc = w >> 1, lr = lane & 15, lk = lane >> 4.
#pragma once
#include "gprx_internal.h"

namespace gprx {
namespace mm {

constexpr int NT = 512;     // threads per workgroup
constexpr int PAD = 16;     // LDS row pad (elements)

// T_UPD2 (round 6): the update of two vertically adjacent tiles (i, j), (i + 1, j) over the same
// panels as one 256 x 128 product (tile_mma_tall): the single-GPU factorisation's paired chunks
enum { T_DIAGX = 0, T_TRSM = 1, T_UPD = 2, T_BUILD = 3, T_TPART = 4, T_UPD2 = 5 };
enum { C_TICKET = 0, C_ERR = 1, C_NCTL = 16 };  // control words at the head of the counter block

typedef double d4_t __attribute__((ext_vector_type(4)));
typedef float f4_t __attribute__((ext_vector_type(4)));
typedef double d2_t __attribute__((ext_vector_type(2)));

template <typename T>
struct Mfma;
template <>
struct Mfma<double> {
    typedef d4_t acc_t;
    typedef d2_t vec_t;
    static constexpr int VEC = 2;
    __device__ static inline acc_t mma(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    __device__ static inline int orow(int lk, int reg) { return lk + 4 * reg; }
};
template <>
struct Mfma<float> {
    typedef f4_t acc_t;
    typedef f4_t vec_t;
    static constexpr int VEC = 4;
    __device__ static inline acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    __device__ static inline int orow(int lk, int reg) { return 4 * lk + reg; }
};

// Operand staging: global_load_lds_dwordx4 (LDS-DMA, no VGPRs) into a ring of NBUF stage
// buffers of BKS k-columns; loads run 3 stages ahead of the MFMAs and stay in flight across
// the per-stage barrier (raw s_barrier + counted vmcnt: a __syncthreads() would drain them).
// One wave-instruction moves 64 x 16 B = 1 KiB = one 128-row f64 column (two f32 columns),
// written contiguously at a wave-uniform LDS base; columns (column pairs) are PAD apart.
#ifndef GPRX_PT_BKS
#define GPRX_PT_BKS 16
#define GPRX_PT_NBUF 4
#endif
constexpr int BKS = GPRX_PT_BKS;
constexpr int NBUF = GPRX_PT_NBUF;
constexpr int AHEAD = NBUF - 1;  // stages in flight ahead of the one being computed
// k-columns per stage of the factorisation's products by precision (the pair statistics keep
// BKS: their feature widths are multiples of 16).  f32 stages are twice as deep (the f64
// stage's LDS bytes, half the barriers per flop): C4's f32 factor 101.9 -> 98.6 ms, same-box
// A/B (profiles/r04f); GPRX_F32_BKS=16 builds the round-3 depth
// (GPRX_F32_BKS=64: two 139 KB ring buffers, one stage ahead -- probe 0.818 -> 0.836 of the f32
// bound, C4's factor only 101.7 -> 100.9 ms same box, profiles/r05yz; not the default: one
// stage of lead is thin for the sharded fit's window-fed operands)
#ifndef GPRX_F32_BKS
#define GPRX_F32_BKS 32
#endif
template <typename T>
struct BkOf {
    static constexpr int v = BKS;
};
template <>
struct BkOf<float> {
    static constexpr int v = GPRX_F32_BKS;
};

// tile_mma's operand feed by precision (scripts/mma_probe.hip decomposes the f64 stage: 4880
// cycles against the 4096-cycle MFMA bound, of which the per-stage barrier costs ~330 and the
// LDS-DMA refill ~400; profiles/r04q):
//   late: the stage barrier sits inside the stage's last k-step -- it publishes the NEXT stage,
//         whose first fragments are then read under this stage's remaining MFMAs, so the waves
//         do not drain at the stage boundary (the refill's lead is one stage shorter);
//   mid:  step kq+1's fragment reads are pinned after the first `mid` MFMAs of step kq (-1: read
//         ahead of all of them, where hipcc then issued them behind the MFMAs and waited on
//         them -- lgkmcnt(0), with an LDS-DMA pending -- before the next step's first MFMA).
// f64: late + mid 1 + spread refill (probe 0.839 -> 0.877 of the bound; C3 launch 26.45 ->
// 25.71 ms and the C5 syrk 2.47 -> 2.39 ms per launch with mid 2, same box, profiles/r04s; mid 1
// another 0.5% on both, r04ak); f32: all off
// (late + mid 2 cost C4's factor 3%: 100.8 -> 103.6 ms, r04q).
// GPRX_MMA_LATE / GPRX_MMA_MID / GPRX_MMA_SPREAD force a form for both (A/B builds).
#ifndef GPRX_PAIR_FEED
#define GPRX_PAIR_FEED 0
#endif
#ifndef GPRX_SHORT_FEED
#define GPRX_SHORT_FEED -1
#endif
template <typename T>
struct FeedOf {
#ifdef GPRX_MMA_LATE
    static constexpr bool late = GPRX_MMA_LATE != 0;
#else
    static constexpr bool late = sizeof(T) == 8;
#endif
#ifdef GPRX_MMA_MID
    static constexpr int mid = GPRX_MMA_MID;
#else
    static constexpr int mid = sizeof(T) == 8 ? 1 : -1;
#endif
    // late form: the refill's LDS-DMA issues one after each of the MFMAs that follow the
    // barrier, not in a burst after it (each issue holds its wave ~60 cycles; behind an MFMA
    // the pipe stays busy meanwhile): probe 0.860 -> 0.873, C3 launch 25.76 -> 25.71 ms
#ifdef GPRX_MMA_SPREAD
    static constexpr bool spread = GPRX_MMA_SPREAD != 0;
#else
    static constexpr bool spread = sizeof(T) == 8;
#endif
};

template <typename T, int BK = BkOf<T>::v>
struct Stage {
    static constexpr int E = 16 / sizeof(T);     // elements per lane per load
    static constexpr int LPC = GT / E;           // lanes per column
    static constexpr int CPI = 64 / LPC;         // columns per wave-instruction
    static constexpr int SRP = CPI * GT + PAD;   // LDS elements per instruction slot
    static constexpr int GRP = BK / CPI;         // instructions per operand per stage
    static constexpr int IPW = 2 * GRP / 8;      // instructions per wave per stage
    static constexpr int STG = 2 * GRP * SRP;    // elements per stage buffer (A slots, then B)
    static constexpr int NB = BK > 32 ? 2 : NBUF;  // ring buffers (deeper stages: fewer of them)
    static constexpr int AH = NB - 1;              // stages in flight ahead of the one computed
    // f32 (two columns per instruction): the second column of a pair is stored rotated by ROT
    // rows.  The fragment reads are ds_read_b32 (banks (a/4) mod 32, lanes 0-31 one group):
    // lanes with lk = 0 and lk = 1 read k-columns kr and kr + 1 of one pair, 128 words apart --
    // the same banks, a 2-way conflict on every f32 fragment read; rotated, the two halves of the
    // group land 16 banks apart
    // (the factorisation's 32-deep f32 stages keep the pair adjacent instead: tile_mma reads
    // both columns with ONE ds_read2_b32 -- PAIRED below -- and the pair's two k-columns are
    // then read by the same lane, in different MFMA steps)
    static constexpr int ROT = (CPI == 2 && BK < 32) ? 16 : 0;
    // row of the operand column that lane `lane`'s 16-B load brings (its LDS position is fixed)
    __device__ static inline int src_row(int lane) {
        const int lcol = lane / LPC, lrow = (lane % LPC) * E;
        return ROT ? (lrow + GT - ROT * lcol) & (GT - 1) : lrow;
    }
    // LDS element of row r of k-column kr of a stage's operand
    __device__ static inline int at(int kr, int r) {
        const int c = kr % CPI;
        return (kr / CPI) * SRP + c * GT + (ROT ? ((r + ROT * c) & (GT - 1)) : r);
    }
};

template <typename T>
constexpr size_t gemm_lds() {  // (the larger of the two stage depths a launch may use)
    return sizeof(T) * (Stage<T>::NB * Stage<T>::STG > NBUF * Stage<T, BKS>::STG ? Stage<T>::NB * Stage<T>::STG
                                                                                  : NBUF * Stage<T, BKS>::STG);
}

template <typename T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_store ... sc1
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Output block (wr, wc) of wave w (64 x 32 outputs at rows 64 wr, columns 32 wc).  Waves w and
// w + 4 share a SIMD (and its MFMA unit), so a shape whose blocks carry unequal work is mapped
// with each SIMD's pair summing to the same work:
//   MAP 0: wr = w & 1, wc = w >> 1 (every block a full 128-deep product);
//   MAP 1: triangular B (TRSM, k < 32 (wc + 1)): pairs take wc {0, 3} or {1, 2} -- 160 of the
//          512 k-columns per SIMD instead of 128/128/192/192;
//   MAP 2: lower (diagonal) tile, 16 x 16 tiles strictly above the diagonal skipped: per SIMD
//          8/8/10/10 of the 36 live tiles instead of 7/15/3/11 (or two full waves).
template <int MAP>
__device__ __forceinline__ void wave_block(int w, int& wr, int& wc) {
    if (MAP == 1) {
        wr = w & 1;
        wc = (w < 4) ? (w >> 1) : 3 - ((w - 4) >> 1);
    } else if (MAP == 2) {
        // w: 0 (1,0)  1 (1,1)  2 (0,0)  3 (1,2)  4 (0,2)  5 (0,3)  6 (1,3)  7 (0,1)
        constexpr unsigned RW = 0b01001011u;          // wr bit per wave
        constexpr unsigned CW = 0x13322010u;          // 4-bit wc per wave: 0,1,0,2,2,3,3,1
        wr = (RW >> w) & 1;
        wc = (CW >> (4 * w)) & 15;
    } else {
        wr = w & 1;
        wc = w >> 1;
    }
}

// acc = A B^T over K (multiple of BKS); this wave multiplies only the first kact k-columns
// (a multiple of BKS: 0 = idle, K = all; the rest of B is zero for it), but every wave takes
// part in the staging and the barriers of all K.  A, B: 128 rows x K, column-major (lda,
// ldb), 16-B aligned.
// Bpan (optional): B given per 128-column panel -- column c of B at Bpan[c / 128] + (c % 128)
// ldb (the distributed factorisation's received tiles: one packed 128 x 128 tile per panel,
// ldb = 128, each panel in its own receive buffer).
// ACC: acc += A B^T (acc is not cleared: consecutive K ranges into one accumulator).
// FEED: -1 the precision's form (FeedOf), 0 the early barrier with reads ahead of each step
// (the pair statistics' K = 32..96 products: the late form made the stand-alone build 4% slower)
template <typename T, int MAP = 0, bool ACC = false, int BK = BkOf<T>::v, int FEED = -1>
__device__ __forceinline__ void tile_mma(typename Mfma<T>::acc_t (&acc)[2][4], const T* __restrict__ A, int64_t lda,
                                         const T* __restrict__ B, int64_t ldb, int K, int kact, T* smem,
                                         const int t, const uint64_t* Bpan = nullptr) {
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    typedef Stage<T, BK> S;
    const int lane = t & 63, w = t >> 6;
    int wr, wc;
    wave_block<MAP>(w, wr, wc);
    const int lr = lane & 15, lk = lane >> 4;
    const int lcol = lane / S::LPC, lrow = S::src_row(lane);
    // Bpan: the K / 128 <= 64 panel addresses, lane l holding panel l's, loaded ONCE here.  (A
    // load of the address inside issue() made every stage's issue wait -- readfirstlane needs
    // the value, and vmcnt counts in order -- for all the staging loads still in flight: the
    // window-fed updates of the sharded fit ran 68% slower per panel than the local ones.)
    uint32_t bp_lo = 0, bp_hi = 0;
    if (Bpan) {
        const int npan = (K + GT - 1) / GT;
        const uint64_t v = (lane < npan) ? Bpan[lane] : 0ull;
        bp_lo = (uint32_t)v;
        bp_hi = (uint32_t)(v >> 32);
    }

    auto issue_u = [&](int st, int u) {
        T* buf = smem + (st % S::NB) * S::STG;
        {
            const int g = w * S::IPW + u;  // wave-uniform slot: A 0..GRP-1, B GRP..2GRP-1
            const bool isB = g >= S::GRP;
            const int gg = isB ? g - S::GRP : g;
            const int64_t col = (int64_t)st * BK + gg * S::CPI + lcol;
            const T* src;
            if (isB && Bpan) {  // the stage's 16 columns lie in one 128-column panel
                // (addresses as integers: a pointer-to-pointer operand crashed hipcc 7.2)
                const int pn = (st * BK) >> 7;
                const uint32_t lo = __builtin_amdgcn_readlane(bp_lo, pn);
                const uint32_t hi = __builtin_amdgcn_readlane(bp_hi, pn);
                const T* pb = reinterpret_cast<const T*>(((uint64_t)hi << 32) | lo);
                src = pb + lrow + (col & (GT - 1)) * ldb;
            } else {
                src = isB ? (B + lrow + col * ldb) : (A + lrow + col * lda);
            }
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (__attribute__((address_space(3))) void*)(buf + g * S::SRP), 16, 0, 0);
        }
    };
    auto issue = [&](int st) {
#pragma unroll
        for (int u = 0; u < S::IPW; u++) issue_u(st, u);
    };

    if (!ACC) {
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 4; y++) acc[x][y] = acc_t{0};
    }

    const int nst = K / BK;
#pragma unroll
    for (int p = 0; p < S::AH; p++)
        if (p < nst) issue(p);
    // this wave's loads of stage st have landed (later stages may stay in flight), and every
    // wave's, and every wave is done reading the buffer refilled next; then the refill
    auto stage_sync = [&](int st) {
        const int ahead = nst - 1 - st;
        if (S::AH >= 3 && ahead >= 2) wait_vm<(S::AH >= 3 ? 2 : 0) * S::IPW>();
        else if (S::AH >= 2 && ahead >= 1) wait_vm<S::IPW>();
        else wait_vm<0>();
        // (Reading the next stage's first fragments before this barrier, so the MFMAs start
        // right after it, measured +0.5% alone but cost 3% inside the factorisation: it
        // shortens the load lead to two stages.)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (st + S::AH < nst) issue(st + S::AH);
    };
    // The MFMA stages and the idle ones (above the diagonal of a diagonal tile, beyond the
    // triangle of a triangular B) are loops of their own with the same barriers: with a
    // wave-uniform test inside one loop, the accumulators merged from two paths every stage
    // (64 register moves, and a wait for the last MFMAs, per stage).
    // (rounded up: kact = 32 (wc + 1) for a triangular B, whose columns beyond it are stored zeros)
    const int nmf = (__builtin_amdgcn_readfirstlane(kact < K ? kact : K) + BK - 1) / BK;
    constexpr bool LATE = FEED < 0 && FeedOf<T>::late;
    constexpr int MID = FEED < 0 ? FeedOf<T>::mid : -1;
    if constexpr (LATE) {
        // late barrier B_st inside stage st's last k-step (after MID of its MFMAs): stage
        // st + 1 has landed for every wave and every wave is past stage st - 1, whose buffer takes
        // stage st + AH; stage st + 1's first fragments are read right after it, under the rest of
        // stage st's MFMAs
        static_assert(S::AH >= 2 && MID >= 0, "late barrier: two stages ahead, mid-step reads");
        constexpr bool SPREAD = FeedOf<T>::spread;
        static_assert(!SPREAD || MID + S::IPW < 8, "spread refill: a DMA behind each MFMA after the barrier");
        auto late_sync = [&](int st, bool refill) {
            if (S::AH >= 3 && nst - 2 - st >= 1) wait_vm<(S::AH >= 3 ? 1 : 0) * S::IPW>();
            else wait_vm<0>();
            __builtin_amdgcn_s_barrier();
            if (refill && st + S::AH < nst) issue(st + S::AH);
        };
        if (nst > 0) {  // stage 0 visible
            if (S::AH >= 3 && nst >= 3) wait_vm<(S::AH >= 3 ? 2 : 0) * S::IPW>();
            else if (S::AH >= 2 && nst >= 2) wait_vm<S::IPW>();
            else wait_vm<0>();
            __builtin_amdgcn_s_barrier();
        }
        {
            const T* a0 = smem;
            const T* b0 = smem + S::GRP * S::SRP;
            T fa[2][4], fb[2][2];
            auto frag = [&](int st, int kq, int r) {
                const T* a = a0 + (st % S::NB) * S::STG;
                const T* b = b0 + (st % S::NB) * S::STG;
                const int kr = kq * 4 + lk;
#pragma unroll
                for (int x = 0; x < 2; x++) fb[r][x] = b[S::at(kr, wc * 32 + x * 16 + lr)];
#pragma unroll
                for (int y = 0; y < 4; y++) fa[r][y] = a[S::at(kr, wr * 64 + y * 16 + lr)];
            };
            if (nmf > 0) frag(0, 0, 0);
            constexpr int KQ = BK / 4;
            static_assert(KQ % 2 == 0, "late barrier: an even number of k-steps per stage");
#pragma nounroll
            for (int st = 0; st < nmf; st++) {
#pragma unroll
                for (int kq = 0; kq < KQ; kq++) {
                    int m = 0;
#pragma unroll
                    for (int x = 0; x < 2; x++)
#pragma unroll
                        for (int y = 0; y < 4; y++) {
                            if (m == MID) {
                                __builtin_amdgcn_sched_barrier(0);
                                if (kq + 1 < KQ) {
                                    frag(st, kq + 1, (kq + 1) & 1);
                                } else {
                                    late_sync(st, !SPREAD);
                                    if (st + 1 < nmf) frag(st + 1, 0, 0);
                                }
                                __builtin_amdgcn_sched_barrier(0);
                            }
                            if (MAP != 2 || 4 * wr + y >= 2 * wc + x)
                                acc[x][y] = Tr::mma(fb[kq & 1][x], fa[kq & 1][y], acc[x][y]);
                            if (SPREAD && kq == KQ - 1 && m > MID && m - MID - 1 < S::IPW) {
                                __builtin_amdgcn_sched_barrier(0);
                                if (st + S::AH < nst) issue_u(st + S::AH, m - MID - 1);
                                __builtin_amdgcn_sched_barrier(0);
                            }
                            m++;
                        }
                }
            }
        }
#pragma nounroll
        for (int st = nmf; st < nst; st++) late_sync(st, true);
    } else {
        int st0 = 0;
        {
            const T* a0 = smem;
            const T* b0 = smem + S::GRP * S::SRP;
#pragma nounroll
            for (int st = 0; st < nmf; st++) {
                stage_sync(st);
                // fragments of step kq+1 are read while the MFMAs of step kq run
                const T* a = a0 + (st % S::NB) * S::STG;
                const T* b = b0 + (st % S::NB) * S::STG;
                T fa[2][4], fb[2][2];
                auto frag = [&](int kq, int r) {
                    const int kr = kq * 4 + lk;
#pragma unroll
                    for (int x = 0; x < 2; x++) fb[r][x] = b[S::at(kr, wc * 32 + x * 16 + lr)];
#pragma unroll
                    for (int y = 0; y < 4; y++) fa[r][y] = a[S::at(kr, wr * 64 + y * 16 + lr)];
                };
                constexpr bool PAIRED = sizeof(T) == 4 && BK >= 32 && S::CPI == 2 && S::ROT == 0;
                if constexpr (PAIRED) {
                    // f32, 32-deep stages: k-step 2 j + h takes the k-columns 2 (4 j + lk) + h, so a
                    // lane's two operands of steps 2j, 2j + 1 are the two columns of ONE DMA pair
                    // (GT floats apart in LDS): one ds_read2_b32 per operand fragment for two MFMA
                    // steps -- half the fragment-read instructions of the 4-consecutive-column
                    // order (the stage's 32 columns are summed in another order)
                    T pa[2][2][4], pb[2][2][2];  // [buffer][h][.]
                    auto frag2 = [&](int j, int r) {
                        const int slot = 4 * j + lk;
                        const T* ac = a + slot * S::SRP;
                        const T* bc = b + slot * S::SRP;
#pragma unroll
                        for (int x = 0; x < 2; x++) {
                            const int row = wc * 32 + x * 16 + lr;
                            pb[r][0][x] = bc[row];
                            pb[r][1][x] = bc[GT + row];
                        }
#pragma unroll
                        for (int y = 0; y < 4; y++) {
                            const int row = wr * 64 + y * 16 + lr;
                            pa[r][0][y] = ac[row];
                            pa[r][1][y] = ac[GT + row];
                        }
                    };
                    frag2(0, 0);
#pragma unroll
                    for (int j = 0; j < BK / 8; j++) {
                        if (j + 1 < BK / 8) frag2(j + 1, (j + 1) & 1);
                        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                        for (int h = 0; h < 2; h++)
#pragma unroll
                            for (int x = 0; x < 2; x++)
#pragma unroll
                                for (int y = 0; y < 4; y++)
                                    if (MAP != 2 || 4 * wr + y >= 2 * wc + x)
                                        acc[x][y] = Tr::mma(pb[j & 1][h][x], pa[j & 1][h][y], acc[x][y]);
                    }
                    continue;
                }
                frag(0, 0);
                if constexpr (MID < 0) {
#pragma unroll
                    for (int kq = 0; kq < BK / 4; kq++) {
                        if (kq + 1 < BK / 4) frag(kq + 1, (kq + 1) & 1);
                        __builtin_amdgcn_sched_barrier(0);  // keep those reads ahead of these MFMAs
#pragma unroll
                        for (int x = 0; x < 2; x++)
#pragma unroll
                            for (int y = 0; y < 4; y++)
                                if (MAP != 2 || 4 * wr + y >= 2 * wc + x)  // (MAP 2: wave-uniform tile skip)
                                    acc[x][y] = Tr::mma(fb[kq & 1][x], fa[kq & 1][y], acc[x][y]);
                    }
                } else {
                    // step kq+1's fragment reads pinned after the first MID MFMAs of step kq
#pragma unroll
                    for (int kq = 0; kq < BK / 4; kq++) {
                        int m = 0;
#pragma unroll
                        for (int x = 0; x < 2; x++)
#pragma unroll
                            for (int y = 0; y < 4; y++) {
                                if (m == MID) {
                                    __builtin_amdgcn_sched_barrier(0);
                                    if (kq + 1 < BK / 4) frag(kq + 1, (kq + 1) & 1);
                                    __builtin_amdgcn_sched_barrier(0);
                                }
                                if (MAP != 2 || 4 * wr + y >= 2 * wc + x)  // (MAP 2: wave-uniform tile skip)
                                    acc[x][y] = Tr::mma(fb[kq & 1][x], fa[kq & 1][y], acc[x][y]);
                                m++;
                            }
                    }
                }
            }
            st0 = nmf;
        }
#pragma nounroll
        for (int st = st0; st < nst; st++) stage_sync(st);
    }
}

// acc = A B^T for a lower-triangular B (128 x 128: B[c][k] = 0 for k > c, stored zeros) -- the
// TRSM task's L_ik = A_ik Linv_k^T -- with the work even across the waves in EVERY stage.  Wave w
// owns output rows 16 w .. 16 w + 15 across all 128 columns (eight 16-column groups g, acc[g >>
// 2][g & 3]), so at stage st each wave multiplies exactly the groups the triangle leaves live
// (16 g + 15 >= st BK): 36 of the full product's 64 group-stages for f64.  tile_mma's MAP 1
// balances the SIMDs' totals but not each stage -- the stage barriers hold every wave to the
// busiest, and its TRSM took 16 us against 15.4 us for a full update panel (the C3 fit trace,
// profiles/r06fb_pt_trace_fit16384.json).  9 fragment reads per 8 MFMAs (MAP 1: 6); stages
// unrolled (K = 128), so the live groups are compile-time.  The in-place call (C = A) is safe:
// A comes through the staging ring, and the stores follow the last stage.
// acc[x][y][reg] = C(row = 16 w + lr, col = 16 (4 x + y) + orow(lk, reg)).
template <typename T>
__device__ __forceinline__ void tile_mma_trirows(typename Mfma<T>::acc_t (&acc)[2][4], const T* __restrict__ A,
                                                 int64_t lda, const T* __restrict__ B, int64_t ldb, T* smem,
                                                 const int t) {
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    constexpr int BK = BkOf<T>::v;
    typedef Stage<T, BK> S;
    constexpr int NST = GT / BK;
    const int lane = t & 63, w = t >> 6;
    const int lr = lane & 15, lk = lane >> 4;
    const int lcol = lane / S::LPC, lrow = S::src_row(lane);
    auto issue = [&](int st) {
        T* buf = smem + (st % S::NB) * S::STG;
#pragma unroll
        for (int u = 0; u < S::IPW; u++) {
            const int g = w * S::IPW + u;
            const bool isB = g >= S::GRP;
            const int gg = isB ? g - S::GRP : g;
            const int64_t col = (int64_t)st * BK + gg * S::CPI + lcol;
            const T* src = isB ? (B + lrow + col * ldb) : (A + lrow + col * lda);
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (__attribute__((address_space(3))) void*)(buf + g * S::SRP), 16, 0, 0);
        }
    };
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 4; y++) acc[x][y] = acc_t{0};
#pragma unroll
    for (int p = 0; p < S::AH; p++)
        if (p < NST) issue(p);
    auto stage = [&](auto stc) {
        constexpr int st = decltype(stc)::value;
        constexpr int ahead = NST - 1 - st;
        if constexpr (S::AH >= 3 && ahead >= 2) wait_vm<2 * S::IPW>();
        else if constexpr (S::AH >= 2 && ahead >= 1) wait_vm<S::IPW>();
        else wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if constexpr (st + S::AH < NST) issue(st + S::AH);
        constexpr int G0 = (st * BK) / 16;  // first live column group
        const T* a = smem + (st % S::NB) * S::STG;
        const T* b = a + S::GRP * S::SRP;
        T fa[2], fb[2][8];
        auto frag = [&](int kq, int r) {
            const int kr = kq * 4 + lk;
            fa[r] = a[S::at(kr, 16 * w + lr)];
#pragma unroll
            for (int g = G0; g < 8; g++) fb[r][g] = b[S::at(kr, 16 * g + lr)];
        };
        frag(0, 0);
#pragma unroll
        for (int kq = 0; kq < BK / 4; kq++) {
            if (kq + 1 < BK / 4) frag(kq + 1, (kq + 1) & 1);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int g = G0; g < 8; g++) acc[g >> 2][g & 3] = Tr::mma(fb[kq & 1][g], fa[kq & 1], acc[g >> 2][g & 3]);
        }
    };
    static_assert(NST <= 8, "trirows: at most 8 stages");
    stage(std::integral_constant<int, 0>{});
    if constexpr (NST > 1) stage(std::integral_constant<int, (NST > 1 ? 1 : 0)>{});
    if constexpr (NST > 2) stage(std::integral_constant<int, (NST > 2 ? 2 : 0)>{});
    if constexpr (NST > 3) stage(std::integral_constant<int, (NST > 3 ? 3 : 0)>{});
    if constexpr (NST > 4) stage(std::integral_constant<int, (NST > 4 ? 4 : 0)>{});
    if constexpr (NST > 5) stage(std::integral_constant<int, (NST > 5 ? 5 : 0)>{});
    if constexpr (NST > 6) stage(std::integral_constant<int, (NST > 6 ? 6 : 0)>{});
    if constexpr (NST > 7) stage(std::integral_constant<int, (NST > 7 ? 7 : 0)>{});
}

// 256 x 128 output tile (A: 256 rows, B: 128 rows), for stand-alone kernels only: 128
// accumulator registers, which the factorisation's task loop (at 256 VGPRs) cannot hold.  The 8
// waves take 4 x 2 blocks of 64 x 64: 16 MFMAs per k-step from 8 fragment reads (the 128 x 128
// tile: 8 MFMAs from 6), and a stage's DMAs bring 384 rows' columns for twice the flops (the 128
// tile: 256).  Two ring buffers of three operand groups (A rows 0-127, A rows 128-255, B): a
// stage is 2 x 64 MFMAs per SIMD (8192 cycles f64), time enough for the next stage's loads,
// issued right after the stage barrier.  Step kq+1's fragments are read after MID MFMAs of step
// kq.  Probe (scripts/mma_probe.hip ... tall): f64 0.901 of the MFMA bound against 0.877 for the
// 128 x 128 tile (profiles/r05u).
template <typename T>
constexpr size_t tall_lds() {
    return sizeof(T) * 2 * 3 * Stage<T>::GRP * Stage<T>::SRP;
}
// Csub (optional): acc = A B^T - C for the 256 x 128 tile C (ldc) -- C is read in four column
// chunks of 16 values per lane, chunk c issued at stage c right after that stage's DMAs and
// subtracted at stage c + 1 (after the stage's vmcnt wait), so its latency hides under the
// MFMAs instead of holding the first one (the factorisation's paired updates, which have no
// registers to prefetch the whole C tile beside their 128 accumulators)
template <typename T, int MID = 1>
__device__ __forceinline__ void tile_mma_tall(typename Mfma<T>::acc_t (&acc)[4][4], const T* __restrict__ A,
                                              int64_t lda, const T* __restrict__ B, int64_t ldb, int K, T* smem,
                                              const int t, const T* __restrict__ Csub = nullptr, int64_t ldc = 0) {
    typedef Mfma<T> Tr;
    typedef Stage<T> S;
    constexpr int BK = BkOf<T>::v;
    static_assert(S::ROT == 0, "tall tile: unrotated staging");
    constexpr int GR3 = 3 * S::GRP, IPW3 = GR3 / 8, STG3 = GR3 * S::SRP;
    static_assert(GR3 % 8 == 0, "tall tile: whole DMA instructions per wave");
    const int lane = t & 63, w = t >> 6;
    const int wr = w & 3, wc = w >> 2, lr = lane & 15, lk = lane >> 4;
    const int lcol = lane / S::LPC, lrow = S::src_row(lane);
    auto issue = [&](int st) {
        T* buf = smem + (st & 1) * STG3;
#pragma unroll
        for (int u = 0; u < IPW3; u++) {
            const int g = w * IPW3 + u, op = g / S::GRP, gg = g - op * S::GRP;  // op 0, 1: A halves, 2: B
            const int64_t col = (int64_t)st * BK + gg * S::CPI + lcol;
            const T* src = (op == 2) ? (B + lrow + col * ldb) : (A + (int64_t)op * GT + lrow + col * lda);
            __builtin_amdgcn_global_load_lds((const void*)src,
                                             (__attribute__((address_space(3))) void*)(buf + g * S::SRP), 16, 0, 0);
        }
    };
#pragma unroll
    for (int x = 0; x < 4; x++)
#pragma unroll
        for (int y = 0; y < 4; y++) acc[x][y] = typename Tr::acc_t{0};
    // C chunk c: this lane's 16 values of columns 64 wc + 16 c + orow(lk, reg), rows 64 wr + 16 y + lr
    T cb[4][4];
    auto cload = [&](int c) {
#pragma unroll
        for (int reg = 0; reg < 4; reg++) {
            const T* ccol = Csub + (int64_t)(64 * wc + 16 * c + Tr::orow(lk, reg)) * ldc + 64 * wr + lr;
#pragma unroll
            for (int y = 0; y < 4; y++) cb[y][reg] = ccol[16 * y];
        }
    };
    auto csub = [&](auto xc) {  // (static chunk index: the accumulators stay register-indexed)
        constexpr int x = decltype(xc)::value;
#pragma unroll
        for (int y = 0; y < 4; y++)
#pragma unroll
            for (int reg = 0; reg < 4; reg++) acc[x][y][reg] -= cb[y][reg];
    };
    const int nst = K / BK;
    if (nst > 0) issue(0);
    const T* ab = smem + (wr >> 1) * S::GRP * S::SRP;  // this wave's half of A
    const T* bb = smem + 2 * S::GRP * S::SRP;
    const int ar = 64 * (wr & 1);
    T fa[2][4], fb[2][4];
    // one stage; CP (compile time) >= 0: the C chunk phase of stages 0..4 (subtract chunk CP - 1,
    // load chunk CP) -- the first five stages are peeled so every accumulator index stays static
    // (a run-time chunk index put the accumulators in scratch)
    // SPREAD (f64, FeedOf::spread): the next stage's DMAs go out one behind each of the stage's
    // first MFMAs instead of in a burst after the barrier, which held both waves of a SIMD (~60
    // cycles an instruction) while its MFMA pipe idled
    constexpr bool SPREAD = FeedOf<T>::spread && MID + IPW3 + 1 <= 16;
    auto issue_u = [&](int st, int u) {
        T* buf = smem + (st & 1) * STG3;
        const int g = w * IPW3 + u, op = g / S::GRP, gg = g - op * S::GRP;
        const int64_t col = (int64_t)st * BK + gg * S::CPI + lcol;
        const T* src = (op == 2) ? (B + lrow + col * ldb) : (A + (int64_t)op * GT + lrow + col * lda);
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(buf + g * S::SRP),
                                         16, 0, 0);
    };
    auto stage = [&](int st, auto cp) {
        constexpr int CP = decltype(cp)::value;
        wait_vm<0>();  // this wave's loads of stage st (issued a stage ago), and C chunk CP - 1
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // every wave's; every wave done with the other buffer
        if (!SPREAD && st + 1 < nst) issue(st + 1);
        const bool more = st + 1 < nst;
        if constexpr (CP >= 1) {
            if (Csub) csub(std::integral_constant<int, CP - 1>{});
        }
        if constexpr (CP >= 0 && CP < 4) {
            if (Csub) cload(CP);
        }
        const T* a = ab + (st & 1) * STG3;
        const T* b = bb + (st & 1) * STG3;
        auto frag = [&](int kq, int r) {
            const int kr = kq * 4 + lk;
#pragma unroll
            for (int x = 0; x < 4; x++) fb[r][x] = b[S::at(kr, 64 * wc + 16 * x + lr)];
#pragma unroll
            for (int y = 0; y < 4; y++) fa[r][y] = a[S::at(kr, ar + 16 * y + lr)];
        };
        frag(0, 0);
#pragma unroll
        for (int kq = 0; kq < BK / 4; kq++) {
            int m = 0;
#pragma unroll
            for (int x = 0; x < 4; x++)
#pragma unroll
                for (int y = 0; y < 4; y++) {
                    if (m == MID) {
                        __builtin_amdgcn_sched_barrier(0);
                        if (kq + 1 < BK / 4) frag(kq + 1, (kq + 1) & 1);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    acc[x][y] = Tr::mma(fb[kq & 1][x], fa[kq & 1][y], acc[x][y]);
                    if (SPREAD && kq == 0 && m > MID && m - MID - 1 < IPW3) {
                        __builtin_amdgcn_sched_barrier(0);
                        if (more) issue_u(st + 1, m - MID - 1);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    m++;
                }
        }
    };
    if (Csub) {
        if (nst > 0) stage(0, std::integral_constant<int, 0>{});
        if (nst > 1) stage(1, std::integral_constant<int, 1>{});
        if (nst > 2) stage(2, std::integral_constant<int, 2>{});
        if (nst > 3) stage(3, std::integral_constant<int, 3>{});
        if (nst > 4) stage(4, std::integral_constant<int, 4>{});
#pragma nounroll
        for (int st = 5; st < nst; st++) stage(st, std::integral_constant<int, -1>{});
        if (nst < 5) {  // short products: the chunks not yet subtracted (nst >= 1: chunk nst - 1 is loaded)
            wait_vm<0>();
            auto tail = [&](auto xc) {
                constexpr int x = decltype(xc)::value;
                if (nst == x + 1) csub(xc);
                if (nst <= x) {
                    cload(x);
                    wait_vm<0>();
                    csub(xc);
                }
            };
            tail(std::integral_constant<int, 0>{});
            tail(std::integral_constant<int, 1>{});
            tail(std::integral_constant<int, 2>{});
            tail(std::integral_constant<int, 3>{});
        }
    } else {
#pragma nounroll
        for (int st = 0; st < nst; st++) stage(st, std::integral_constant<int, -1>{});
    }
}

// Two products over consecutive column ranges of the same operands in ONE pass of the
// staging ring: acc1 = A[:, 0:K1] B[:, 0:K1]^T, acc2 = A[:, K1:K1+K2] B[:, K1:K1+K2]^T (K1, K2
// multiples of BKS).  Two back-to-back tile_mma calls pay the ring's fill and drain twice
// and a barrier between them; the pair statistics of a periodic + r2 tree are such a pair
// (k_pairs.h: the r2 and periodic feature columns are adjacent).  Every wave multiplies.
template <typename T>
__device__ __forceinline__ void ring_issue(const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
                                           int st, T* smem, const int t) {
    typedef Stage<T, BKS> S;
    const int lane = t & 63, w = t >> 6;
    const int lcol = lane / S::LPC, lrow = S::src_row(lane);
    T* buf = smem + (st % NBUF) * S::STG;
#pragma unroll
    for (int u = 0; u < S::IPW; u++) {
        const int g = w * S::IPW + u;
        const bool isB = g >= S::GRP;
        const int gg = isB ? g - S::GRP : g;
        const int64_t col = (int64_t)st * BKS + gg * S::CPI + lcol;
        const T* src = isB ? (B + lrow + col * ldb) : (A + lrow + col * lda);
        __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(buf + g * S::SRP),
                                         16, 0, 0);
    }
}

template <typename T>
__device__ __forceinline__ void tile_mma2(typename Mfma<T>::acc_t (&acc1)[2][4], typename Mfma<T>::acc_t (&acc2)[2][4],
                                          const T* __restrict__ A, int64_t lda, const T* __restrict__ B, int64_t ldb,
                                          int K1, int K2, T* smem, const int t) {
    typedef Mfma<T> Tr;
    typedef typename Tr::acc_t acc_t;
    typedef Stage<T, BKS> S;
    const int lane = t & 63, w = t >> 6;
    const int wr = w & 1, wc = w >> 1;
    const int lr = lane & 15, lk = lane >> 4;
    auto issue = [&](int st) { ring_issue<T>(A, lda, B, ldb, st, smem, t); };
#pragma unroll
    for (int x = 0; x < 2; x++)
#pragma unroll
        for (int y = 0; y < 4; y++) {
            acc1[x][y] = acc_t{0};
            acc2[x][y] = acc_t{0};
        }
    const int nst1 = __builtin_amdgcn_readfirstlane(K1) / BKS;
    const int nst = nst1 + __builtin_amdgcn_readfirstlane(K2) / BKS;
#pragma unroll
    for (int p = 0; p < AHEAD; p++)
        if (p < nst) issue(p);
    auto stage_sync = [&](int st) {
        const int ahead = nst - 1 - st;
        if (AHEAD >= 3 && ahead >= 2) wait_vm<(AHEAD >= 3 ? 2 : 0) * S::IPW>();
        else if (AHEAD >= 2 && ahead >= 1) wait_vm<S::IPW>();
        else wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (st + AHEAD < nst) issue(st + AHEAD);
    };
    const T* a0 = smem;
    const T* b0 = smem + S::GRP * S::SRP;
    // one loop per accumulator set (a run-time choice inside one loop would merge them)
    auto stages = [&](acc_t(&acc)[2][4], int sbeg, int send) {
#pragma nounroll
        for (int st = sbeg; st < send; st++) {
            stage_sync(st);
            const T* a = a0 + (st % NBUF) * S::STG;
            const T* b = b0 + (st % NBUF) * S::STG;
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
    stages(acc1, 0, nst1);
    stages(acc2, nst1, nst);
}

}  // namespace mm
}  // namespace gprx
