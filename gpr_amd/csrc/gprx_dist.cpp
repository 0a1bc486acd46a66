// gprx_dist.cpp — the storage-sharded multi-GPU fit (north_star: "the N x N matrix shards
// row-block across the GPUs with a broadcast of the diagonal panel at each potrf step").
//
// Replaces the same reference step as the single-GPU fit -- GaussianProcess::Initialize ->
// ComputeRegressionVectors, kernel matrix + lapack::lu_invert + C Y (lib/GaussianProcess.cpp
// :118-130, 642-672; include/LAPACKUtils.h:38-56) -- for a matrix dealt over g ranks:
//
//   storage   row block i (128 rows) lives on rank (i / gb) mod g (groups of gb blocks dealt
//             cyclically; gb from the simulated makespan): N^2/g of the lower factor per rank,
//             plus the tiles of other ranks' rows it receives (each rank ends with the whole
//             factor, in tiles, so the solve runs locally everywhere)
//   compute   each rank runs the persistent tile-dataflow launch (k_ptiles.hip,
//             potrf_tiles_kernel<T, true>) over its own row blocks: covariance BUILD tasks,
//             DIAGX (the diagonal 128-block chain), TRSM and UPD tasks, in the order of a list
//             schedule simulated over all ranks (potrf_dist_schedule)
//   exchange  per diagonal step k two transport steps, issued by this host thread as the
//             device reports its pieces ready (host-visible flags the kernel stores):
//             bcast(k)  Linv_k, the inverse of the factored diagonal block, from its rank to
//                       all (RCCL ncclBroadcast over xGMI): the only exchange on the chain
//             panel(k)  every final tile L_ik (i > k) from its rank to every other rank, one
//                       message per (rank, peer) pair fused in an RCCL group: the full-mesh
//                       all-gather of the panel, off the chain
//             each followed by a stream write of a counter the kernel polls (uncached memory)
//   reduce    log det (each rank's diagonal blocks) and the non-finite / pivot flags: one
//             RCCL all-reduce each at the end
//
// A second transport runs g "virtual ranks" in one process on one GPU (gprx_ctx_create_virtual,
// include/gprx_dev.h): the same kernels, buffers and issue loop, with device copies in place
// of RCCL -- the distributed algorithm, exchange protocol and deadlock freedom testable on a
// single GPU (tests/test_gpu_dist.py).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "gprx_dist.h"

namespace gprx {

namespace {

template <typename T>
ncclDataType_t nccl_t();
template <>
ncclDataType_t nccl_t<double>() {
    return ncclFloat64;
}
template <>
ncclDataType_t nccl_t<float>() {
    return ncclFloat32;
}

void rccl_ok(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw Error{GPRX_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r)};
}

// one device allocation, optionally fine-grained / uncached
struct DMem {
    void* p = nullptr;
    size_t bytes = 0;
    unsigned flags = 0;
    void ensure(size_t b, unsigned fl = 0) {
        if (p && b <= bytes && fl == flags) return;
        release();
        if (b == 0) return;
        if (fl) GPRX_HIP(hipExtMallocWithFlags(&p, b, fl));
        else GPRX_HIP(hipMalloc(&p, b));
        bytes = b;
        flags = fl;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        bytes = 0;
    }
    template <typename U>
    U* as() const {
        return reinterpret_cast<U*>(p);
    }
    ~DMem() { release(); }
};

struct HMem {  // coherent host memory the device stores to (kernel -> issue loop)
    void* p = nullptr;
    size_t bytes = 0;
    void ensure(size_t b) {
        if (p && b <= bytes) return;
        release();
        GPRX_HIP(hipHostMalloc(&p, b, hipHostMallocCoherent | hipHostMallocMapped));
        bytes = b;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        bytes = 0;
    }
    unsigned* u() const { return reinterpret_cast<unsigned*>(p); }
    ~HMem() { release(); }
};

}  // namespace

// ---------------------------------------------------------------------------------------
// layout: which rank holds which tile, where the send slots and received tiles live
// ---------------------------------------------------------------------------------------
struct DistLayout {
    // Row block i (128 rows; i = nc is the label block) lives on rank (i / gb) mod g: groups
    // of gb consecutive blocks dealt cyclically.  gb > 1 keeps gb - 1 of every gb diagonal
    // steps on one rank (the chain DIAGX(k) -> DIAGX(k + 1) then needs no broadcast hop).
    int g = 1, gb = 1, nc = 0, nr = 0;
    std::vector<int> own, lidx;          // per row block: owner rank, index in its rows
    std::vector<std::vector<int>> rows;  // per rank: owned row blocks, ascending
    int owner(int i) const { return own[i]; }
    int loc(int i) const { return lidx[i]; }
    int nloc(int q) const { return (int)rows[q].size(); }
    int firstpos(int q, int b) const {  // index in rows[q] of the first row block > b
        return (int)(std::upper_bound(rows[q].begin(), rows[q].end(), b) - rows[q].begin());
    }
    int cnt(int q, int b) const { return nloc(q) - firstpos(q, b); }  // row blocks in (b, nr) on q
    int pos(int q, int i, int b) const { return lidx[i] - firstpos(q, b); }
    // send slot offsets (tiles) of rank q: panel b after all earlier panels
    std::vector<std::vector<int64_t>> soff;             // [q][b]
    std::vector<std::vector<std::vector<int64_t>>> roff;  // [r][b][q]: rank r's received chunk from q
    std::vector<int64_t> stot, rtot;
    void init(int g_, int gb_, int nc_, int nr_) {
        g = g_;
        gb = std::max(1, gb_);
        nc = nc_;
        nr = nr_;
        own.assign(nr, 0);
        lidx.assign(nr, 0);
        rows.assign(g, std::vector<int>());
        for (int i = 0; i < nr; i++) {
            own[i] = (i / gb) % g;
            lidx[i] = (int)rows[own[i]].size();
            rows[own[i]].push_back(i);
        }
        soff.assign(g, std::vector<int64_t>(nc + 1, 0));
        stot.assign(g, 0);
        for (int q = 0; q < g; q++) {
            int64_t o = 0;
            for (int b = 0; b < nc; b++) {
                soff[q][b] = o;
                o += cnt(q, b);
            }
            soff[q][nc] = o;
            stot[q] = o;
        }
        roff.assign(g, std::vector<std::vector<int64_t>>(nc, std::vector<int64_t>(g, -1)));
        rtot.assign(g, 0);
        for (int r = 0; r < g; r++) {
            int64_t o = 0;
            for (int b = 0; b < nc; b++)
                for (int q = 0; q < g; q++) {
                    if (q == r) continue;
                    roff[r][b][q] = o;
                    o += cnt(q, b);
                }
            rtot[r] = o;
        }
    }
};

// one rank's buffers and launch state
template <typename T>
struct DistRank {
    int r = 0;
    hipStream_t s = nullptr;  // compute stream
    bool own_stream = false;
    DMem A, Linv, send, recv, ctr, info, flag, pd, loc, tptr, sptr, drecv, tiles, tld, red, alpha, tab, list, trace;
    HMem hdiag, hslot, dbg;
    std::vector<int4> hlist;
    int64_t ld = 0;
    int ntasks = 0;
    hipEvent_t done = nullptr;
    hipEvent_t t0 = nullptr, t1 = nullptr, t2 = nullptr;  // launch start / end, back-solve end
    ~DistRank() {
        if (done) (void)hipEventDestroy(done);
        if (t0) (void)hipEventDestroy(t0);
        if (t1) (void)hipEventDestroy(t1);
        if (t2) (void)hipEventDestroy(t2);
        if (own_stream && s) (void)hipStreamDestroy(s);
    }
};

struct DistEngineBase {
    virtual ~DistEngineBase() {}
};

template <typename T>
struct DistEngine : DistEngineBase {
    int g = 1;
    bool virt = false;
    int device = 0;
    std::vector<std::unique_ptr<DistRank<T>>> ranks;  // virtual: all g; RCCL: this rank only
    ncclComm_t commB = nullptr, commP = nullptr;       // RCCL: broadcast / panel communicators
    bool own_commP = false;
    hipStream_t sB = nullptr, sP = nullptr;            // transport streams
    DistLayout L;
    int64_t key_n = -1;
    int key_m = -1;
    bool key_fused = false;
    int P = 0;
    double est_us = 0;
    std::vector<std::vector<int4>> lists;
    ~DistEngine() override {
        ranks.clear();
        if (sB) (void)hipStreamDestroy(sB);
        if (sP) (void)hipStreamDestroy(sP);
        if (own_commP && commP) (void)ncclCommDestroy(commP);
    }
};

// ---------------------------------------------------------------------------------------
// small kernels
// ---------------------------------------------------------------------------------------
namespace {

template <typename T>
__global__ void diag_fix_local_kernel(T* __restrict__ A, int64_t ld, int64_t row0, int64_t c0, int64_t n, T s2) {
    const int t = threadIdx.x;
    if (t >= DB) return;
    const int64_t gi = c0 + t;
    T* p = A + row0 + t + gi * ld;
    *p = (gi < n) ? *p + s2 : T(1);
}

// out[0] = sum of 2 log L_ii over this rank's diagonal blocks (global index < n),
// out[1] = sum of z^2 over the label tiles (from the tile table, every rank has them all)
template <typename T>
__global__ __launch_bounds__(256) void dist_reduce_kernel(const T* __restrict__ A, int64_t ld, const int* __restrict__ loc,
                                                          int g, int r, int nc, int64_t n, int m,
                                                          const uint64_t* __restrict__ tiles,
                                                          const int64_t* __restrict__ tld, double* __restrict__ out) {
    __shared__ double s0[256], s1[256];
    const int t = threadIdx.x;
    double a = 0, b = 0;
    for (int k = 0; k < nc; k++) {  // this rank's diagonal blocks
        if (loc[k] < 0) continue;
        const int64_t gi = (int64_t)k * DB + (t & (DB - 1));
        if (t < DB && gi < n) a += 2.0 * log((double)A[(int64_t)loc[k] * DB + t + gi * ld]);
    }
    const int64_t lz = tld[nc];
    for (int k = 0; k < nc; k++) {
        const T* z = reinterpret_cast<const T*>(tiles[(int64_t)nc * nc + k]);
        for (int e = t; e < m * DB; e += 256) {
            const int rr = e % m, c = e / m;
            if ((int64_t)k * DB + c < n) {
                const double v = (double)z[rr + (int64_t)c * lz];
                b += v * v;
            }
        }
    }
    s0[t] = a;
    s1[t] = b;
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

}  // namespace

// ---------------------------------------------------------------------------------------
// engine setup (per shape): layout, buffers, tables, schedule
// ---------------------------------------------------------------------------------------
template <typename T>
static void setup(DistEngine<T>& E, const DistContext& C, int64_t n, int m, bool fused) {
    const int64_t np = (n + DB - 1) / DB * DB;
    const int nc = (int)(np / DB), nr = nc + 1;  // + the label row block
    if (E.key_n == n && E.key_m == m && E.key_fused == fused && !E.ranks.empty()) return;
    GPRX_REQUIRE(m <= GT, GPRX_ERR_DIM, "distributed fit: at most 128 label columns");
    E.g = C.world;
    E.virt = C.virt;
    E.device = C.device;
    // CU partition.  The transport kernels (RCCL, copies) and every (virtual) rank's
    // persistent launch run on streams whose CU masks are disjoint: a persistent launch can
    // never starve the transport of CUs, nor one virtual rank another.  Without the masks
    // the transport stalled behind the persistent launches (measured: 2 x 124 workgroups,
    // the copies waited until the launches timed out).  Mask bit b selects logical CU b / X
    // of XCC b % X (tools/cu_mask_probe.hip, gfx950; an XCC without a bit is unrestricted,
    // so every mask covers every XCC): a CU "slot" is one CU on each XCC.
    int ncu = 0, nxcc = 1;
    GPRX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, C.device));
    if (hipDeviceGetAttribute(&nxcc, hipDeviceAttributeNumberOfXccs, C.device) != hipSuccess || nxcc < 1) nxcc = 1;
    const int cu_xcc = std::max(1, ncu / nxcc);
    // transport slots: one CU per XCC for the virtual ranks' copies; two for RCCL, whose
    // kernels run one workgroup per channel
    int reserve = E.virt ? 1 : 2;
    if (const char* e = std::getenv("GPRX_DIST_RESERVE_CU")) reserve = std::max(1, std::atoi(e));
    const int nloc_ranks = E.virt ? E.g : 1;
    GPRX_REQUIRE(cu_xcc - reserve >= nloc_ranks, GPRX_ERR_ARG, "distributed fit: too many virtual ranks for the CUs");
    const int per = (cu_xcc - reserve) / nloc_ranks;  // compute slots per rank
    E.P = nxcc * per;  // one workgroup per CU (LDS)
    if (const char* e = std::getenv("GPRX_DIST_P")) E.P = std::max(1, std::atoi(e));
    auto masked_stream = [&](int slot0, int nslot) {
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int c = slot0; c < slot0 + nslot; c++)
            for (int x = 0; x < nxcc; x++) {
                const int b = c * nxcc + x;
                if (b < ncu) mask[b / 32] |= 1u << (b % 32);
            }
        hipStream_t st = nullptr;
        GPRX_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
        return st;
    };
    // row-block grouping: the simulated makespan picks gb (GPRX_DIST_GROUP forces it)
    int gb = 1;
    if (const char* e = std::getenv("GPRX_DIST_GROUP")) {
        gb = std::max(1, std::atoi(e));
        E.lists = potrf_dist_schedule(nc, nr, E.P, E.g, gb, fused, &E.est_us);
    } else {
        E.lists = potrf_dist_schedule(nc, nr, E.P, E.g, 1, fused, &E.est_us);
        for (int cand = 2; E.g > 1 && cand <= 8 && nc >= 2 * cand * E.g; cand *= 2) {
            double est = 0;
            auto l = potrf_dist_schedule(nc, nr, E.P, E.g, cand, fused, &est);
            if (est < E.est_us) {
                E.est_us = est;
                E.lists = std::move(l);
                gb = cand;
            }
        }
    }
    E.L.init(E.g, gb, nc, nr);
    if (!E.sB) {
        E.sB = masked_stream(0, reserve);
        E.sP = masked_stream(0, reserve);
    }
    if (!E.virt && !E.commP) {
        E.commB = C.comm;
        if (E.g > 1) {  // a second communicator: the two transport streams progress independently
            rccl_ok(ncclCommSplit(C.comm, 0, C.rank, &E.commP, nullptr), "ncclCommSplit");
            E.own_commP = true;
        } else {
            E.commP = C.comm;
        }
    }
    E.ranks.clear();
    const int nranks = E.virt ? E.g : 1;
    const int64_t DB2 = (int64_t)DB * DB;
    for (int v = 0; v < nranks; v++) {
        auto R = std::make_unique<DistRank<T>>();
        R->r = E.virt ? v : C.rank;
        const int r = R->r;
        R->s = masked_stream(reserve + v * per, per);  // this rank's CUs
        R->own_stream = true;
        GPRX_HIP(hipEventCreateWithFlags(&R->done, hipEventDisableTiming));
        GPRX_HIP(hipEventCreate(&R->t0));
        GPRX_HIP(hipEventCreate(&R->t1));
        GPRX_HIP(hipEventCreate(&R->t2));
        const int nl = E.L.nloc(r);
        R->ld = (int64_t)nl * DB;
        R->A.ensure(sizeof(T) * R->ld * np);
        R->Linv.ensure(sizeof(T) * nc * DB2, hipDeviceMallocFinegrained);
        R->send.ensure(sizeof(T) * std::max<int64_t>(1, E.L.stot[r]) * DB2);
        R->recv.ensure(sizeof(T) * std::max<int64_t>(1, E.L.rtot[r]) * DB2, hipDeviceMallocFinegrained);
        R->ctr.ensure(sizeof(int) * ((size_t)C_NCTL_DIST + nr + (size_t)nr * nc));
        R->info.ensure(sizeof(int));
        R->flag.ensure(sizeof(int));
        R->drecv.ensure(2 * sizeof(unsigned), hipDeviceMallocUncached);
        R->red.ensure(2 * sizeof(double));
        R->alpha.ensure(sizeof(T) * np * m);
        R->hdiag.ensure(sizeof(unsigned) * nc);
        R->hslot.ensure(sizeof(unsigned) * (size_t)nr * nc);
        // tables
        std::vector<int> loc(nr);
        std::vector<uint64_t> tptr((size_t)nr * nc, 0), sptr((size_t)nr * nc, 0), tiles((size_t)nr * nc, 0);
        std::vector<int64_t> tld(nr);
        T* Ab = R->A.template as<T>();
        for (int i = 0; i < nr; i++) {
            const int q = E.L.owner(i);
            loc[i] = (q == r) ? E.L.loc(i) : -1;
            tld[i] = (q == r) ? R->ld : (int64_t)DB;
            for (int b = 0; b < std::min(i, nc); b++) {
                if (q == r) {
                    sptr[(size_t)i * nc + b] =
                        (uint64_t)(R->send.template as<T>() + (E.L.soff[r][b] + E.L.pos(r, i, b)) * DB2);
                    tiles[(size_t)i * nc + b] = (uint64_t)(Ab + (int64_t)loc[i] * DB + (int64_t)b * DB * R->ld);
                } else {
                    const uint64_t p = (uint64_t)(R->recv.template as<T>() + (E.L.roff[r][b][q] + E.L.pos(q, i, b)) * DB2);
                    tptr[(size_t)i * nc + b] = p;
                    tiles[(size_t)i * nc + b] = p;
                }
            }
        }
        R->loc.ensure(sizeof(int) * nr);
        R->tptr.ensure(sizeof(uint64_t) * tptr.size());
        R->sptr.ensure(sizeof(uint64_t) * sptr.size());
        R->tiles.ensure(sizeof(uint64_t) * tiles.size());
        R->tld.ensure(sizeof(int64_t) * nr);
        GPRX_HIP(hipMemcpy(R->loc.p, loc.data(), sizeof(int) * nr, hipMemcpyHostToDevice));
        GPRX_HIP(hipMemcpy(R->tptr.p, tptr.data(), sizeof(uint64_t) * tptr.size(), hipMemcpyHostToDevice));
        GPRX_HIP(hipMemcpy(R->sptr.p, sptr.data(), sizeof(uint64_t) * sptr.size(), hipMemcpyHostToDevice));
        GPRX_HIP(hipMemcpy(R->tiles.p, tiles.data(), sizeof(uint64_t) * tiles.size(), hipMemcpyHostToDevice));
        GPRX_HIP(hipMemcpy(R->tld.p, tld.data(), sizeof(int64_t) * nr, hipMemcpyHostToDevice));
        PtDist<T> pd;
        pd.g = E.g;
        pd.r = r;
        pd.loc = R->loc.template as<int>();
        pd.tptr = reinterpret_cast<const T* const*>(R->tptr.p);
        pd.sptr = reinterpret_cast<T* const*>(R->sptr.p);
        unsigned *hd = nullptr, *hs = nullptr;
        GPRX_HIP(hipHostGetDevicePointer((void**)&hd, R->hdiag.p, 0));
        GPRX_HIP(hipHostGetDevicePointer((void**)&hs, R->hslot.p, 0));
        pd.hdiag = hd;
        pd.hslot = hs;
        pd.drecv = R->drecv.template as<unsigned>();
        pd.precv = R->drecv.template as<unsigned>() + 1;
        R->pd.ensure(sizeof(PtDist<T>));
        GPRX_HIP(hipMemcpy(R->pd.p, &pd, sizeof(pd), hipMemcpyHostToDevice));
        const std::vector<int4>& lst = E.lists[r];
        R->hlist = lst;
        R->ntasks = (int)lst.size();
        R->list.ensure(sizeof(int4) * std::max<size_t>(1, lst.size()));
        if (!lst.empty()) GPRX_HIP(hipMemcpy(R->list.p, lst.data(), sizeof(int4) * lst.size(), hipMemcpyHostToDevice));
        E.ranks.push_back(std::move(R));
    }
    E.key_n = n;
    E.key_m = m;
    E.key_fused = fused;
}

// ---------------------------------------------------------------------------------------
// transport steps
// ---------------------------------------------------------------------------------------
template <typename T>
static void issue_bcast(DistEngine<T>& E, int k) {
    const int64_t DB2 = (int64_t)DB * DB;
    const int root = E.L.owner(k);
    if (E.virt) {
        const DistRank<T>& Rt = *E.ranks[root];
        for (auto& R : E.ranks)
            if (R->r != root)
                GPRX_HIP(hipMemcpyAsync(R->Linv.template as<T>() + k * DB2, Rt.Linv.template as<T>() + k * DB2,
                                        sizeof(T) * DB2, hipMemcpyDeviceToDevice, E.sB));
        for (auto& R : E.ranks) GPRX_HIP(hipStreamWriteValue32(E.sB, R->drecv.p, (uint32_t)(k + 1), 0));
    } else {
        DistRank<T>& R = *E.ranks[0];
        T* p = R.Linv.template as<T>() + k * DB2;
        if (E.g > 1) rccl_ok(ncclBroadcast(p, p, (size_t)DB2, nccl_t<T>(), root, E.commB, E.sB), "ncclBroadcast");
        GPRX_HIP(hipStreamWriteValue32(E.sB, R.drecv.p, (uint32_t)(k + 1), 0));
    }
}

template <typename T>
static void issue_panel(DistEngine<T>& E, int b) {
    const int64_t DB2 = (int64_t)DB * DB;
    if (E.virt) {
        for (auto& R : E.ranks)
            for (auto& Q : E.ranks) {
                if (Q->r == R->r) continue;
                const int64_t c = E.L.cnt(Q->r, b);
                if (c == 0) continue;
                GPRX_HIP(hipMemcpyAsync(R->recv.template as<T>() + E.L.roff[R->r][b][Q->r] * DB2,
                                        Q->send.template as<T>() + E.L.soff[Q->r][b] * DB2, sizeof(T) * c * DB2,
                                        hipMemcpyDeviceToDevice, E.sP));
            }
        for (auto& R : E.ranks)
            GPRX_HIP(hipStreamWriteValue32(E.sP, R->drecv.template as<unsigned>() + 1, (uint32_t)(b + 1), 0));
    } else {
        DistRank<T>& R = *E.ranks[0];
        const int r = R.r;
        if (E.g > 1) {
            rccl_ok(ncclGroupStart(), "ncclGroupStart");
            const int64_t cs = E.L.cnt(r, b);
            for (int q = 0; q < E.g; q++) {
                if (q == r) continue;
                if (cs > 0)
                    rccl_ok(ncclSend(R.send.template as<T>() + E.L.soff[r][b] * DB2, (size_t)(cs * DB2), nccl_t<T>(), q,
                                     E.commP, E.sP),
                            "ncclSend");
                const int64_t cq = E.L.cnt(q, b);
                if (cq > 0)
                    rccl_ok(ncclRecv(R.recv.template as<T>() + E.L.roff[r][b][q] * DB2, (size_t)(cq * DB2), nccl_t<T>(),
                                     q, E.commP, E.sP),
                            "ncclRecv");
            }
            rccl_ok(ncclGroupEnd(), "ncclGroupEnd");
        }
        GPRX_HIP(hipStreamWriteValue32(E.sP, R.drecv.template as<unsigned>() + 1, (uint32_t)(b + 1), 0));
    }
}

// this host's ranks have every tile of panel b in its send slot
template <typename T>
static bool panel_ready(const DistEngine<T>& E, int b) {
    for (auto& R : E.ranks) {
        const unsigned* hs = R->hslot.u();
        const std::vector<int>& rw = E.L.rows[R->r];
        for (int x = E.L.firstpos(R->r, b); x < (int)rw.size(); x++)
            if (__atomic_load_n(hs + (size_t)rw[x] * E.L.nc + b, __ATOMIC_ACQUIRE) == 0) return false;
    }
    return true;
}

template <typename T>
static bool bcast_ready(const DistEngine<T>& E, int k) {
    const int root = E.L.owner(k);
    for (auto& R : E.ranks)
        if (R->r == root) return __atomic_load_n(R->hdiag.u() + k, __ATOMIC_ACQUIRE) != 0;
    return true;  // another process's rank: RCCL waits for it on the device
}

// ---------------------------------------------------------------------------------------
// the fit
// ---------------------------------------------------------------------------------------
template <typename T>
void dist_fit(DistEngineBase*& eng, const DistContext& C, const DistFitIn<T>& in, DistFitOut& out, T* alpha_dev,
              Exec& ex) {
    if (!eng) eng = new DistEngine<T>();
    DistEngine<T>& E = *static_cast<DistEngine<T>*>(eng);
    const bool fused = in.tb.mode != 0;
    setup<T>(E, C, in.n, in.m, fused);
    const int nc = E.L.nc, nr = E.L.nr;
    const int64_t np = (int64_t)nc * DB, n = in.n;
    const int64_t DB2 = (int64_t)DB * DB;
    DistRank<T>& R0 = *E.ranks[0];
    // ---- per rank: reset, build; then the launches -------------------------------------------
    std::vector<DistLaunch<T>> launches(E.ranks.size());
    for (auto& Rp : E.ranks) {
        DistRank<T>& R = *Rp;
        const int r = R.r;
        hipStream_t s = R.s;
        std::memset(R.hdiag.p, 0, R.hdiag.bytes);
        std::memset(R.hslot.p, 0, R.hslot.bytes);
        const size_t nctr = (size_t)C_NCTL_DIST + nr + (size_t)nr * nc;
        GPRX_HIP(hipMemsetAsync(R.ctr.p, 0, sizeof(int) * nctr, s));
        GPRX_HIP(hipMemsetAsync(R.drecv.p, 0, 2 * sizeof(unsigned), s));
        GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)R.info.p, INT_MAX, 1, s));
        GPRX_HIP(hipMemsetAsync(R.flag.p, 0, sizeof(int), s));
        T* A = R.A.template as<T>();
        if (fused) {
            // BUILD tasks write the lower tiles: ver = -1 until built (rows of the matrix only)
            GPRX_HIP(hipMemsetAsync(R.ctr.template as<int>() + C_NCTL_DIST + nr, 0xff, sizeof(int) * (size_t)nc * nc, s));
        } else {
            // the direct build: each owned row block against the columns up to its diagonal
            GPRX_HIP(hipMemsetAsync(A, 0, sizeof(T) * R.ld * np, s));
            for (int i : E.L.rows[r]) {
                if (i >= nc) continue;
                const int64_t r0 = (int64_t)i * DB, rows = std::min<int64_t>(DB, n - r0), cols = std::min<int64_t>(r0 + DB, n);
                T* Ai = A + (int64_t)E.L.loc(i) * DB;
                if (rows > 0) {
                    const T *tabr = nullptr, *tabc = nullptr;
                    if (in.K.nper > 0) {  // sin/cos tables of the block's rows and of its columns
                        const size_t slot = (size_t)2 * in.K.nper * in.d;
                        R.tab.ensure(sizeof(T) * slot * ((size_t)DB + (size_t)n));
                        T* tr = R.tab.template as<T>();
                        T* tc = tr + slot * DB;
                        launch_sincos_tables<T>(in.K, in.X + r0 * in.d, rows, in.d, tr, s);
                        launch_sincos_tables<T>(in.K, in.X, cols, in.d, tc, s);
                        tabr = tr;
                        tabc = tc;
                    }
                    launch_kbuild<T>(in.K, in.X + r0 * in.d, tabr, rows, in.X, tabc, cols, in.d, Ai, R.ld, 0, false,
                                     T(0), R.flag.template as<int>(), s);
                }
                hipLaunchKernelGGL(diag_fix_local_kernel<T>, dim3(1), dim3(DB), 0, s, A, R.ld,
                                   (int64_t)E.L.loc(i) * DB, r0, n, in.sigma2);
            }
        }
        if (E.L.owner(nc) == r)  // the label rows: Y^T as row block nc
            launch_label_rows<T>(in.Y, n, in.m, A, R.ld, (int64_t)E.L.loc(nc) * DB, np, GT, s);
        TileBuild<T> tbl = in.tb;
        tbl.flag = R.flag.template as<int>();
        void* tbdev = nullptr;
        if (fused) {
            R.red.ensure(std::max<size_t>(R.red.bytes, sizeof(TileBuild<T>) + 64));
            tbdev = static_cast<char*>(R.red.p) + 64;  // after the reduction doubles
            // synchronous, before any rank's persistent launch: a pageable copy queued behind
            // one could wait for it (and the virtual ranks' launches must be co-resident)
            GPRX_HIP(hipStreamSynchronize(s));
            GPRX_HIP(hipMemcpy(tbdev, &tbl, sizeof(tbl), hipMemcpyHostToDevice));
        }
        DistLaunch<T>& Lc = launches[&Rp - &E.ranks[0]];
        Lc.A = A;
        Lc.ld = R.ld;
        Lc.Linv = R.Linv.template as<T>();
        Lc.info = R.info.template as<int>();
        Lc.list = R.list.template as<int4>();
        Lc.ntasks = R.ntasks;
        Lc.nc = nc;
        Lc.nr = nr;
        Lc.ctr = R.ctr.template as<int>();
        Lc.tb_dev = reinterpret_cast<const TileBuild<T>*>(tbdev);
        Lc.dist_dev = R.pd.template as<PtDist<T>>();
        Lc.tlimit = (long long)(1e8 * (2.0 + 20.0 * E.est_us * 1e-6));
        Lc.P = E.P;
        Lc.s = s;
        Lc.dbg = nullptr;
        Lc.trace = nullptr;
        static const char* tdir = std::getenv("GPRX_DIST_TRACE_DEV");  // directory for per-rank task traces
        if (tdir) {
            R.trace.ensure(sizeof(long long) * 4 * ((size_t)R.ntasks + 2 * (size_t)nc));
            GPRX_HIP(hipMemsetAsync(R.trace.p, 0, R.trace.bytes, s));
            Lc.trace = R.trace.template as<long long>();
        }
        static const bool dbgw = std::getenv("GPRX_DIST_DEBUG") != nullptr;
        if (dbgw) {
            R.dbg.ensure(sizeof(int) * 4 * E.P);
            std::memset(R.dbg.p, 0xff, sizeof(int) * 4 * E.P);
            GPRX_HIP(hipHostGetDevicePointer((void**)&Lc.dbg, R.dbg.p, 0));
        }
    }
    // every rank's persistent launch back to back, nothing that could block in between
    for (size_t v = 0; v < E.ranks.size(); v++) {
        GPRX_HIP(hipEventRecord(E.ranks[v]->t0, E.ranks[v]->s));
        potrf_tiles_dist_launch<T>(launches[v]);
        GPRX_HIP(hipEventRecord(E.ranks[v]->done, E.ranks[v]->s));
        GPRX_HIP(hipEventRecord(E.ranks[v]->t1, E.ranks[v]->s));
    }
    // ---- issue loop: transport steps as their inputs become ready --------------------------
    const auto ts = std::chrono::steady_clock::now();
    int kb = 0, kp = 0;
    bool flush = false;
    double issue_s = 0;  // host time spent inside the transport calls (diagnostics)
    double dbg_next = 0.25;
    const double limit_s = 4.0 + 40.0 * E.est_us * 1e-6;
    static const bool trace = std::getenv("GPRX_DIST_TRACE") != nullptr;
    std::vector<double> tb_issue(trace ? nc : 0), tp_issue(trace ? nc : 0);
    auto now_us = [&]() { return 1e6 * std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count(); };
    while (kb < nc || kp < nc) {
        bool progress = false;
        if (kb < nc && (flush || bcast_ready(E, kb))) {
            const auto t0 = std::chrono::steady_clock::now();
            if (trace) tb_issue[kb] = now_us();
            issue_bcast(E, kb++);
            issue_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            progress = true;
        }
        if (kp < nc && kp < kb + 1 && (flush || panel_ready(E, kp))) {
            const auto t0 = std::chrono::steady_clock::now();
            if (trace) tp_issue[kp] = now_us();
            issue_panel(E, kp++);
            issue_s += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            progress = true;
        }
        if (progress || flush) continue;
        // stalled: kernels ended early (a timed-out wait drained them) or out of time -> issue
        // the rest (their data is stale, the fit reports the error) so peers are not left
        // waiting inside RCCL
        bool all_done = true;
        for (auto& R : E.ranks) all_done &= hipEventQuery(R->done) == hipSuccess;
        const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count();
        static const bool dbgw = std::getenv("GPRX_DIST_DEBUG") != nullptr;
        if (dbgw && !flush && el > dbg_next) {  // a stall: where every workgroup is
            dbg_next += 0.5;
            for (auto& Rp : E.ranks) {
                const int* w = reinterpret_cast<const int*>(Rp->dbg.p);
                unsigned rc[2] = {9999, 9999};
                (void)hipMemcpy(rc, Rp->drecv.p, sizeof(rc), hipMemcpyDeviceToHost);
                int nun = 0, nwait = 0, nwork = 0, nend = 0;
                for (int x = 0; x < E.P; x++) {
                    const int ph = __atomic_load_n(w + 4 * x + 1, __ATOMIC_ACQUIRE);
                    nun += ph < 0;
                    nwait += ph >= 0 && ph % 10 == 1;
                    nwork += ph >= 0 && ph % 10 == 2;
                    nend += ph == 9;
                }
                std::fprintf(stderr,
                             "gprx dist stall rank %d (issued bcast %d panel %d, %.3f s; device drecv %u precv %u; "
                             "issue calls took %.3f s; workgroups unstarted %d waiting %d working %d ended %d; hdiag0 %u):",
                             Rp->r, kb, kp, el, rc[0], rc[1], issue_s, nun, nwait, nwork, nend, Rp->hdiag.u()[0]);
                int shown = 0;
                for (int x = 0; x < E.P && shown < 16; x++) {
                    const int q = __atomic_load_n(w + 4 * x, __ATOMIC_ACQUIRE), ph = w[4 * x + 1];
                    if (q < 0 || q >= (int)Rp->hlist.size() || ph % 10 != 1) continue;
                    const int4 t = Rp->hlist[q];
                    shown++;
                    std::fprintf(stderr, " [t%d %s(%d,%d,b0 %d,nb %d)]", q,
                                 (t.x & 255) == 0 ? "DIAGX" : (t.x & 255) == 1 ? "TRSM" : (t.x & 255) == 2 ? "UPD" : "BUILD",
                                 t.y, t.z, t.w, t.x >> 8);
                }
                std::fprintf(stderr, "\n");
            }
        }
        if (all_done || el > limit_s) flush = true;
        else std::this_thread::yield();
    }
    for (auto& R : E.ranks) GPRX_HIP(hipStreamSynchronize(R->s));
    if (const char* tdir = std::getenv("GPRX_DIST_TRACE_DEV")) {  // raw per-rank task traces
        for (auto& Rp : E.ranks) {
            std::vector<long long> tr(4 * ((size_t)Rp->ntasks + 2 * (size_t)nc));
            GPRX_HIP(hipMemcpy(tr.data(), Rp->trace.p, sizeof(long long) * tr.size(), hipMemcpyDeviceToHost));
            const std::string path = std::string(tdir) + "/rank" + std::to_string(Rp->r) + ".bin";
            if (FILE* f = std::fopen(path.c_str(), "wb")) {
                const int hdr[4] = {Rp->ntasks, nc, E.g, E.L.gb};
                std::fwrite(hdr, sizeof(int), 4, f);
                std::fwrite(Rp->hlist.data(), sizeof(int4), Rp->hlist.size(), f);
                std::fwrite(tr.data(), sizeof(long long), tr.size(), f);
                std::fclose(f);
            }
        }
    }
    if (trace) {  // host times of the transport issues (us from the launches)
        const double tend = now_us();
        std::fprintf(stderr, "gprx dist trace g %d P %d nc %d: end %.0f us, issue calls %.0f us\n", E.g, E.P, nc, tend,
                     1e6 * issue_s);
        for (int k = 0; k < nc; k++)
            if (k < 8 || k % 16 == 0 || k >= nc - 4)
                std::fprintf(stderr, "  k %4d bcast %9.1f panel %9.1f  (bcast step %7.1f)\n", k, tb_issue[k], tp_issue[k],
                             k ? tb_issue[k] - tb_issue[k - 1] : tb_issue[k]);
    }
    GPRX_HIP(hipStreamSynchronize(E.sB));
    GPRX_HIP(hipStreamSynchronize(E.sP));
    GPRX_HIP(hipGetLastError());
    static const bool dbg = std::getenv("GPRX_DIST_DEBUG") != nullptr;
    if (dbg || flush) {  // the state the issue loop ended in (flush: a stall)
        for (auto& Rp : E.ranks) {
            DistRank<T>& R = *Rp;
            unsigned rc[2] = {0, 0};
            int ctl[2] = {0, 0};
            GPRX_HIP(hipMemcpy(rc, R.drecv.p, sizeof(rc), hipMemcpyDeviceToHost));
            GPRX_HIP(hipMemcpy(ctl, R.ctr.p, sizeof(ctl), hipMemcpyDeviceToHost));
            int nd = 0, ns = 0, nsw = 0;
            for (int k = 0; k < nc; k++) nd += R.hdiag.u()[k] != 0;
            for (int i = 0; i < nr; i++)
                for (int b = 0; b < std::min(i, nc); b++)
                    if (E.L.owner(i) == R.r) {
                        nsw++;
                        ns += R.hslot.u()[(size_t)i * nc + b] != 0;
                    }
            std::fprintf(stderr,
                         "gprx dist rank %d/%d: P %d tickets %d/%d err %d | diag flags %d/%d (own) send slots %d/%d | "
                         "drecv %u precv %u | issued bcast %d panel %d of %d%s\n",
                         R.r, E.g, E.P, ctl[0], R.ntasks, ctl[1], nd, E.L.cnt(R.r, -1) - (E.L.owner(nc) == R.r), ns, nsw, rc[0], rc[1],
                         kb, kp, nc, flush ? " (flushed)" : "");
        }
    }
    // ---- reductions, back substitution (every rank holds every tile) -------------------------
    double logdet = 0, datafit = 0;
    int info = INT_MAX, flag = 0;
    for (auto& Rp : E.ranks) {
        DistRank<T>& R = *Rp;
        hipLaunchKernelGGL(dist_reduce_kernel<T>, dim3(1), dim3(256), 0, R.s, R.A.template as<T>(), R.ld,
                           R.loc.template as<int>(), E.g, R.r, nc, n, in.m, R.tiles.template as<uint64_t>(),
                           R.tld.template as<int64_t>(), R.red.template as<double>());
        double red[2];
        int hi = 0, hf = 0;
        GPRX_HIP(hipMemcpyAsync(red, R.red.p, sizeof(red), hipMemcpyDeviceToHost, R.s));
        GPRX_HIP(hipMemcpyAsync(&hi, R.info.p, sizeof(int), hipMemcpyDeviceToHost, R.s));
        GPRX_HIP(hipMemcpyAsync(&hf, R.flag.p, sizeof(int), hipMemcpyDeviceToHost, R.s));
        GPRX_HIP(hipStreamSynchronize(R.s));
        logdet += red[0];
        datafit = red[1];
        info = std::min(info, hi);
        flag = std::max(flag, hf);
    }
    if (!E.virt && E.g > 1) {  // combine over the ranks: sum of log det, min info, max flag
        DMem dv;
        dv.ensure(sizeof(double) + 2 * sizeof(int));
        double* dl = dv.as<double>();
        int* di = reinterpret_cast<int*>(dl + 1);
        GPRX_HIP(hipMemcpyAsync(dl, &logdet, sizeof(double), hipMemcpyHostToDevice, R0.s));
        GPRX_HIP(hipMemcpyAsync(di, &info, sizeof(int), hipMemcpyHostToDevice, R0.s));
        GPRX_HIP(hipMemcpyAsync(di + 1, &flag, sizeof(int), hipMemcpyHostToDevice, R0.s));
        rccl_ok(ncclGroupStart(), "ncclGroupStart");
        rccl_ok(ncclAllReduce(dl, dl, 1, ncclFloat64, ncclSum, E.commB, R0.s), "ncclAllReduce");
        rccl_ok(ncclAllReduce(di, di, 1, ncclInt32, ncclMin, E.commB, R0.s), "ncclAllReduce");
        rccl_ok(ncclAllReduce(di + 1, di + 1, 1, ncclInt32, ncclMax, E.commB, R0.s), "ncclAllReduce");
        rccl_ok(ncclGroupEnd(), "ncclGroupEnd");
        GPRX_HIP(hipMemcpyAsync(&logdet, dl, sizeof(double), hipMemcpyDeviceToHost, R0.s));
        GPRX_HIP(hipMemcpyAsync(&info, di, sizeof(int), hipMemcpyDeviceToHost, R0.s));
        GPRX_HIP(hipMemcpyAsync(&flag, di + 1, sizeof(int), hipMemcpyDeviceToHost, R0.s));
        GPRX_HIP(hipStreamSynchronize(R0.s));
    }
    out.logdet = logdet;
    out.datafit = datafit;
    out.info = info;
    out.flag = flag;
    out.est_us = E.est_us;
    out.P = E.P;
    out.ms_kernel = 0;
    for (auto& Rp : E.ranks) {  // the persistent launches' device time (the slowest rank)
        float ms = 0;
        if (hipEventElapsedTime(&ms, Rp->t0, Rp->t1) == hipSuccess) out.ms_kernel = std::max(out.ms_kernel, (double)ms);
    }
    if (info < 0 || info != INT_MAX || flag) return;  // the caller reports it
    // alpha = L^{-T} z on rank 0 of this process (the factor is complete on every rank)
    GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)R0.info.p, INT_MAX, 1, R0.s));
    launch_backsolve_chain<T>(nullptr, 0, np, in.m, R0.Linv.template as<T>(), alpha_dev, R0.info.template as<int>(), ex,
                              R0.s, R0.tiles.template as<uint64_t>(), R0.tld.template as<int64_t>());
    GPRX_HIP(hipEventRecord(R0.t2, R0.s));
    int hi = 0;
    GPRX_HIP(hipMemcpyAsync(&hi, R0.info.p, sizeof(int), hipMemcpyDeviceToHost, R0.s));
    GPRX_HIP(hipStreamSynchronize(R0.s));
    if (hi != INT_MAX) out.info = hi;
    float ms = 0;
    if (hipEventElapsedTime(&ms, R0.t1, R0.t2) == hipSuccess) out.ms_solve = ms;
    (void)DB2;
}

void dist_engine_free(DistEngineBase* e) { delete e; }

namespace {
template <typename T>
__global__ __launch_bounds__(256) void assemble_tiles_kernel(const uint64_t* __restrict__ tiles,
                                                             const int64_t* __restrict__ tld, int nc, T* __restrict__ A,
                                                             int64_t ld) {
    const int i = blockIdx.x, j = blockIdx.y;  // tile (i, j), i > j
    if (j >= i) return;
    const T* src = reinterpret_cast<const T*>(tiles[(int64_t)i * nc + j]);
    const int64_t sl = tld[i];
    T* dst = A + (int64_t)i * DB + (int64_t)j * DB * ld;
    for (int e = threadIdx.x; e < DB * DB; e += 256) {
        const int r = e & (DB - 1), c = e >> 7;
        dst[r + (int64_t)c * ld] = src[r + (int64_t)c * sl];
    }
}
}  // namespace

template <typename T>
void dist_assemble_factor(DistEngineBase* eng, T* A, int64_t ld, T* Linv, hipStream_t s) {
    GPRX_REQUIRE(eng, GPRX_ERR_STATE, "distributed fit: no factor");
    DistEngine<T>& E = *static_cast<DistEngine<T>*>(eng);
    GPRX_REQUIRE(!E.ranks.empty(), GPRX_ERR_STATE, "distributed fit: no factor");
    const DistRank<T>& R0 = *E.ranks[0];
    const int nc = E.L.nc;
    GPRX_HIP(hipMemsetAsync(A, 0, sizeof(T) * (size_t)ld * nc * DB, s));
    if (nc > 1)
        hipLaunchKernelGGL(assemble_tiles_kernel<T>, dim3((unsigned)nc, (unsigned)nc), dim3(256), 0, s,
                           R0.tiles.template as<uint64_t>(), R0.tld.template as<int64_t>(), nc, A, ld);
    GPRX_HIP(hipMemcpyAsync(Linv, R0.Linv.p, sizeof(T) * (size_t)nc * DB * DB, hipMemcpyDeviceToDevice, s));
    GPRX_HIP(hipStreamSynchronize(s));
}
template void dist_assemble_factor<double>(DistEngineBase*, double*, int64_t, double*, hipStream_t);
template void dist_assemble_factor<float>(DistEngineBase*, float*, int64_t, float*, hipStream_t);

template <typename T>
static bool layout_of(DistEngineBase* eng, int* g, int* gb, int* rank, bool* virt) {
    auto* E = dynamic_cast<DistEngine<T>*>(eng);
    if (!E || E->ranks.empty()) return false;
    *g = E->g;
    *gb = E->L.gb;
    *rank = E->ranks[0]->r;
    *virt = E->virt;
    return true;
}

void dist_layout(DistEngineBase* eng, int* g, int* gb, int* rank, bool* virt) {
    GPRX_REQUIRE(eng && (layout_of<double>(eng, g, gb, rank, virt) || layout_of<float>(eng, g, gb, rank, virt)),
                 GPRX_ERR_STATE, "distributed fit: no layout");
}

template <typename T>
static bool allreduce_of(DistEngineBase* eng, double* dev, int count, hipStream_t s) {
    auto* E = dynamic_cast<DistEngine<T>*>(eng);
    if (!E) return false;
    if (!E->virt && E->g > 1) {
        rccl_ok(ncclAllReduce(dev, dev, (size_t)count, ncclFloat64, ncclSum, E->commB, s), "ncclAllReduce");
        GPRX_HIP(hipStreamSynchronize(s));
    }
    return true;
}

void dist_allreduce_sum(DistEngineBase* eng, double* dev, int count, hipStream_t s) {
    GPRX_REQUIRE(eng && (allreduce_of<double>(eng, dev, count, s) || allreduce_of<float>(eng, dev, count, s)),
                 GPRX_ERR_STATE, "distributed fit: no engine");
}

template void dist_fit<double>(DistEngineBase*&, const DistContext&, const DistFitIn<double>&, DistFitOut&, double*,
                               Exec&);
template void dist_fit<float>(DistEngineBase*&, const DistContext&, const DistFitIn<float>&, DistFitOut&, float*, Exec&);

}  // namespace gprx
