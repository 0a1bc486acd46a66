// gprx_dist.cpp — the storage-sharded multi-GPU fit (north_star: "the N x N matrix shards
// row-block across the GPUs with a broadcast of the diagonal panel at each potrf step").
//
// Replaces the same reference step as the single-GPU fit -- GaussianProcess::Initialize ->
// ComputeRegressionVectors, kernel matrix + lapack::lu_invert + C Y (lib/GaussianProcess.cpp
// :118-130, 642-672; include/LAPACKUtils.h:38-56) -- and the likelihood's inverse
// (include/Likelihood.h:204-285) for a matrix dealt over g ranks:
//
//   storage   row block i (128 rows; i = nc is the label block Y^T) lives on rank (i / gb) mod g
//             (groups of gb blocks dealt cyclically; gb from the simulated makespan).  A rank
//             keeps only the LOWER tiles of its own row blocks, packed (PtDist,
//             gprx_internal.h): ~N^2 / (2 g) of the factor.  Tiles of other ranks' rows pass
//             through a bounded WINDOW of ww panels (flow-controlled, below).
//   compute   each rank runs the persistent tile-dataflow launch (k_ptiles.hip,
//             potrf_tiles_kernel<T, true>) over its own row blocks: covariance BUILD tasks,
//             DIAGX (the diagonal 128-block chain), TRSM and UPD tasks, in the order of a list
//             schedule simulated over all ranks (potrf_dist_schedule)
//   exchange  device-initiated, no host thread in the loop: a task that finishes a tile other
//             ranks read stores it straight into their mailboxes (xGMI peer stores through IPC
//             mappings; the same process's memory for virtual ranks) and raises their per-tile
//             flag; DIAGX(k) pushes Linv_k to every rank -- the north star's broadcast of the
//             diagonal panel, issued by the kernel that produced it
//   flow      a window slot is refilled with panel p + ww only after every consumer released
//             panel p (its last window-reading update chunk done), so per-rank memory stays
//             N^2/(2g) + ww N 128 s + O(N 128 s) at any N
//   solve     alpha by a distributed back substitution (k_dsolve.hip): partial sums pushed to the
//             owner of each block, alpha_k pushed to every rank
//   reduce    log det (each rank's diagonal blocks), data fit, status: one host all-gather of a
//             few bytes per fit (RCCL, or the caller's collective)
//   LML mode  the inverse's identity rows ride along on their row's rank (U = L^{-T}) and the
//             lower C = U U^T accumulates in tiles of the same launch: the sharded potri
//             (SURVEY.md 8(f) rank 2); the gradient is reduced from each rank's own C tiles
//
// A second form runs g "virtual ranks" in one process on one GPU (gprx_ctx_create_virtual,
// include/gprx_dev.h): the same kernels, each rank on its own share of the CUs, pushing into the
// other ranks' buffers directly -- the distributed algorithm, exchange protocol and deadlock
// freedom testable on a single GPU (tests/test_gpu_dist.py).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "gprx_dist.h"

namespace gprx {

namespace {

void rccl_ok(ncclResult_t r, const char* what) {
    if (r != ncclSuccess) throw Error{GPRX_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r)};
}

// one device allocation, optionally fine-grained (the mailbox: stored into by other GPUs)
struct DMem {
    void* p = nullptr;
    size_t bytes = 0;
    void alloc(size_t b, bool fine) {
        release();
        if (b == 0) b = 256;
        if (fine) GPRX_HIP(hipExtMallocWithFlags(&p, b, hipDeviceMallocFinegrained));
        else GPRX_HIP(hipMalloc(&p, b));
        bytes = b;
        static const bool poison = std::getenv("GPRX_POISON") != nullptr;  // (debugging, as DevBuf)
        if (poison) GPRX_HIP(hipMemset(p, 0x41, b));
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

template <typename U>
void upload_vec(DMem& m, const std::vector<U>& v) {
    m.alloc(sizeof(U) * std::max<size_t>(1, v.size()), false);
    if (!v.empty()) GPRX_HIP(hipMemcpy(m.p, v.data(), sizeof(U) * v.size(), hipMemcpyHostToDevice));
}

int64_t align256(int64_t b) { return (b + 255) / 256 * 256; }

}  // namespace

// ---------------------------------------------------------------------------------------
// host collectives
// ---------------------------------------------------------------------------------------
struct RcclColl : HostColl {
    ncclComm_t comm;
    int world, device;
    hipStream_t s = nullptr;
    DMem sb, rb;
    RcclColl(ncclComm_t c, int w, int d) : comm(c), world(w), device(d) {
        GPRX_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    }
    ~RcclColl() override {
        if (s) (void)hipStreamDestroy(s);
    }
    void allgather(const void* send, size_t bytes, void* recv) override {
        if (world == 1) {
            std::memcpy(recv, send, bytes);
            return;
        }
        if (sb.bytes < bytes) sb.alloc(bytes, false);
        if (rb.bytes < bytes * world) rb.alloc(bytes * world, false);
        GPRX_HIP(hipMemcpy(sb.p, send, bytes, hipMemcpyHostToDevice));
        rccl_settle(comm, ncclAllGather(sb.p, rb.p, bytes, ncclUint8, comm, s), "ncclAllGather");
        GPRX_HIP(hipStreamSynchronize(s));
        GPRX_HIP(hipMemcpy(recv, rb.p, bytes * world, hipMemcpyDeviceToHost));
    }
};
HostColl* make_rccl_coll(ncclComm_t comm, int world, int device) { return new RcclColl(comm, world, device); }

void rccl_settle(ncclComm_t comm, ncclResult_t r, const char* what, double timeout_s) {
    const auto t0 = std::chrono::steady_clock::now();
    while (r == ncclInProgress) {
        ncclResult_t a = ncclInProgress;
        const ncclResult_t q = ncclCommGetAsyncError(comm, &a);
        if (q != ncclSuccess) {
            r = q;
            break;
        }
        r = a;
        if (r != ncclInProgress) break;
        if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
            throw Error{GPRX_ERR_RCCL, std::string(what) + ": not complete after " + std::to_string((int)timeout_s) +
                                           " s"};
        std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
    rccl_ok(r, what);
}

struct CallbackColl : HostColl {
    gprx_allgather_fn fn;
    void* user;
    int world;
    CallbackColl(gprx_allgather_fn f, void* u, int w) : fn(f), user(u), world(w) {}
    void allgather(const void* send, size_t bytes, void* recv) override {
        if (fn(user, send, bytes, recv) != 0) throw Error{GPRX_ERR_RCCL, "gprx: the caller's all-gather failed"};
    }
};
HostColl* make_callback_coll(gprx_allgather_fn fn, void* user, int world) { return new CallbackColl(fn, user, world); }

template <typename T>
void hostcoll_allreduce_dev(HostColl* hc, T* dev, int count, hipStream_t s) {
    std::vector<T> mine(count);
    GPRX_HIP(hipStreamSynchronize(s));
    GPRX_HIP(hipMemcpy(mine.data(), dev, sizeof(T) * count, hipMemcpyDeviceToHost));
    int world = 1;
    if (auto* r = dynamic_cast<RcclColl*>(hc)) world = r->world;
    if (auto* c = dynamic_cast<CallbackColl*>(hc)) world = c->world;
    std::vector<T> all((size_t)count * world);
    hc->allgather(mine.data(), sizeof(T) * count, all.data());
    for (int e = 0; e < count; e++) {  // rank order: every rank sums identically
        T v = 0;
        for (int q = 0; q < world; q++) v += all[(size_t)q * count + e];
        mine[e] = v;
    }
    GPRX_HIP(hipMemcpy(dev, mine.data(), sizeof(T) * count, hipMemcpyHostToDevice));
}
template void hostcoll_allreduce_dev<double>(HostColl*, double*, int, hipStream_t);
template void hostcoll_allreduce_dev<float>(HostColl*, float*, int, hipStream_t);

// ---------------------------------------------------------------------------------------
// layout: which rank holds which row block, and where in its packed storage
// ---------------------------------------------------------------------------------------
// A rank's storage is one or more PIECES (separate allocations of whole row blocks, each at most
// piece_elems): only allocations below 2 GiB can be mapped into another process (kIpcMaxBytes).
struct DistLayout {
    int g = 1, gb = 1, nc = 0, nr = 0, nci = 0;
    bool inv = false;
    std::vector<int> own, loc;            // per row block: owner rank, index among its rows
    std::vector<std::vector<int>> rows;   // per rank: owned row blocks, ascending
    std::vector<std::vector<int64_t>> roff;  // per rank: element offset of each own row block in its piece
    std::vector<std::vector<int>> piece;     // per rank: the piece of each own row block
    std::vector<std::vector<int64_t>> pelems;  // per rank: elements of each piece
    std::vector<int64_t> elems;           // per rank: storage elements (all pieces)
    int ncols(int i) const { return i < nc ? i + 1 : (i == nc ? nc : nc + 1); }
    void init(int g_, int gb_, int nc_, bool inv_, int64_t piece_elems) {
        g = g_;
        gb = std::max(1, gb_);
        nc = nc_;
        inv = inv_;
        nr = nc + 1 + (inv ? nc : 0);
        nci = inv ? 2 * nc : nc;
        own.assign(nr, 0);
        loc.assign(nr, 0);
        rows.assign(g, {});
        for (int i = 0; i < nr; i++) {
            own[i] = i <= nc ? (i / gb) % g : ((i - nc - 1) / gb) % g;
            loc[i] = (int)rows[own[i]].size();
            rows[own[i]].push_back(i);
        }
        roff.assign(g, {});
        piece.assign(g, {});
        pelems.assign(g, {});
        elems.assign(g, 0);
        const int64_t DB2 = (int64_t)DB * DB;
        for (int q = 0; q < g; q++) {
            int64_t o = 0;
            int p = 0;
            for (int i : rows[q]) {
                const int64_t sz = (int64_t)ncols(i) * DB2;
                if (o > 0 && o + sz > piece_elems) {  // the next piece
                    pelems[q].push_back(o);
                    p++;
                    o = 0;
                }
                roff[q].push_back(o);
                piece[q].push_back(p);
                o += sz;
                elems[q] += sz;
            }
            pelems[q].push_back(o);
        }
    }
};

// the largest allocation mapped into another process (hipIpcOpenMemHandle of a larger one never
// returned on this stack: the sharded LML's 2.19 GB mailbox, a 2.1 GB rank storage at N = 32768)
constexpr int64_t kIpcMaxBytes = (int64_t(1) << 31) - (int64_t(1) << 20);

// query chunks of 128 columns one sharded posterior solve takes at most (its flag words)
constexpr int kPvChunks = 64;

// mailbox byte layout (identical on every rank): see PtDist / DSArgs.  The receive window is
// not in it: its ww x nr tile slots are separate pieces below 2 GiB (WindowLayout)
struct MailboxLayout {
    int64_t o_linv = 0, o_z = 0, o_alpha = 0, o_zf = 0, o_part = 0, o_flags = 0, o_sflags = 0, o_tags = 0, o_vflags = 0,
            bytes = 0;
    void init(int g, int nc, int nr, int ww, int m, size_t s, bool window) {
        const int64_t DB2 = (int64_t)DB * DB, np = (int64_t)nc * DB;
        int64_t o = 0;
        o_linv = o;
        o = align256(o + (int64_t)nc * DB2 * (int64_t)s);
        o_z = o;
        o = align256(o + (int64_t)nc * DB2 * (int64_t)s);
        o_alpha = o;
        o = align256(o + np * m * (int64_t)s);
        o_zf = o;
        o = align256(o + np * m * (int64_t)s);
        o_part = o;
        o = align256(o + (int64_t)g * nc * DB * m * (int64_t)s);
        o_flags = o;
        o = align256(o + 4 * (dist_f_rel(nr, nc) + (int64_t)g * nc));
        o_sflags = o;
        o = align256(o + 4 * ((int64_t)(2 + g) * nc));
        o_vflags = o;  // the posterior solve's V_k(c) flags (dist_posterior): nc x kPvChunks words
        o = align256(o + 4 * (int64_t)nc * kPvChunks);
        o_tags = o;
        o = align256(o + 4 * (window ? (int64_t)ww * nr : 1));
        bytes = o;
    }
};

// the receive window: slot (b mod ww, row j) = tile s = (b mod ww) nr + j, in piece s / tpp
struct WindowLayout {
    int64_t tiles = 0, tpp = 1;
    int npc = 0;
    void init(int ww, int nr, size_t s, int64_t piece_bytes, bool window) {
        tiles = window ? (int64_t)ww * nr : 0;
        tpp = std::max<int64_t>(1, piece_bytes / ((int64_t)DB * DB * (int64_t)s));
        npc = (int)((tiles + tpp - 1) / tpp);
    }
    int64_t piece_tiles(int p) const { return std::min(tpp, tiles - (int64_t)p * tpp); }
};

// one rank's buffers and launch state
template <typename T>
struct DistRank {
    int r = 0;
    hipStream_t s = nullptr;
    std::vector<std::unique_ptr<DMem>> store;  // the packed own row blocks, in pieces (DistLayout)
    std::vector<std::unique_ptr<DMem>> win;    // the receive window, in pieces (WindowLayout)
    DMem mbox, ctr, info, flag, red, sctl, part, pbuf;
    DMem t_loc, t_roff, t_own, t_tptr, t_cons, t_need, t_mb, t_wpc, t_orows, t_lastof, t_ctab, pd, list;
    DMem trace;                        // GPRX_DIST_TRACE_FILE: per-ticket timeline of the last launch
    std::vector<uint64_t> mb;          // every rank's mailbox as mapped here
    std::vector<std::vector<uint64_t>> st;  // every rank's storage pieces as mapped here
    std::vector<std::vector<uint64_t>> wp;  // every rank's window pieces as mapped here
    std::vector<int64_t> roff;         // own row blocks: element offset from the first piece's base
    DMem t_vslot, pvpart, pvsum;       // posterior solve: window slots of V_k(c) on every rank, partial sums
    DMem pvR, pvX, pvTab;              // posterior solve: K(Z, X_own) / W (nq x own rows), X_own, its tables
    std::vector<void*> opened;         // IPC mappings to close
    T* sbase() const { return store.empty() ? nullptr : store[0]->template as<T>(); }
    int64_t store_bytes() const {
        int64_t b = 0;
        for (auto& p : store) b += (int64_t)p->bytes;
        return b;
    }
    int64_t win_bytes() const {
        int64_t b = 0;
        for (auto& p : win) b += (int64_t)p->bytes;
        return b;
    }
    std::vector<int> orows;            // own matrix row blocks
    int ntasks = 0;
    hipEvent_t t0 = nullptr, t1 = nullptr;
    ~DistRank() {
        for (void* p : opened) (void)hipIpcCloseMemHandle(p);
        if (t0) (void)hipEventDestroy(t0);
        if (t1) (void)hipEventDestroy(t1);
        if (s) (void)hipStreamDestroy(s);
    }
};

struct DistEngineBase {
    virtual ~DistEngineBase() {}
};

template <typename T>
struct DistEngine : DistEngineBase {
    int g = 1, device = 0, P = 0, gb = 1, ww = 2, W = 1;
    bool virt = false;
    bool shared_dev = false;  // processes sharing one GPU (GPRX_DIST_SHARED_GPU)
    HostColl* hc = nullptr;
    DistLayout L;
    MailboxLayout MB;
    WindowLayout WL;
    DistSched S;
    int64_t key_n = -1;
    int key_m = -1;
    bool key_fused = false, key_inv = false;
    int64_t n = 0, np = 0;
    int m = 0;
    unsigned ep = 0, sep = 0;  // epochs of the fits and of the solves (flag values)
    unsigned vep = 0;          // epoch of the posterior solves
    int pv_nch = 0;            // query chunks per posterior solve (0: none: one rank, or no window)
    std::vector<std::unique_ptr<DistRank<T>>> ranks;  // virtual: all g; otherwise this process's rank
    int* dbg = nullptr;  // GPRX_PT_DEBUG: the launch's per-workgroup status words (pinned host memory)
    int dbg_n = 0;
    void free_dbg() {
        if (!dbg) return;
        pt_debug_register(dbg, 0);
        (void)hipHostFree(dbg);
        dbg = nullptr;
        dbg_n = 0;
    }
    // On a multi-process context the destruction is COLLECTIVE: teardown() ends with a host
    // all-gather (every process unmaps its peers' allocations before any frees its own), so
    // every process must destroy its model (or re-key its engine) in the same order
    ~DistEngine() override {
        teardown();
        free_dbg();
    }
    void teardown() {
        if (!virt && hc && !ranks.empty()) {  // every rank unmaps before any rank frees
            for (auto& R : ranks) {
                for (void* p : R->opened) (void)hipIpcCloseMemHandle(p);
                R->opened.clear();
            }
            try {
                int x = 0;
                std::vector<int> all(g);
                hc->allgather(&x, sizeof(int), all.data());
            } catch (...) {
            }
        }
        ranks.clear();
    }
};

// Every process of a multi-process context reaches this point before any goes on (a one-int
// all-gather; a no-op for virtual ranks and one rank).  Used before each sharded launch, so ranks
// that enter a fit seconds apart (I/O, GC on one of them) do not run into the launch's per-wait
// time limit, and after a gather that read the peers' storage, before any of them rewrites it.
template <typename T>
static void host_barrier(DistEngine<T>& E) {
    if (E.virt || E.g <= 1) return;
    int x = 0;
    std::vector<int> all(E.g);
    E.hc->allgather(&x, sizeof(int), all.data());
}

// A status agreed by every process: the minimum over the ranks (INT_MAX = ok).
template <typename T>
static int agree_min(DistEngine<T>& E, int v) {
    if (E.virt || E.g <= 1) return v;
    std::vector<int> all(E.g);
    E.hc->allgather(&v, sizeof(int), all.data());
    return *std::min_element(all.begin(), all.end());
}

// ---------------------------------------------------------------------------------------
// small kernels: counters, packed-storage initialisation, the factor gather
// ---------------------------------------------------------------------------------------
namespace {

// ver = -1 for the BUILD tiles (matrix rows, j <= i); identity row E_a: lcnt = a, ver[.] = a
__global__ void dist_init_counters(int* __restrict__ lcnt, int* __restrict__ ver, int nc, int nr, int nci, int build) {
    const int i = blockIdx.x;
    if (i >= nr) return;
    const int a = i > nc ? i - nc - 1 : 0;
    if (threadIdx.x == 0 && i > nc) lcnt[i] = a;
    for (int c = threadIdx.x; c < nci; c += blockDim.x) {
        int v = 0;
        if (i > nc) v = a;
        else if (build && i < nc && c <= i) v = -1;
        ver[(int64_t)i * nci + c] = v;
    }
}

// identity row block E_a (packed: columns a..nc-1, then the C tiles): the first tile the
// identity, everything else 0
template <typename T>
__global__ void dist_init_identity(T* __restrict__ rowbase, int ntile) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t tot = (int64_t)ntile * DB * DB;
    if (e >= tot) return;
    const int64_t r = e % DB, c = (e / DB) % DB, tile = e / ((int64_t)DB * DB);
    rowbase[e] = (tile == 0 && r == c) ? T(1) : T(0);
}

// the direct build's diagonal tile: + sigma^2 inside the matrix, identity in the padding
template <typename T>
__global__ void dist_diag_fix(T* __restrict__ tile, int64_t r0, int64_t n, T s2) {
    const int t = threadIdx.x;
    if (t >= DB) return;
    T* p = tile + t + (int64_t)t * DB;
    *p = (r0 + t < n) ? *p + s2 : T(1);
}

// dense gather: tile (i, j), i > j, of the factor from its rank's storage (src table) into A
template <typename T>
__global__ __launch_bounds__(256) void dist_gather_kernel(const uint64_t* __restrict__ src, int nc, T* __restrict__ A,
                                                          int64_t ld) {
    const int i = blockIdx.x, j = blockIdx.y;
    if (j >= i) return;
    const T* s = reinterpret_cast<const T*>(src[(int64_t)i * nc + j]);
    T* d = A + (int64_t)i * DB + (int64_t)j * DB * ld;
    for (int e = threadIdx.x; e < DB * DB; e += 256) {
        const int r = e & (DB - 1), c = e >> 7;
        d[r + (int64_t)c * ld] = s[e];
    }
}

// out of a mailbox (alpha, Linv) into ordinary memory: system-scope loads.  A plain copy
// (hipMemcpy D2D) of a mailbox that the ranks' kernels wrote from other XCDs was seen to return
// the previous solve's values (alpha + 2 delta_1 in place of alpha + delta_1 + delta_2 in the
// fp32 refinement, one run in six; stale columns in an m = 2 fit).
template <typename T>
__global__ __launch_bounds__(256) void dist_copy_sys(const T* __restrict__ src, T* __restrict__ dst, int64_t count) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e < count) dst[e] = __hip_atomic_load(src + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <typename T>
void copy_from_mailbox(const void* src, T* dst, int64_t count, hipStream_t s) {
    if (count <= 0) return;
    hipLaunchKernelGGL(dist_copy_sys<T>, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, s,
                       reinterpret_cast<const T*>(src), dst, count);
    GPRX_HIP(hipGetLastError());
}

}  // namespace

// GPRX_DIST_VERBOSE=1: host-side progress of the setup and the fit, with timestamps (stderr)
static void dist_say(int rank, const char* what, long long a = -1) {
    static const bool on = std::getenv("GPRX_DIST_VERBOSE") != nullptr;
    if (!on) return;
    static const auto t0 = std::chrono::steady_clock::now();
    const double t = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::fprintf(stderr, "[gprx dist r%d %8.3f] %s %lld\n", rank, t, what, a);
}

// ---------------------------------------------------------------------------------------
// engine setup (per shape): layout, schedule, buffers, mailbox mappings, tables
// ---------------------------------------------------------------------------------------
template <typename T>
static void setup(DistEngine<T>& E, const DistContext& C, int64_t n, int m, bool fused, bool inv) {
    if (E.key_n == n && E.key_m == m && E.key_fused == fused && E.key_inv == inv && !E.ranks.empty()) return;
    GPRX_REQUIRE(m <= GT, GPRX_ERR_DIM, "distributed fit: at most 128 label columns");
    GPRX_REQUIRE(C.world >= 1 && C.world <= 32, GPRX_ERR_ARG, "distributed fit: 1..32 ranks");
    dist_say(C.rank, "setup: teardown", n);
    E.teardown();
    dist_say(C.rank, "setup: teardown done", inv ? 1 : 0);
    const int64_t np = (n + DB - 1) / DB * DB;
    const int nc = (int)(np / DB);
    E.g = C.world;
    E.virt = C.virt;
    E.shared_dev = !C.virt && C.cu_slots > 1;
    E.device = C.device;
    E.hc = C.hc;
    E.n = n;
    E.np = np;
    E.m = m;
    // CU partition.  A real rank has its GPU to itself (one workgroup per CU: nothing else runs
    // during the fit, the exchange is the kernel's own stores).  Virtual ranks, and processes
    // sharing one GPU (tests), each take a disjoint slice: every rank's persistent launch must be
    // resident for the others to progress.  Mask bit b selects logical CU b / X of XCC b % X
    // (tools/cu_mask_probe.hip, gfx950), so a slice is a range of "slots" of one CU per XCC.
    int ncu = 0, nxcc = 1;
    GPRX_HIP(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, C.device));
    if (hipDeviceGetAttribute(&nxcc, hipDeviceAttributeNumberOfXccs, C.device) != hipSuccess || nxcc < 1) nxcc = 1;
    const int cu_xcc = std::max(1, ncu / nxcc);
    const int nlocal = E.virt ? E.g : 1;
    const int shares = E.virt ? E.g : std::max(1, C.cu_slots);
    GPRX_REQUIRE(cu_xcc >= shares, GPRX_ERR_ARG, "distributed fit: too many ranks sharing the GPU's CUs");
    const int per = cu_xcc / shares;
    E.P = nxcc * per;
    if (const char* e = std::getenv("GPRX_DIST_P")) E.P = std::max(1, std::atoi(e));
    auto masked_stream = [&](int slot0, int nslot) {
        hipStream_t st = nullptr;
        if (shares == 1) {
            GPRX_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
            return st;
        }
        std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
        for (int c = slot0; c < slot0 + nslot; c++)
            for (int x = 0; x < nxcc; x++) {
                const int b = c * nxcc + x;
                if (b < ncu) mask[b / 32] |= 1u << (b % 32);
            }
        GPRX_HIP(hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data()));
        return st;
    };
    // row-block grouping and window: the simulated makespan picks them (GPRX_DIST_GROUP /
    // GPRX_DIST_WINDOW force them).  Every rank runs the same deterministic simulation.
    int gb = 1, ww = std::min(32, nc);
    double best = 0;
    constexpr bool f64 = std::is_same<T, double>::value;
    auto sim = [&](int gbc, int wwc) { return potrf_dist_schedule(nc, E.g, gbc, wwc, E.P, fused, inv, 0, f64); };
    const char* eg = std::getenv("GPRX_DIST_GROUP");
    const char* ew = std::getenv("GPRX_DIST_WINDOW");
    if (ew) ww = std::max(2, std::min(nc, std::atoi(ew)));
    if (E.g == 1) ww = std::max(2, nc);  // nothing goes through a window: chunks as on one GPU
    if (eg) {
        gb = std::max(1, std::atoi(eg));
        E.S = sim(gb, ww);
    } else {
        E.S = sim(1, ww);
        best = E.S.est_us;
        for (int cand = 2; E.g > 1 && cand <= 8 && nc >= 2 * cand * E.g; cand *= 2) {
            DistSched c = sim(cand, ww);
            if (c.est_us < best) {
                best = c.est_us;
                E.S = std::move(c);
                gb = cand;
            }
        }
    }
    if (!ew && E.g > 1) {
        // the window with the shortest simulated makespan among those within the memory budget
        // (GPRX_DIST_WINDOW_MB; default an eighth of the device's memory per rank -- a wider
        // window means wider update chunks: C3 on 8 virtual ranks 35.0 ms at 64 panels, 34.0 at
        // 128), near-ties (0.5%) to the smaller window
        size_t fr = 0, tot = 0;
        GPRX_HIP(hipMemGetInfo(&fr, &tot));
        double budget = (double)tot / 8.0 / (double)(E.virt ? E.g : std::max(1, C.cu_slots));
        if (const char* e = std::getenv("GPRX_DIST_WINDOW_MB")) budget = std::atof(e) * 1048576.0;
        const int nrw = nc + 1 + (inv ? nc : 0);
        auto wbytes = [&](int w) { return (double)w * nrw * DB * DB * (double)sizeof(T); };
        // (the window is allocated in pieces below 2 GiB, so IPC puts no limit on its width)
        std::vector<int> cws;
        for (int w = 8; w < nc; w *= 2) cws.push_back(w);
        cws.push_back(std::max(2, nc));
        int pick = -1;
        DistSched ps;
        for (int w : cws) {
            if (pick >= 0 && wbytes(w) > budget) break;
            DistSched c = sim(gb, w);
            if (pick < 0 || c.est_us < 0.995 * ps.est_us) {
                pick = w;
                ps = std::move(c);
            }
        }
        ww = pick;
        E.S = std::move(ps);
    }
    // the update-chunk rule (k_ptiles.hip tile_chunks): the capped rules, tried for the chosen
    // grouping and window, replace the fixed one when they simulate > 0.5% shorter
    // (on every tile, or on the last 16 column blocks only: the chain-bound tail)
    for (int ratio : {4, 2})
        for (int tail : {0, 16}) {
            if (tail >= nc) continue;
            DistSched c = potrf_dist_schedule(nc, E.g, gb, ww, E.P, fused, inv, ratio, f64, tail);
            if (c.est_us < 0.995 * E.S.est_us) E.S = std::move(c);
        }
    E.gb = gb;
    E.ww = ww;
    E.W = E.S.W;
    // allocation pieces: below kIpcMaxBytes when other processes map them (GPRX_DIST_PIECE_MB
    // forces smaller pieces in every mode, so the split layout runs at test sizes)
    int64_t piece_bytes = (!E.virt && E.g > 1) ? kIpcMaxBytes : INT64_MAX / 2;
    if (const char* e = std::getenv("GPRX_DIST_PIECE_MB"))
        piece_bytes = std::min(piece_bytes, std::max<int64_t>(1, std::atoll(e)) << 20);
    E.L.init(E.g, gb, nc, inv, piece_bytes / (int64_t)sizeof(T));
    const int nr = E.L.nr, nci = E.L.nci;
    E.MB.init(E.g, nc, nr, ww, m, sizeof(T), E.g > 1);
    E.WL.init(ww, nr, sizeof(T), piece_bytes, E.g > 1);
    E.pv_nch = E.g > 1 ? (int)std::min<int64_t>(kPvChunks, E.WL.tiles / nc) : 0;
    GPRX_REQUIRE(E.virt || E.g == 1 || E.MB.bytes <= kIpcMaxBytes, GPRX_ERR_ARG,
                 "distributed fit: the mailbox would exceed 2 GiB, the largest allocation another process can map");
    const int64_t DB2 = (int64_t)DB * DB;
    // ---- per local rank: buffers -------------------------------------------------------------
    dist_say(C.rank, "setup: schedule done, window", ww);
    for (int v = 0; v < nlocal; v++) {
        auto R = std::make_unique<DistRank<T>>();
        R->r = E.virt ? v : C.rank;
        const int r = R->r;
        const int slot = E.virt ? v : (shares > 1 ? C.cu_slot : 0);
        R->s = masked_stream(slot * per, per);
        GPRX_HIP(hipEventCreate(&R->t0));
        GPRX_HIP(hipEventCreate(&R->t1));
        for (int64_t pe : E.L.pelems[r]) {
            R->store.push_back(std::make_unique<DMem>());
            R->store.back()->alloc(sizeof(T) * (size_t)pe, false);
        }
        R->roff.clear();
        for (size_t x = 0; x < E.L.rows[r].size(); x++)  // (pieces are 256-byte aligned allocations)
            R->roff.push_back(((int64_t)R->store[E.L.piece[r][x]]->p - (int64_t)R->store[0]->p) / (int64_t)sizeof(T) +
                              E.L.roff[r][x]);
        static const bool coarse = std::getenv("GPRX_DIST_COARSE") && std::atoi(std::getenv("GPRX_DIST_COARSE")) != 0;
        for (int p = 0; p < E.WL.npc; p++) {
            R->win.push_back(std::make_unique<DMem>());
            R->win.back()->alloc(sizeof(T) * (size_t)E.WL.piece_tiles(p) * DB2, !coarse);
        }
        dist_say(C.rank, "setup: store and window allocated, mailbox bytes", (long long)E.MB.bytes);
        R->mbox.alloc((size_t)E.MB.bytes, !coarse);
        dist_say(C.rank, "setup: mailbox allocated");
        GPRX_HIP(hipMemset(R->mbox.p, 0, E.MB.bytes));  // flags 0: below every epoch
        dist_say(C.rank, "setup: mailbox cleared");
        R->ctr.alloc(sizeof(int) * ((size_t)C_NCTL_DIST + nr + (size_t)nr * nci + nc + TP_STRIDE * (size_t)nc), false);
        if (potrf_split_for(std::is_same<T, double>::value, E.P)) R->pbuf.alloc(sizeof(T) * 4 * DB * DB, false);
        R->info.alloc(160 * sizeof(int), false);  // info, then the GPRX_DIST_CHECK counters and log
        GPRX_HIP(hipMemset(R->info.p, 0, 160 * sizeof(int)));
        R->flag.alloc(sizeof(int), false);
        R->red.alloc(sizeof(double) * 4 + sizeof(TileBuild<T>) + 64, false);
        R->sctl.alloc(sizeof(int) * 8, false);
        R->part.alloc(sizeof(double) * MAX_LEAF * 3 * (size_t)nc * (nc + 1) / 2 + 64, false);
        E.ranks.push_back(std::move(R));
    }
    // ---- every rank's mailbox and storage as mapped in this process ------------------------------
    auto own_view = [](const DistRank<T>& Q, std::vector<uint64_t>& st, std::vector<uint64_t>& wp) {
        st.clear();
        wp.clear();
        for (auto& p : Q.store) st.push_back((uint64_t)p->p);
        for (auto& p : Q.win) wp.push_back((uint64_t)p->p);
    };
    for (auto& R : E.ranks) {
        R->mb.assign(E.g, 0);
        R->st.assign(E.g, {});
        R->wp.assign(E.g, {});
    }
    if (E.virt) {
        for (auto& R : E.ranks)
            for (auto& Q : E.ranks) {
                R->mb[Q->r] = (uint64_t)Q->mbox.p;
                own_view(*Q, R->st[Q->r], R->wp[Q->r]);
            }
    } else {
        DistRank<T>& R = *E.ranks[0];
        R.mb[R.r] = (uint64_t)R.mbox.p;
        own_view(R, R.st[R.r], R.wp[R.r]);
        if (E.g > 1) {
            // every allocation a peer reads or writes, one IPC handle each, every one below 2 GiB
            // (hipIpcOpenMemHandle of a larger allocation never returned on this stack: DESIGN.md 6):
            // [mailbox, window pieces, storage pieces]; the layout (identical on every rank) tells
            // how many of each a rank has
            size_t maxsp = 0;
            for (int q = 0; q < E.g; q++) maxsp = std::max(maxsp, E.L.pelems[q].size());
            const size_t nh = 1 + (size_t)E.WL.npc + maxsp;
            GPRX_REQUIRE(E.hc, GPRX_ERR_STATE, "distributed fit: no host collective");
            std::vector<hipIpcMemHandle_t> mine(nh);
            std::memset(mine.data(), 0, sizeof(hipIpcMemHandle_t) * nh);
            GPRX_HIP(hipIpcGetMemHandle(&mine[0], R.mbox.p));
            for (int p = 0; p < E.WL.npc; p++) GPRX_HIP(hipIpcGetMemHandle(&mine[1 + p], R.win[p]->p));
            for (size_t p = 0; p < R.store.size(); p++)
                GPRX_HIP(hipIpcGetMemHandle(&mine[1 + E.WL.npc + p], R.store[p]->p));
            std::vector<hipIpcMemHandle_t> all(nh * (size_t)E.g);
            dist_say(C.rank, "setup: ipc handles taken", (long long)nh);
            E.hc->allgather(mine.data(), sizeof(hipIpcMemHandle_t) * nh, all.data());
            dist_say(C.rank, "setup: ipc handles exchanged");
            auto open = [&](const hipIpcMemHandle_t& h) {
                void* p = nullptr;
                GPRX_HIP(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
                R.opened.push_back(p);
                return (uint64_t)p;
            };
            for (int q = 0; q < E.g; q++) {
                if (q == R.r) continue;
                const hipIpcMemHandle_t* hq = all.data() + nh * (size_t)q;
                R.mb[q] = open(hq[0]);
                for (int p = 0; p < E.WL.npc; p++) R.wp[q].push_back(open(hq[1 + p]));
                for (size_t p = 0; p < E.L.pelems[q].size(); p++) R.st[q].push_back(open(hq[1 + E.WL.npc + p]));
                dist_say(C.rank, "setup: ipc handles opened, rank", q);
            }
        }
    }
    // ---- tables -------------------------------------------------------------------------------
    std::vector<int> lastof(E.g, -1);
    for (int q = 0; q < E.g; q++)
        for (int i : E.L.rows[q])
            if (i < nc) lastof[q] = std::max(lastof[q], i);
    for (auto& Rp : E.ranks) {
        DistRank<T>& R = *Rp;
        const int r = R.r;
        std::vector<int> loc(nr, -1);
        for (int i = 0; i < nr; i++)
            if (E.L.own[i] == r) loc[i] = E.L.loc[i];
        std::vector<uint64_t> tptr((size_t)nr * nc, 0);
        if (E.g > 1)
            for (int j = 0; j < nr; j++)
                for (int b = 0; b < nc; b++) {
                    const int64_t t = (int64_t)(b % ww) * nr + j;
                    tptr[(size_t)j * nc + b] = R.wp[r][t / E.WL.tpp] + (uint64_t)((t % E.WL.tpp) * DB2 * (int64_t)sizeof(T));
                }
        std::vector<uint64_t> wpc((size_t)E.g * std::max(1, E.WL.npc), 0);  // every rank's window pieces
        for (int q = 0; q < E.g; q++)
            for (int p = 0; p < E.WL.npc; p++) wpc[(size_t)q * E.WL.npc + p] = R.wp[q][p];
        R.orows.clear();
        for (int i : E.L.rows[r])
            if (i < nc) R.orows.push_back(i);
        upload_vec(R.t_loc, loc);
        upload_vec(R.t_roff, R.roff);
        upload_vec(R.t_wpc, wpc);
        // the posterior solve's V_k(c) slots: tile t = c nc + k of every rank's window
        if (E.g > 1 && E.pv_nch > 0) {
            std::vector<uint64_t> vs((size_t)E.g * E.pv_nch * nc);
            for (int q = 0; q < E.g; q++)
                for (int c = 0; c < E.pv_nch; c++)
                    for (int k = 0; k < nc; k++) {
                        const int64_t t = (int64_t)c * nc + k;
                        vs[((size_t)q * E.pv_nch + c) * nc + k] =
                            R.wp[q][t / E.WL.tpp] + (uint64_t)((t % E.WL.tpp) * DB2 * (int64_t)sizeof(T));
                    }
            upload_vec(R.t_vslot, vs);
        }
        upload_vec(R.t_own, E.L.own);
        upload_vec(R.t_tptr, tptr);
        upload_vec(R.t_cons, E.S.cons);
        upload_vec(R.t_need, E.S.need);
        upload_vec(R.t_mb, R.mb);
        upload_vec(R.t_orows, R.orows);
        upload_vec(R.t_lastof, lastof);
        R.pd.alloc(sizeof(PtDist<T>), false);
        const std::vector<int4>& lst = E.S.lists[r];
        R.ntasks = (int)lst.size();
        upload_vec(R.list, lst);
        if (inv) {  // C tile (ti, tj) of this rank's identity rows, for the gradient pass
            std::vector<uint64_t> ctab((size_t)nc * nc, 0);
            for (int a = 0; a < nc; a++) {
                const int i = nc + 1 + a;
                if (E.L.own[i] != r) continue;
                for (int c = 0; c <= a; c++)
                    ctab[(size_t)a * nc + c] = (uint64_t)(R.sbase() + R.roff[E.L.loc[i]] + (int64_t)(nc - a + c) * DB2);
            }
            upload_vec(R.t_ctab, ctab);
        }
    }
    E.key_n = n;
    E.key_m = m;
    E.key_fused = fused;
    E.key_inv = inv;
}

template <typename T>
static PtDist<T> make_ptdist(const DistEngine<T>& E, const DistRank<T>& R) {
    PtDist<T> pd;
    std::memset(&pd, 0, sizeof(pd));
    pd.g = E.g;
    pd.r = R.r;
    pd.nc = E.L.nc;
    pd.nr = E.L.nr;
    pd.ww = E.ww;
    pd.nci = E.L.nci;
    pd.ep = E.ep;
    pd.loc = R.t_loc.template as<int>();
    pd.roff = R.t_roff.template as<int64_t>();
    pd.own = R.t_own.template as<int>();
    pd.tptr = R.t_tptr.template as<uint64_t>();
    pd.cons = R.t_cons.template as<unsigned char>();
    pd.need = R.t_need.template as<int>();
    pd.ucnt = R.ctr.template as<int>() + C_NCTL_DIST + E.L.nr + (size_t)E.L.nr * E.L.nci;
    pd.mb = R.t_mb.template as<uint64_t>();
    pd.o_linv = E.MB.o_linv;
    pd.wpc = R.t_wpc.template as<uint64_t>();
    pd.tpp = E.WL.tpp;
    pd.npc = E.WL.npc;
    pd.o_z = E.MB.o_z;
    pd.o_flags = E.MB.o_flags;
    pd.o_tags = E.MB.o_tags;
    pd.check = std::getenv("GPRX_DIST_CHECK") != nullptr ? 1 : 0;
    // ranks on one device (virtual, or processes sharing a GPU) read each other's pushes through
    // the shared L2s: plain stores + one release per push measured 3-6% faster there (C3, 2-8
    // virtual ranks) than written-through stores; across devices the release would write back
    // every dirty line of the producer's L2 for a tile that lives on another GPU
    pd.wt = (E.virt || E.shared_dev) ? 0 : 1;
    if (const char* e = std::getenv("GPRX_DIST_WT")) pd.wt = std::atoi(e) != 0;
    pd.acq_agent = 0;
    if (const char* e = std::getenv("GPRX_DIST_ACQ_AGENT")) pd.acq_agent = std::atoi(e) != 0;
    pd.check_err = R.info.template as<int>() + 1;
    return pd;
}

template <typename T>
static DSArgs<T> make_dsargs(const DistEngine<T>& E, const DistRank<T>& R) {
    DSArgs<T> a;
    std::memset(&a, 0, sizeof(a));
    a.g = E.g;
    a.r = R.r;
    a.nc = E.L.nc;
    a.m = E.m;
    a.own = R.t_own.template as<int>();
    a.loc = R.t_loc.template as<int>();
    a.roff = R.t_roff.template as<int64_t>();
    a.store = R.sbase();
    a.orows = R.t_orows.template as<int>();
    a.nown = (int)R.orows.size();
    a.last_of = R.t_lastof.template as<int>();
    a.last_own = R.orows.empty() ? -1 : R.orows.back();
    a.Linv = reinterpret_cast<const T*>(R.mbox.template as<char>() + E.MB.o_linv);
    a.mb = R.t_mb.template as<uint64_t>();
    a.o_ztile = E.MB.o_z;
    a.o_alpha = E.MB.o_alpha;
    a.o_zf = E.MB.o_zf;
    a.o_part = E.MB.o_part;
    a.o_fflags = E.MB.o_flags;
    a.o_sflags = E.MB.o_sflags;
    a.fit_ep = E.ep;
    a.sep = E.sep;
    a.ctl = R.sctl.template as<int>();
    a.info = R.info.template as<int>();
    a.tlimit = (long long)(1e8 * 4.0);
    return a;
}

// ---------------------------------------------------------------------------------------
// the fit
// ---------------------------------------------------------------------------------------
template <typename T>
void dist_fit(DistEngineBase*& eng, const DistContext& C, const DistFitIn<T>& in, DistFitOut& out, T* alpha_dev) {
    if (!eng) eng = new DistEngine<T>();
    DistEngine<T>* Ep = dynamic_cast<DistEngine<T>*>(eng);
    if (!Ep) {  // the model changed scalar type
        delete eng;
        eng = Ep = new DistEngine<T>();
    }
    DistEngine<T>& E = *Ep;
    const bool fused = in.tb.mode != 0;
    setup<T>(E, C, in.n, in.m, fused, in.inv);
    dist_say(C.rank, "fit: setup done", in.inv ? 1 : 0);
    const int nc = E.L.nc, nr = E.L.nr, nci = E.L.nci;
    const int64_t np = E.np, n = in.n;
    const int64_t DB2 = (int64_t)DB * DB;
    E.ep++;
    // ---- per rank: counters, storage, then the launches ------------------------------------------
    std::vector<DistLaunch<T>> launches(E.ranks.size());
    for (size_t v = 0; v < E.ranks.size(); v++) {
        DistRank<T>& R = *E.ranks[v];
        const int r = R.r;
        hipStream_t s = R.s;
        const size_t nctr = (size_t)C_NCTL_DIST + nr + (size_t)nr * nci + nc + TP_STRIDE * (size_t)nc;  // + split-step states
        GPRX_HIP(hipMemsetAsync(R.ctr.p, 0, sizeof(int) * nctr, s));
        int* lcnt = R.ctr.template as<int>() + C_NCTL_DIST;
        hipLaunchKernelGGL(dist_init_counters, dim3((unsigned)nr), dim3(256), 0, s, lcnt, lcnt + nr, nc, nr, nci,
                           fused ? 1 : 0);
        GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)R.info.p, INT_MAX, 1, s));
        GPRX_HIP(hipMemsetAsync(R.flag.p, 0, sizeof(int), s));
        T* A = R.sbase();
        for (int x = 0; x < (int)E.L.rows[r].size(); x++) {
            const int i = E.L.rows[r][x];
            T* base = A + R.roff[x];
            if (i == nc) {  // the label rows: Y^T as row block nc (DB x np, ld DB)
                launch_label_rows<T>(in.Y, n, in.m, base, DB, 0, np, GT, s);
            } else if (i > nc) {  // identity row block of the inverse (LML mode)
                const int64_t e = (int64_t)E.L.ncols(i) * DB2;
                hipLaunchKernelGGL(dist_init_identity<T>, dim3((unsigned)((e + 255) / 256)), dim3(256), 0, s, base,
                                   E.L.ncols(i));
            } else if (!fused) {  // the direct build: row block i against the columns up to its diagonal
                const int64_t r0 = (int64_t)i * DB, rows = std::min<int64_t>(DB, n - r0), cols = std::min<int64_t>(r0 + DB, n);
                GPRX_HIP(hipMemsetAsync(base, 0, sizeof(T) * (size_t)E.L.ncols(i) * DB2, s));
                if (rows > 0) {
                    const T *tabr = nullptr, *tabc = nullptr;
                    DMem tab;
                    if (in.K.nper > 0) {  // sin/cos tables of the block's rows and of its columns
                        const size_t slot = (size_t)2 * in.K.nper * in.d;
                        tab.alloc(sizeof(T) * slot * ((size_t)DB + (size_t)n), false);
                        T* tr = tab.as<T>();
                        T* tc = tr + slot * DB;
                        launch_sincos_tables<T>(in.K, in.X + r0 * in.d, rows, in.d, tr, s);
                        launch_sincos_tables<T>(in.K, in.X, cols, in.d, tc, s);
                        tabr = tr;
                        tabc = tc;
                    }
                    launch_kbuild<T>(in.K, in.X + r0 * in.d, tabr, rows, in.X, tabc, cols, in.d, base, DB, 0, false, T(0),
                                     R.flag.template as<int>(), s);
                    if (tab.p) GPRX_HIP(hipStreamSynchronize(s));  // before the tables are freed
                }
                hipLaunchKernelGGL(dist_diag_fix<T>, dim3(1), dim3(DB), 0, s, base + (int64_t)i * DB2, r0, n, in.sigma2);
            }
        }
        const PtDist<T> pd = make_ptdist(E, R);
        GPRX_HIP(hipMemcpyAsync(R.pd.p, &pd, sizeof(pd), hipMemcpyHostToDevice, s));
        void* tbdev = nullptr;
        if (fused) {
            TileBuild<T> tbl = in.tb;
            tbl.flag = R.flag.template as<int>();
            tbdev = static_cast<char*>(R.red.p) + 64;
            GPRX_HIP(hipMemcpyAsync(tbdev, &tbl, sizeof(tbl), hipMemcpyHostToDevice, s));
        }
        GPRX_HIP(hipStreamSynchronize(s));  // pageable copies done before any rank's persistent launch
        DistLaunch<T>& Lc = launches[v];
        Lc.A = A;
        Lc.Linv = reinterpret_cast<T*>(R.mbox.template as<char>() + E.MB.o_linv);
        Lc.info = R.info.template as<int>();
        Lc.list = R.list.template as<int4>();
        Lc.ntasks = R.ntasks;
        Lc.nc = nc;
        Lc.nr = nr;
        Lc.nci = nci;
        Lc.ctr = R.ctr.template as<int>();
        Lc.tb_dev = reinterpret_cast<const TileBuild<T>*>(tbdev);
        Lc.dist_dev = R.pd.template as<PtDist<T>>();
        Lc.tlimit = (long long)(1e8 * (2.0 + 20.0 * E.S.est_us * 1e-6));
        Lc.P = E.P;
        Lc.s = s;
        Lc.dbg = nullptr;
        static const bool dbg_on = std::getenv("GPRX_PT_DEBUG") != nullptr;
        if (dbg_on && E.ranks.size() == 1) {  // {ticket, phase, i, j} per workgroup, read by gprx_dev_pt_debug
            if (E.dbg_n < E.P) {
                E.free_dbg();
                GPRX_HIP(hipHostMalloc((void**)&E.dbg, sizeof(int) * 4 * E.P, hipHostMallocCoherent));
                E.dbg_n = E.P;
            }
            std::memset(E.dbg, 0xff, sizeof(int) * 4 * E.P);
            pt_debug_register(E.dbg, E.P);
            Lc.dbg = E.dbg;
        }
        Lc.trace = nullptr;
        Lc.split = potrf_split_for(std::is_same<T, double>::value, E.P) ? 1 : 0;
        Lc.pbuf = R.pbuf.template as<T>();
        Lc.tflag = R.ctr.template as<int>() + C_NCTL_DIST + nr + (size_t)nr * nci + nc;
        if (std::getenv("GPRX_DIST_TRACE_FILE")) {  // {taken, ready, published, workgroup} per ticket
            const size_t tb = sizeof(long long) * 4 * ((size_t)R.ntasks + 2 * (size_t)nc);
            if (R.trace.bytes < tb) R.trace.alloc(tb, false);
            Lc.trace = R.trace.template as<long long>();
        }
    }
    // every process has prepared its storage: the persistent launches start together (a rank's
    // waits on its peers' pushes are time-limited per wait, the processes' arrival is not)
    host_barrier(E);
    // every rank's persistent launch back to back, nothing that could block in between
    dist_say(C.rank, "fit: launching");
    for (size_t v = 0; v < E.ranks.size(); v++) {
        GPRX_HIP(hipEventRecord(E.ranks[v]->t0, E.ranks[v]->s));
        potrf_tiles_dist_launch<T>(launches[v]);
        GPRX_HIP(hipEventRecord(E.ranks[v]->t1, E.ranks[v]->s));
    }
    for (auto& R : E.ranks) GPRX_HIP(hipStreamSynchronize(R->s));
    GPRX_HIP(hipGetLastError());
    if (const char* tf = std::getenv("GPRX_DIST_TRACE_FILE")) {
        // one file per rank (overwritten each fit): int32 ntasks, int32 rank, int32 g, int32 nc,
        // then the ticket list (int4 per ticket) and the timeline (4 int64 per ticket, 100 MHz)
        for (auto& Rp : E.ranks) {
            DistRank<T>& R = *Rp;
            std::vector<long long> tm((size_t)4 * R.ntasks);
            GPRX_HIP(hipMemcpy(tm.data(), R.trace.p, sizeof(long long) * tm.size(), hipMemcpyDeviceToHost));
            const std::string path = std::string(tf) + ".r" + std::to_string(R.r);
            if (FILE* f = std::fopen(path.c_str(), "wb")) {
                const int hdr[4] = {R.ntasks, R.r, E.g, nc};
                std::fwrite(hdr, sizeof(hdr), 1, f);
                std::fwrite(E.S.lists[R.r].data(), sizeof(int4), E.S.lists[R.r].size(), f);
                std::fwrite(tm.data(), sizeof(long long), tm.size(), f);
                std::fclose(f);
            }
        }
    }
    // ---- reductions: log det, data fit, status (one small all-gather over the processes) --------
    struct Part {
        double logdet, datafit;
        int info, flag;
    };
    Part tot{0, 0, INT_MAX, 0};
    if (std::getenv("GPRX_DIST_CHECK"))  // the window-slot verification's findings (PtDist::check)
        for (auto& Rp : E.ranks) {
            int ce[3 + 1 + 128];
            GPRX_HIP(hipMemcpy(ce, Rp->info.template as<int>() + 1, sizeof(ce), hipMemcpyDeviceToHost));
            if (ce[0] || ce[1]) {
                std::fprintf(stderr, "gprx dist check rank %d fit %u: %d stale window reads, %d slots overwritten during a read:",
                             Rp->r, E.ep, ce[0], ce[1]);
                for (int e = 0; e < std::min(ce[2], 32); e++)
                    std::fprintf(stderr, " [%s: row %d panel %d]", ce[4 + 4 * e] ? "during" : "stale", ce[5 + 4 * e],
                                 ce[6 + 4 * e]);
                std::fprintf(stderr, "\n");
            }
            GPRX_HIP(hipMemset(Rp->info.template as<int>() + 1, 0, sizeof(ce)));
        }
    for (auto& Rp : E.ranks) {
        DistRank<T>& R = *Rp;
        DSArgs<T> a = make_dsargs(E, R);
        launch_dist_reduce<T>(a, n, R.red.template as<double>(), R.s);
        double red[2];
        int hi = 0, hf = 0;
        GPRX_HIP(hipMemcpyAsync(red, R.red.p, sizeof(red), hipMemcpyDeviceToHost, R.s));
        GPRX_HIP(hipMemcpyAsync(&hi, R.info.p, sizeof(int), hipMemcpyDeviceToHost, R.s));
        GPRX_HIP(hipMemcpyAsync(&hf, R.flag.p, sizeof(int), hipMemcpyDeviceToHost, R.s));
        GPRX_HIP(hipStreamSynchronize(R.s));
        tot.logdet += red[0];
        tot.datafit += red[1];
        tot.info = std::min(tot.info, hi);
        tot.flag = std::max(tot.flag, hf);
    }
    if (tot.info != INT_MAX && tot.info < 0)  // a timed-out wait: where each rank stood
        for (auto& Rp : E.ranks) {
            int rec[8], tk = 0;
            GPRX_HIP(hipMemcpy(rec, Rp->info.template as<int>() + 1 + 132, sizeof(rec), hipMemcpyDeviceToHost));
            GPRX_HIP(hipMemcpy(&tk, Rp->ctr.p, sizeof(int), hipMemcpyDeviceToHost));
            std::fprintf(stderr,
                         "gprx dist timeout rank %d/%d fit %u: tickets %d of %d; first timed-out wait: kind %d type %d "
                         "i %d j %d b0 %d nb %d detail 0x%x seen %d (ww %d gb %d P %d)\n",
                         Rp->r, E.g, E.ep, tk, Rp->ntasks, rec[0], rec[1], rec[2], rec[3], rec[4] & 0xffff, rec[4] >> 16,
                         rec[5], rec[6], E.ww, E.gb, E.P);
            GPRX_HIP(hipMemset(Rp->info.template as<int>() + 1 + 132, 0, sizeof(rec)));
        }
    if (!E.virt && E.g > 1) {  // across the processes (rank order: identical sums everywhere)
        std::vector<Part> all(E.g);
        E.hc->allgather(&tot, sizeof(Part), all.data());
        tot = Part{0, 0, INT_MAX, 0};
        for (const Part& p : all) {
            tot.logdet += p.logdet;
            tot.datafit += p.datafit;
            tot.info = std::min(tot.info, p.info);
            tot.flag = std::max(tot.flag, p.flag);
        }
    }
    out.logdet = tot.logdet;
    out.datafit = tot.datafit;
    out.info = tot.info;
    out.flag = tot.flag;
    out.est_us = E.S.est_us;
    out.P = E.P;
    out.gb = E.gb;
    out.ww = E.ww;
    out.chunk_w = E.W;
    out.ms_kernel = 0;
    out.bytes_rank = 0;
    out.bytes_storage = 0;
    {  // the pushes of this process's first rank, from the layout and the schedule's consumers
        const int r0 = E.ranks.front()->r;
        int64_t nl = 0, nt = 0;
        for (int i = 0; i < nc; i++) {
            if (E.L.own[i] != r0) continue;
            nl += E.g - 1;  // Linv_i to every peer
            int peers = 0;
            for (int q = 0; q < E.g; q++) peers += (q != r0 && E.S.cons[(size_t)q * nr + i]) ? 1 : 0;
            nt += (int64_t)peers * i;  // the final tiles L_ib, b < i
        }
        out.push_rank = r0;
        out.push_linv = nl;
        out.push_tiles = nt;
        out.push_bytes = (nl + nt) * (int64_t)DB * DB * (int64_t)sizeof(T);
    }
    for (auto& Rp : E.ranks) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, Rp->t0, Rp->t1) == hipSuccess) out.ms_kernel = std::max(out.ms_kernel, (double)ms);
        const int64_t b = Rp->store_bytes() + Rp->win_bytes() +
                          (int64_t)(Rp->mbox.bytes + Rp->ctr.bytes + Rp->part.bytes + Rp->pbuf.bytes + Rp->t_tptr.bytes +
                                    Rp->t_cons.bytes + Rp->t_need.bytes + Rp->list.bytes + Rp->t_ctab.bytes);
        out.bytes_rank = std::max(out.bytes_rank, b);
        out.bytes_storage = std::max(out.bytes_storage, Rp->store_bytes());
    }
    if (tot.info != INT_MAX || tot.flag) return;  // the caller reports it
    // ---- alpha = L^{-T} z: the distributed back substitution ---------------------------------
    E.sep++;
    const auto ts0 = std::chrono::steady_clock::now();
    for (auto& Rp : E.ranks) {
        DistRank<T>& R = *Rp;
        GPRX_HIP(hipMemsetAsync(R.sctl.p, 0, sizeof(int) * 8, R.s));
        GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)R.info.p, INT_MAX, 1, R.s));
    }
    for (auto& Rp : E.ranks) {
        DSArgs<T> a = make_dsargs(E, *Rp);
        a.zmode = 0;
        launch_dist_back<T>(a, Rp->s);
    }
    int hinfo = INT_MAX;
    for (auto& Rp : E.ranks) {
        int hi = 0;
        GPRX_HIP(hipMemcpyAsync(&hi, Rp->info.p, sizeof(int), hipMemcpyDeviceToHost, Rp->s));
        GPRX_HIP(hipStreamSynchronize(Rp->s));
        hinfo = std::min(hinfo, hi);
    }
    hinfo = agree_min(E, hinfo);  // every process reports the same outcome
    out.ms_solve = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - ts0).count();
    if (hinfo != INT_MAX) {
        out.info = -1;
        return;
    }
    const DistRank<T>& R0 = *E.ranks[0];
    copy_from_mailbox<T>(R0.mbox.template as<char>() + E.MB.o_alpha, alpha_dev, np * E.m, R0.s);
    GPRX_HIP(hipStreamSynchronize(R0.s));
}

// ---------------------------------------------------------------------------------------
// solves with the sharded factor (the fp32 refinement's correction)
// ---------------------------------------------------------------------------------------
template <typename T>
void dist_solve(DistEngineBase* eng, const T* rhs, T* out, hipStream_t s) {
    auto* Ep = dynamic_cast<DistEngine<T>*>(eng);
    GPRX_REQUIRE(Ep && !Ep->ranks.empty(), GPRX_ERR_STATE, "distributed solve: no factor");
    DistEngine<T>& E = *Ep;
    GPRX_HIP(hipStreamSynchronize(s));  // rhs written on the caller's stream
    host_barrier(E);                    // as before a fit: the ranks' solve launches start together
    E.sep++;
    for (auto& Rp : E.ranks) {
        GPRX_HIP(hipMemsetAsync(Rp->sctl.p, 0, sizeof(int) * 8, Rp->s));
        GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)Rp->info.p, INT_MAX, 1, Rp->s));
    }
    for (auto& Rp : E.ranks) {
        DSArgs<T> a = make_dsargs(E, *Rp);
        a.rhs = rhs;
        launch_dist_forward<T>(a, Rp->s);
    }
    for (auto& Rp : E.ranks) GPRX_HIP(hipMemsetAsync(Rp->sctl.p, 0, sizeof(int) * 8, Rp->s));
    for (auto& Rp : E.ranks) {
        DSArgs<T> a = make_dsargs(E, *Rp);
        a.zmode = 1;
        launch_dist_back<T>(a, Rp->s);
    }
    int hinfo = INT_MAX;
    for (auto& Rp : E.ranks) {
        int hi = 0;
        GPRX_HIP(hipMemcpyAsync(&hi, Rp->info.p, sizeof(int), hipMemcpyDeviceToHost, Rp->s));
        GPRX_HIP(hipStreamSynchronize(Rp->s));
        hinfo = std::min(hinfo, hi);
    }
    if (agree_min(E, hinfo) != INT_MAX) throw Error{GPRX_ERR_HIP, "gprx: distributed solve timed out (flag wait)"};
    const DistRank<T>& R0 = *E.ranks[0];
    copy_from_mailbox<T>(R0.mbox.template as<char>() + E.MB.o_alpha, out, E.np * E.m, s);
}
template void dist_solve<double>(DistEngineBase*, const double*, double*, hipStream_t);
template void dist_solve<float>(DistEngineBase*, const float*, float*, hipStream_t);

// ---------------------------------------------------------------------------------------
// the dense factor on this process (posterior covariance, core matrix): a documented gather
// ---------------------------------------------------------------------------------------
template <typename T>
void dist_gather_factor(DistEngineBase* eng, T* A, int64_t ld, T* Linv, hipStream_t s) {
    auto* Ep = dynamic_cast<DistEngine<T>*>(eng);
    GPRX_REQUIRE(Ep && !Ep->ranks.empty(), GPRX_ERR_STATE, "distributed fit: no factor");
    DistEngine<T>& E = *Ep;
    const DistRank<T>& R0 = *E.ranks[0];
    const int nc = E.L.nc;
    const int64_t DB2 = (int64_t)DB * DB;
    std::vector<uint64_t> src((size_t)nc * nc, 0);
    for (int i = 0; i < nc; i++) {
        const int q = E.L.own[i], x = E.L.loc[i];
        const uint64_t base = R0.st[q][E.L.piece[q][x]];  // the piece of row block i, as mapped here
        for (int j = 0; j < i; j++) src[(size_t)i * nc + j] = base + sizeof(T) * (uint64_t)(E.L.roff[q][x] + (int64_t)j * DB2);
    }
    DMem tab;
    upload_vec(tab, src);
    GPRX_HIP(hipMemsetAsync(A, 0, sizeof(T) * (size_t)ld * nc * DB, s));
    if (nc > 1)
        hipLaunchKernelGGL(dist_gather_kernel<T>, dim3((unsigned)nc, (unsigned)nc), dim3(256), 0, s,
                           tab.as<uint64_t>(), nc, A, ld);
    copy_from_mailbox<T>(R0.mbox.template as<char>() + E.MB.o_linv, Linv, (int64_t)nc * DB2, s);
    GPRX_HIP(hipStreamSynchronize(s));
    GPRX_HIP(hipGetLastError());
    host_barrier(E);  // no peer rewrites its storage (the next fit) while this process still reads it
}
template void dist_gather_factor<double>(DistEngineBase*, double*, int64_t, double*, hipStream_t);
template void dist_gather_factor<float>(DistEngineBase*, float*, int64_t, float*, hipStream_t);

// ---------------------------------------------------------------------------------------
// posterior covariance with the sharded factor: k(x, y) - (L^{-1} k_x) . (L^{-1} k_y) with no
// rank holding more than its own rows of L (GaussianProcess::operator() / GetCredibleInterval,
// lib/GaussianProcess.cpp:84-114; the reference uses C = K^{-1}, the same quantity)
// ---------------------------------------------------------------------------------------
namespace {
// out[j] = sum over the rows li < nown of part[li][j] (fixed order)
__global__ void pv_rowsum(const double* __restrict__ part, int nown, int64_t nq, double* __restrict__ out) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nq) return;
    double v = 0;
    for (int li = 0; li < nown; li++) v += part[(int64_t)li * nq + j];
    out[j] = v;
}
}  // namespace

template <typename T>
static int pv_chunks_of(DistEngineBase* eng) {
    auto* E = dynamic_cast<DistEngine<T>*>(eng);
    return (E && !E->ranks.empty()) ? E->pv_nch : -1;
}
int dist_pvar_chunks(DistEngineBase* eng) {
    int v = pv_chunks_of<double>(eng);
    if (v < 0) v = pv_chunks_of<float>(eng);
    return std::max(0, v);
}

template <typename T>
static int64_t pv_bytes_of(DistEngineBase* eng) {
    auto* E = dynamic_cast<DistEngine<T>*>(eng);
    if (!E) return -1;
    int64_t b = 0;
    for (auto& Rp : E->ranks) b = std::max<int64_t>(b, (int64_t)Rp->pvR.bytes);
    return b;
}
int64_t dist_pvar_bytes(DistEngineBase* eng) {
    int64_t v = pv_bytes_of<double>(eng);
    if (v < 0) v = pv_bytes_of<float>(eng);
    return std::max<int64_t>(0, v);
}

template <typename T>
void dist_posterior(DistEngineBase* eng, const KCanon<T>& K, const T* X, const T* tabX, int64_t n, int d, const T* Z,
                    const T* tabZ, int nch, bool pairs, std::vector<double>& sum, hipStream_t s) {
    auto* Ep = dynamic_cast<DistEngine<T>*>(eng);
    GPRX_REQUIRE(Ep && !Ep->ranks.empty() && Ep->pv_nch > 0, GPRX_ERR_STATE, "distributed posterior: no sharded factor");
    DistEngine<T>& E = *Ep;
    GPRX_REQUIRE(nch >= 1 && nch <= E.pv_nch, GPRX_ERR_ARG, "distributed posterior: too many query chunks");
    const int nc = E.L.nc;
    const int64_t nq = (int64_t)nch * DB;
    (void)tabX;
    // per rank: K(Z, X_own), nq x (own row blocks x 128), ld nq -- only the rank's own training rows
    // (packed in orows order; the padding columns >= n stay zero); each task overwrites its block's
    // columns with W = K - sum L V.  X_own is gathered from X and gets its own sin/cos tables.
    int* nfl = E.ranks[0]->flag.template as<int>();
    GPRX_HIP(hipMemsetAsync(nfl, 0, sizeof(int), s));
    for (auto& Rp : E.ranks) {
        DistRank<T>& Rk = *Rp;
        const int64_t nown = (int64_t)Rk.orows.size();
        if (nown == 0) continue;
        const size_t rb = sizeof(T) * (size_t)nq * nown * DB;
        if (Rk.pvR.bytes < rb) Rk.pvR.alloc(rb, false);
        if (Rk.pvX.bytes < sizeof(T) * (size_t)nown * DB * d) Rk.pvX.alloc(sizeof(T) * (size_t)nown * DB * d, false);
        T* Xo = Rk.pvX.template as<T>();
        int64_t nvalid = 0;
        for (int64_t li = 0; li < nown; li++) {
            const int64_t r0 = (int64_t)Rk.orows[li] * DB, cnt = std::min<int64_t>(DB, n - r0);
            if (cnt <= 0) continue;
            // (own blocks are full but possibly the last one, nc - 1, which comes last in orows)
            GPRX_HIP(hipMemcpyAsync(Xo + li * DB * d, X + r0 * d, sizeof(T) * cnt * d, hipMemcpyDeviceToDevice, s));
            nvalid = li * DB + cnt;
        }
        const T* tabo = nullptr;
        if (K.nper > 0) {
            const size_t tb = sizeof(T) * 2 * K.nper * (size_t)std::max<int64_t>(nvalid, 1) * d;
            if (Rk.pvTab.bytes < tb) Rk.pvTab.alloc(tb, false);
            launch_sincos_tables<T>(K, Xo, nvalid, d, Rk.pvTab.template as<T>(), s);
            tabo = Rk.pvTab.template as<T>();
        }
        GPRX_HIP(hipMemsetAsync(Rk.pvR.p, 0, rb, s));
        launch_kbuild<T>(K, Z, tabZ, nq, Xo, tabo, nvalid, d, Rk.pvR.template as<T>(), nq, 0, false, T(0), nfl, s);
    }
    // (non-finite query kernel values are not an error: the reference's ComputeKernelVectorInternal
    // has no check, lib/GaussianProcess.cpp:684-693, and its operator() returns the NaN, as the
    // single-GPU path does; the flag the build raises is cleared here and by the next fit)
    GPRX_HIP(hipMemsetAsync(nfl, 0, sizeof(int), s));
    GPRX_HIP(hipStreamSynchronize(s));
    host_barrier(E);  // every rank's previous use of its window (a fit, an earlier batch) is over
    E.vep++;
    for (auto& Rp : E.ranks) {
        DistRank<T>& Rk = *Rp;
        const size_t pb = sizeof(double) * std::max<size_t>(1, Rk.orows.size()) * (size_t)nq;
        if (Rk.pvpart.bytes < pb) Rk.pvpart.alloc(pb, false);
        if (Rk.pvsum.bytes < sizeof(double) * (size_t)nq) Rk.pvsum.alloc(sizeof(double) * (size_t)nq, false);
        GPRX_HIP(hipMemsetAsync(Rk.sctl.p, 0, sizeof(int) * 8, Rk.s));
        GPRX_HIP(hipMemsetD32Async((hipDeviceptr_t)Rk.info.p, INT_MAX, 1, Rk.s));
        PVArgs<T> a;
        std::memset(&a, 0, sizeof(a));
        a.g = E.g;
        a.r = Rk.r;
        a.nc = nc;
        a.loc = Rk.t_loc.template as<int>();
        a.roff = Rk.t_roff.template as<int64_t>();
        a.store = Rk.sbase();
        a.orows = Rk.t_orows.template as<int>();
        a.nown = (int)Rk.orows.size();
        a.Linv = reinterpret_cast<const T*>(Rk.mbox.template as<char>() + E.MB.o_linv);
        a.mb = Rk.t_mb.template as<uint64_t>();
        a.o_vflags = E.MB.o_vflags;
        a.vslot = Rk.t_vslot.template as<uint64_t>();
        a.vstride = E.pv_nch;
        a.R = Rk.pvR.template as<T>();
        a.nch = nch;
        a.pairs = pairs ? 1 : 0;
        a.ep = E.vep;
        a.part = Rk.pvpart.template as<double>();
        a.ctl = Rk.sctl.template as<int>();
        a.info = Rk.info.template as<int>();
        a.tlimit = (long long)(1e8 * 4.0);
        if (a.nown > 0) launch_dist_pvar<T>(a, E.P, Rk.s);
    }
    int hinfo = INT_MAX;
    for (auto& Rp : E.ranks) {
        int hi = 0;
        GPRX_HIP(hipMemcpyAsync(&hi, Rp->info.p, sizeof(int), hipMemcpyDeviceToHost, Rp->s));
        GPRX_HIP(hipStreamSynchronize(Rp->s));
        hinfo = std::min(hinfo, hi);
    }
    if (agree_min(E, hinfo) != INT_MAX) throw Error{GPRX_ERR_HIP, "gprx: distributed posterior solve timed out (flag wait)"};
    // this process's ranks' sums (rank order), then over the processes (rank order)
    sum.assign((size_t)nq, 0.0);
    std::vector<double> mine((size_t)nq);
    for (auto& Rp : E.ranks) {
        DistRank<T>& Rk = *Rp;
        if (Rk.orows.empty()) continue;
        hipLaunchKernelGGL(pv_rowsum, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, Rk.s,
                           Rk.pvpart.template as<double>(), (int)Rk.orows.size(), nq, Rk.pvsum.template as<double>());
        GPRX_HIP(hipMemcpyAsync(mine.data(), Rk.pvsum.p, sizeof(double) * nq, hipMemcpyDeviceToHost, Rk.s));
        GPRX_HIP(hipStreamSynchronize(Rk.s));
        for (int64_t j = 0; j < nq; j++) sum[j] += mine[j];
    }
    if (!E.virt && E.g > 1) {
        std::vector<double> all((size_t)nq * E.g);
        E.hc->allgather(sum.data(), sizeof(double) * nq, all.data());
        for (int64_t j = 0; j < nq; j++) {
            double v = 0;
            for (int q = 0; q < E.g; q++) v += all[(size_t)q * nq + j];
            sum[j] = v;
        }
    }
}
template void dist_posterior<double>(DistEngineBase*, const KCanon<double>&, const double*, const double*, int64_t, int,
                                     const double*, const double*, int, bool, std::vector<double>&, hipStream_t);
template void dist_posterior<float>(DistEngineBase*, const KCanon<float>&, const float*, const float*, int64_t, int,
                                    const float*, const float*, int, bool, std::vector<double>&, hipStream_t);

// ---------------------------------------------------------------------------------------
// LML gradient from the ranks' C tiles
// ---------------------------------------------------------------------------------------
template <typename T>
void dist_lml_grad(DistEngineBase* eng, const KCanon<T>& K, const KCanon<T>* Kd, const T* X, int64_t n, int d,
                   const T* FU, const T* FV, T* GU, T* GV, int64_t nf, const T* alpha, double* part, double* acc,
                   hipStream_t s) {
    auto* Ep = dynamic_cast<DistEngine<T>*>(eng);
    GPRX_REQUIRE(Ep && !Ep->ranks.empty() && Ep->key_inv, GPRX_ERR_STATE, "distributed gradient: no LML-mode factor");
    DistEngine<T>& E = *Ep;
    double tot[MAX_LEAF * 3] = {0};
    for (auto& Rp : E.ranks) {
        launch_lml_grad_mma<T>(K, Kd, X, n, d, FU, FV, GU, GV, nf, alpha, nullptr, 0, part, acc, s,
                               Rp->t_ctab.template as<uint64_t>());
        double p[MAX_LEAF * 3];
        GPRX_HIP(hipStreamSynchronize(s));
        GPRX_HIP(hipMemcpy(p, acc, sizeof(p), hipMemcpyDeviceToHost));
        for (int q = 0; q < MAX_LEAF * 3; q++) tot[q] += p[q];
    }
    GPRX_HIP(hipMemcpy(acc, tot, sizeof(tot), hipMemcpyHostToDevice));
    if (!E.virt && E.g > 1) hostcoll_allreduce_dev<double>(E.hc, acc, MAX_LEAF * 3, s);
}
template void dist_lml_grad<double>(DistEngineBase*, const KCanon<double>&, const KCanon<double>*, const double*, int64_t,
                                    int, const double*, const double*, double*, double*, int64_t, const double*,
                                    double*, double*, hipStream_t);
template void dist_lml_grad<float>(DistEngineBase*, const KCanon<float>&, const KCanon<float>*, const float*, int64_t,
                                   int, const float*, const float*, float*, float*, int64_t, const float*, double*,
                                   double*, hipStream_t);

template <typename T>
static bool own_blocks_of(DistEngineBase* eng, std::vector<int>& out) {
    auto* E = dynamic_cast<DistEngine<T>*>(eng);
    if (!E || E->ranks.empty()) return false;
    out.clear();
    for (auto& R : E->ranks)
        for (int i : R->orows) out.push_back(i);
    std::sort(out.begin(), out.end());
    return true;
}
std::vector<int> dist_own_blocks(DistEngineBase* eng) {
    std::vector<int> v;
    GPRX_REQUIRE(eng && (own_blocks_of<double>(eng, v) || own_blocks_of<float>(eng, v)), GPRX_ERR_STATE,
                 "distributed fit: no layout");
    return v;
}

template <typename T>
static bool allreduce_of(DistEngineBase* eng, double* dev, int count, hipStream_t s) {
    auto* E = dynamic_cast<DistEngine<T>*>(eng);
    if (!E) return false;
    if (!E->virt && E->g > 1) hostcoll_allreduce_dev<double>(E->hc, dev, count, s);
    return true;
}
void dist_allreduce_sum(DistEngineBase* eng, double* dev, int count, hipStream_t s) {
    GPRX_REQUIRE(eng && (allreduce_of<double>(eng, dev, count, s) || allreduce_of<float>(eng, dev, count, s)),
                 GPRX_ERR_STATE, "distributed fit: no engine");
}

void dist_engine_free(DistEngineBase* e) { delete e; }

template void dist_fit<double>(DistEngineBase*&, const DistContext&, const DistFitIn<double>&, DistFitOut&, double*);
template void dist_fit<float>(DistEngineBase*&, const DistContext&, const DistFitIn<float>&, DistFitOut&, float*);

}  // namespace gprx
