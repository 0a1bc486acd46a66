// gprx_dist.h — the storage-sharded multi-GPU fit (gprx_dist.cpp): interface used by the
// model code (gprx_api.cpp).
#pragma once
#include "gprx_internal.h"

namespace gprx {

constexpr int C_NCTL_DIST = 16;  // control words at the head of a tile launch's counter block (k_mma.h)

// Small host-side collectives between the processes of a distributed context: exchanging the
// mailboxes' IPC handles, and the per-fit reductions (log det, status) of a few bytes.  The bulk
// exchange never goes through here -- it is device-initiated (pushes into the peers' mailboxes).
struct HostColl {
    virtual ~HostColl() {}
    // recv (world * bytes) receives every rank's `send` in rank order
    virtual void allgather(const void* send, size_t bytes, void* recv) = 0;
};
// RCCL (ncclAllGather through a device staging buffer)
HostColl* make_rccl_coll(ncclComm_t comm, int world, int device);
// An RCCL call on a nonblocking communicator (gprx_ctx_create_dist creates it with
// config.blocking = 0 so that its initialisation can be time-limited): a result of
// ncclInProgress is polled with ncclCommGetAsyncError until it settles; a failure, or no
// result after `timeout_s`, throws GPRX_ERR_RCCL (the context's destruction then aborts the
// communicator: gprx_ctx_destroy uses ncclCommAbort, which never waits on the peers).
void rccl_settle(ncclComm_t comm, ncclResult_t r, const char* what, double timeout_s = 600.0);
// the caller's function (gprx_ctx_create_peer)
HostColl* make_callback_coll(gprx_allgather_fn fn, void* user, int world);

// sum over the ranks of `count` values in device memory (in place), through the collective
template <typename T>
void hostcoll_allreduce_dev(HostColl* hc, T* dev, int count, hipStream_t s);

// the process's view of the ranks: one rank per process (RCCL or caller collectives), or g
// virtual ranks on one GPU
struct DistContext {
    int device = 0;
    int rank = 0, world = 1;
    bool virt = false;             // world virtual ranks in this process (direct pointers)
    HostColl* hc = nullptr;        // multi-process collectives (not virt)
    int cu_slot = 0, cu_slots = 1;  // this process's share of the CUs (ranks sharing one GPU)
};

template <typename T>
struct DistFitIn {
    const KCanon<T>& K;
    const T* X;  // n x d, device, replicated
    const T* Y;  // n x m, device, replicated
    int64_t n;
    int d, m;
    T sigma2;
    TileBuild<T> tb;  // mode != 0: the fused MFMA build (features of all n samples); else the direct build
    bool inv;         // LML mode: the inverse's identity rows and C = (K + s^2 I)^{-1} ride along
};

struct DistFitOut {
    double logdet = 0, datafit = 0, est_us = 0;
    double ms_kernel = 0, ms_solve = 0;  // device time: persistent launch (slowest local rank), back-solve
    int info = 0, flag = 0, P = 0;
    int gb = 1, ww = 0, chunk_w = 0;     // the layout and window the schedule picked
    int64_t bytes_rank = 0;              // device bytes the engine holds per rank (max over this process's ranks)
    int64_t bytes_storage = 0;           // of which the packed own rows
    // this process's (first) rank's pushes per fit, from the schedule: Linv_k to every peer, final
    // tiles to the peers that read their row through the window (gprx_dev_dist_info out[11..14])
    int64_t push_linv = 0, push_tiles = 0, push_bytes = 0;
    int push_rank = 0;
};

struct DistEngineBase;
// One distributed fit: alpha_dev (np x m, row-major, this process) receives the regression
// vectors when the factorisation succeeds (out.info == INT_MAX, out.flag == 0).
template <typename T>
void dist_fit(DistEngineBase*& eng, const DistContext& C, const DistFitIn<T>& in, DistFitOut& out, T* alpha_dev);
void dist_engine_free(DistEngineBase* e);

// (L L^T)^{-1} rhs with the sharded factor of the last fit: the forward and back substitutions
// chained on the devices across the ranks.  rhs: np x m row-major (each rank reads its own row
// blocks; a virtual context's ranks all read this buffer); out: np x m, every rank.
template <typename T>
void dist_solve(DistEngineBase* eng, const T* rhs, T* out, hipStream_t s);
// After a successful dist_fit: the dense factor on this process, gathered from every rank's
// storage (a documented N^2 copy for the calls that need the whole factor: the core matrix, a
// VALU-gradient LML): the strictly-lower blocks of L into A (np x np, column-major, ld) and Linv.
template <typename T>
void dist_gather_factor(DistEngineBase* eng, T* A, int64_t ld, T* Linv, hipStream_t s);
// After an LML-mode fit: this process's ranks' gradient partials of
// sum over the lower tiles of their own row blocks of (alpha alpha^T - C) o dK/dp (k_pairs.hip),
// summed over the ranks into acc (device, MAX_LEAF * 3 doubles).  C tiles from the storage.
template <typename T>
void dist_lml_grad(DistEngineBase* eng, const KCanon<T>& K, const KCanon<T>* Kd, const T* X, int64_t n, int d,
                   const T* FU, const T* FV, T* GU, T* GV, int64_t nf, const T* alpha, double* part, double* acc,
                   hipStream_t s);
// The sharded posterior covariance (dist_pvar_kernel): the query chunks of 128 columns one solve
// takes (0: not available -- one rank, or no receive window to carry the V tiles).
int dist_pvar_chunks(DistEngineBase* eng);
// device bytes of the last posterior solve's K(Z, X_own) workspace (max over this process's ranks)
int64_t dist_pvar_bytes(DistEngineBase* eng);
// sum[j] = sum over the n training rows of V[., j] V[., j'] with V = L^{-1} K(X, Z), Z = nch x 128
// queries (device, row-major nch 128 x d; tabZ their sin/cos tables when K has periodic leaves),
// j' = j, or (pairs) j' = j + 64 within each chunk of 128; summed over every rank (host result).
template <typename T>
void dist_posterior(DistEngineBase* eng, const KCanon<T>& K, const T* X, const T* tabX, int64_t n, int d, const T* Z,
                    const T* tabZ, int nch, bool pairs, std::vector<double>& sum, hipStream_t s);
// The rows this process's ranks own (row blocks of 128, the label block excluded), ascending.
std::vector<int> dist_own_blocks(DistEngineBase* eng);
// Sum over the ranks of `count` doubles in device memory (no-op for virtual ranks).
void dist_allreduce_sum(DistEngineBase* eng, double* dev, int count, hipStream_t s);

// ---- the sharded solves and reductions (k_dsolve.hip), one launch per rank ----------------
template <typename T>
struct DSArgs {
    int g, r, nc, m;
    const int* own;        // [nc + 1] owner of each row block (the label block last)
    const int* loc;        // [nr] local index of an own row block
    const int64_t* roff;   // [nloc] element offset of local row block li in the packed storage
    const T* store;        // this rank's packed row blocks (tile (i, k) at roff[loc[i]] + k DB^2)
    const int* orows;      // this rank's matrix row blocks (< nc), ascending
    int nown;
    const int* last_of;    // [g] last matrix row block of each rank (-1: none)
    int last_own;
    const T* Linv;         // this rank's diagonal-block inverses (all nc)
    const uint64_t* mb;    // [g] mailbox bases as mapped here
    int64_t o_ztile, o_alpha, o_zf, o_part, o_fflags, o_sflags;  // mailbox byte offsets
    int zmode;             // back substitution's z: 0 the label tiles (fit), 1 the z area (forward solve)
    const T* rhs;          // forward substitution: np x m, row-major
    unsigned fit_ep, sep;  // epochs of the fit (label tiles) and of this solve
    int* ctl;              // [4] ticket, error (zeroed per launch)
    int* info;             // atomicMin -1 on a timed-out wait
    long long tlimit;
};
// ---- the sharded posterior covariance (k_dsolve.hip dist_pvar_kernel), one launch per rank ----
// V = L^{-1} K(X, Z) for nch chunks of 128 query columns, by a distributed forward substitution:
// task (own row block i, chunk c) accumulates sum_{k<i} L_ik V_k(c) on the MFMA tiles as the
// V_k(c) of every rank arrive in its window, forms V_i(c) = Linv_i (K(X_i, Z_c) - sum), pushes it
// into every rank's window slot (c, i) and adds its rows' sum of V[., j] V[., j'] (the
// ||L^{-1} k||^2 of the pairs) to part.  No rank holds more than its own rows of L.
template <typename T>
struct PVArgs {
    int g, r, nc;
    const int* loc;          // [nr] local index of an own row block
    const int64_t* roff;     // [nloc] element offset of local row block li in the packed storage
    const T* store;          // this rank's packed row blocks
    const int* orows;        // this rank's matrix row blocks (< nc), ascending
    int nown;
    const T* Linv;           // all nc diagonal inverses (this rank's mailbox)
    const uint64_t* mb;      // [g] mailbox bases as mapped here (flags)
    int64_t o_vflags;        // byte offset of the V flags: rank q's word (c nc + k) = ep when V_k(c) landed
    const uint64_t* vslot;   // [(q vstride + c) nc + k] window slot of V_k(c) in rank q (DB x DB, (query, row))
    int vstride;
    T* R;                    // nch DB x nown DB, ld nch DB: K(Z, X_own), own block orows[li] at column
                             // block li; W = K - sum L V overwrites it
    int nch;                 // chunks of 128 query columns
    int pairs;               // 0: column j with itself; 1: columns j and 64 + j of a chunk (j < 64)
    unsigned ep;             // this solve's epoch
    double* part;            // [nown][nch DB]: sum over block i's rows of V[., j] V[., j']
    int* ctl;                // [4] ticket, error (zeroed)
    int* info;               // atomicMin -1 on a timed-out wait
    long long tlimit;
};
template <typename T>
void launch_dist_pvar(const PVArgs<T>& a, int P, hipStream_t s);

template <typename T>
void launch_dist_back(const DSArgs<T>& a, hipStream_t s);
template <typename T>
void launch_dist_forward(const DSArgs<T>& a, hipStream_t s);
template <typename T>
void launch_dist_reduce(const DSArgs<T>& a, int64_t n, double* out, hipStream_t s);

}  // namespace gprx
