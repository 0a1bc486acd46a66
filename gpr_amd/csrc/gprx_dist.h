// gprx_dist.h — the storage-sharded multi-GPU fit (gprx_dist.cpp): interface used by the
// model code (gprx_api.cpp).
#pragma once
#include "gprx_internal.h"

namespace gprx {

constexpr int C_NCTL_DIST = 16;  // control words at the head of a tile launch's counter block (k_mma.h)

// the process's view of the ranks: one RCCL rank per process, or g virtual ranks on one GPU
struct DistContext {
    int device = 0;
    int rank = 0, world = 1;
    bool virt = false;           // world virtual ranks in this process (device copies, no RCCL)
    ncclComm_t comm = nullptr;   // RCCL communicator (not virt)
    hipStream_t stream = nullptr;  // the rank's compute stream (not virt)
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
};

struct DistFitOut {
    double logdet = 0, datafit = 0, est_us = 0;
    double ms_kernel = 0, ms_solve = 0;  // device time: persistent launch (slowest local rank), back-solve
    int info = 0, flag = 0, P = 0;
};

struct DistEngineBase;
// One distributed fit: alpha_dev (np x m, this process's rank 0) receives the regression
// vectors when the factorisation succeeds (out.info == INT_MAX, out.flag == 0).
template <typename T>
void dist_fit(DistEngineBase*& eng, const DistContext& C, const DistFitIn<T>& in, DistFitOut& out, T* alpha_dev,
              Exec& ex);
void dist_engine_free(DistEngineBase* e);

// After a successful dist_fit: the dense factor on this process (every rank holds every
// off-diagonal tile and every diagonal inverse): the strictly-lower blocks of L into A
// (np x np, column-major, ld) and Linv (nc blocks of DB x DB), on `s` (synchronised).
template <typename T>
void dist_assemble_factor(DistEngineBase* eng, T* A, int64_t ld, T* Linv, hipStream_t s);
// The layout of the last fit: ranks, row-block group size, this process's first rank, and
// whether its ranks are virtual (all in this process).
void dist_layout(DistEngineBase* eng, int* g, int* gb, int* rank, bool* virt);
// In-place sum over the ranks of `count` doubles in device memory (RCCL; no-op for virtual
// ranks and one-rank communicators).
void dist_allreduce_sum(DistEngineBase* eng, double* dev, int count, hipStream_t s);

}  // namespace gprx
