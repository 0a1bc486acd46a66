// gprx_dev.cpp — developer timing hooks (include/gprx_dev.h).
#include <hip/hip_runtime.h>

#include <climits>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gprx_dev.h"
#include "gprx_internal.h"

namespace gprx {
template <typename T>
void launch_gemm_nt(T* C, int64_t ldc, const T* A, int64_t lda, const T* B, int64_t ldb, int64_t M, int64_t N,
                    int64_t K, T alpha, T beta, bool lower, hipStream_t s);
template <typename T>
void launch_diag_public(T* Akk, int64_t ld, T* Lk, int* info, int64_t col0, hipStream_t s, int ph = 3);
template <typename T>
void launch_diag_prof(T* Akk, int64_t ld, T* Lk, int* info, long long* prof, hipStream_t s);
namespace pt {
template <typename T>
void launch_diag_bench(int variant, T* A, int64_t ld, T* Linv, int* info, long long* prof, int reps, hipStream_t s);
}
}  // namespace gprx

using namespace gprx;

template <typename T>
__global__ void dev_fill_spd(T* A, int64_t ld, int64_t n, uint64_t seed) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= ld * n) return;
    int64_t i = e % ld, j = e / ld;
    uint64_t z = (uint64_t)e * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    T v = (T)((double)(z >> 11) * (1.0 / 9007199254740992.0)) * T(1e-3);
    if (i == j) v += T(n);  // diagonally dominant -> SPD
    A[e] = v;
}

__global__ void dev_fexp_kernel(const double* __restrict__ x, int64_t n, double* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = fexp(x[i]);
}

template <typename T>
static gprx_status bench_impl(int what, int64_t M, int64_t N, int64_t K, int iters, double* ms, Exec& ex) {
    hipStream_t s = ex.s0;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    std::vector<void*> bufs;
    auto alloc = [&](size_t b) {
        void* p = nullptr;
        if (hipMalloc(&p, b) != hipSuccess) throw Error{GPRX_ERR_OOM, "dev bench: hipMalloc failed"};
        bufs.push_back(p);
        return p;
    };
    int* info = (int*)alloc(sizeof(int));
    float tms = 0;
    try {
        if (what == 11 || what == 12 || what == 13) {  // tile-engine diagonal factor (k_ptiles.hip), variant what - 11:
            // ms[0] = us per factor (events), ms[1..5] = per-factor phase ticks (100 MHz)
            const int reps = std::max(1, iters);
            T* A = (T*)alloc(sizeof(T) * DB * DB * (size_t)reps);
            T* L = (T*)alloc(sizeof(T) * DB * DB);
            long long* pr = (long long*)alloc(sizeof(long long) * 8);
            (void)hipMemsetAsync(pr, 0, sizeof(long long) * 8, s);
            for (int it = 0; it < reps; it++)
                hipLaunchKernelGGL(dev_fill_spd<T>, dim3((DB * DB + 255) / 256), dim3(256), 0, s, A + (size_t)it * DB * DB,
                                   (int64_t)DB, (int64_t)DB, (uint64_t)it);
            (void)hipMemsetAsync(info, 0x7f, sizeof(int), s);
            pt::launch_diag_bench<T>(what - 11, A, DB, L, info, pr, 1, s);  // warm (factors block 0 in place)
            for (int it = 0; it < 1; it++)
                hipLaunchKernelGGL(dev_fill_spd<T>, dim3((DB * DB + 255) / 256), dim3(256), 0, s, A, (int64_t)DB,
                                   (int64_t)DB, (uint64_t)0);
            (void)hipEventRecord(e0, s);
            pt::launch_diag_bench<T>(what - 11, A, DB, L, info, pr, reps, s);
            (void)hipEventRecord(e1, s);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&tms, e0, e1);
            long long h[8];
            (void)hipMemcpy(h, pr, sizeof(h), hipMemcpyDeviceToHost);
            ms[0] = 1e3 * tms / reps;
            for (int i = 0; i < 8; i++) ms[1 + i] = (double)h[i] / reps;
        } else if (what == 6) {  // in-kernel phase ticks of the diagonal kernel: ms[0..4] per launch
            T* A = (T*)alloc(sizeof(T) * DB * DB * (size_t)iters);
            T* L = (T*)alloc(sizeof(T) * DB * DB);
            long long* pr = (long long*)alloc(sizeof(long long) * 8);
            (void)hipMemset(pr, 0, sizeof(long long) * 8);
            for (int it = 0; it < iters; it++)
                hipLaunchKernelGGL(dev_fill_spd<T>, dim3((DB * DB + 255) / 256), dim3(256), 0, s, A + (size_t)it * DB * DB,
                                   (int64_t)DB, (int64_t)DB, (uint64_t)it);
            for (int it = 0; it < iters; it++) launch_diag_prof<T>(A + (size_t)it * DB * DB, DB, L, info, pr, s);
            long long h[8];
            (void)hipStreamSynchronize(s);
            (void)hipMemcpy(h, pr, sizeof(h), hipMemcpyDeviceToHost);
            for (int i = 0; i < 5; i++) ms[i] = (double)h[i] / iters;
        } else if (what == 0) {
            const int ph = 3;
            T* A = (T*)alloc(sizeof(T) * DB * DB * (size_t)iters);
            T* L = (T*)alloc(sizeof(T) * DB * DB);
            for (int it = 0; it < iters; it++)
                hipLaunchKernelGGL(dev_fill_spd<T>, dim3((DB * DB + 255) / 256), dim3(256), 0, s, A + (size_t)it * DB * DB,
                                   (int64_t)DB, (int64_t)DB, (uint64_t)it);
            launch_diag_public<T>(A, DB, L, info, 0, s, ph);  // warm
            (void)hipEventRecord(e0, s);
            for (int it = 1; it < iters; it++) launch_diag_public<T>(A + (size_t)it * DB * DB, DB, L, info, 0, s, ph);
            (void)hipEventRecord(e1, s);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&tms, e0, e1);
            *ms = tms / std::max(1, iters - 1);
        } else if (what == 1 || what == 2) {
            const int64_t ld = M;
            T* C = (T*)alloc(sizeof(T) * ld * N);
            T* A = (T*)alloc(sizeof(T) * ld * K);
            T* B = (T*)alloc(sizeof(T) * N * K);
            (void)hipMemset(C, 0, sizeof(T) * ld * N);
            (void)hipMemset(A, 0, sizeof(T) * ld * K);
            (void)hipMemset(B, 0, sizeof(T) * N * K);
            hipLaunchKernelGGL(dev_fill_spd<T>, dim3((unsigned)((ld * K + 255) / 256)), dim3(256), 0, s, A, ld, K,
                               (uint64_t)1);
            hipLaunchKernelGGL(dev_fill_spd<T>, dim3((unsigned)((N * K + 255) / 256)), dim3(256), 0, s, B, N, K,
                               (uint64_t)2);
            launch_gemm_nt<T>(C, ld, A, ld, B, N, M, N, K, T(-1), T(1), what == 2, s);
            (void)hipEventRecord(e0, s);
            for (int it = 0; it < iters; it++) launch_gemm_nt<T>(C, ld, A, ld, B, N, M, N, K, T(-1), T(1), what == 2, s);
            (void)hipEventRecord(e1, s);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&tms, e0, e1);
            *ms = tms / iters;
        } else if (what == 3 || what == 4 || what == 5 || what == 9 || what == 10) {
            const int64_t n = M;
            T* A = (T*)alloc(sizeof(T) * n * n);
            T* Li = (T*)alloc(sizeof(T) * n * DB);
            T* z = (T*)alloc(sizeof(T) * n);
            T* al = (T*)alloc(sizeof(T) * n);
            Exec single;
            single.s0 = s;
            single.s1 = nullptr;
            Exec& use = (what == 4) ? ex : single;
            double total = 0;
            for (int it = 0; it < iters + 1; it++) {
                hipLaunchKernelGGL(dev_fill_spd<T>, dim3((unsigned)((n * n + 255) / 256)), dim3(256), 0, s, A, n, n,
                                   (uint64_t)it);
                (void)hipMemsetD32Async((hipDeviceptr_t)info, INT_MAX, 1, s);
                if (what == 5 || what == 10) potrf_blocked<T>(A, n, n, n, Li, info, use);
                (void)hipEventRecord(e0, s);
                if (what == 5) launch_backsolve<T>(A, n, n - DB, 1, Li, z, al, s);
                else if (what == 10) launch_backsolve_chain<T>(A, n, n - DB, 1, Li, al, info, ex, s);
                else if (what == 9) potrf_tiles<T>(A, n, n, n, Li, info, ex);
                else potrf_blocked<T>(A, n, n, n, Li, info, use);
                (void)hipEventRecord(e1, s);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&tms, e0, e1);
                if (it > 0) total += tms;
            }
            *ms = total / iters;
        } else if (what == 7 || what == 8) {  // the same sequences replayed from a captured hipGraph
            const int64_t n = M;
            T* A = (T*)alloc(sizeof(T) * n * n);
            T* Li = (T*)alloc(sizeof(T) * n * DB);
            T* z = (T*)alloc(sizeof(T) * n);
            T* al = (T*)alloc(sizeof(T) * n);
            hipLaunchKernelGGL(dev_fill_spd<T>, dim3((unsigned)((n * n + 255) / 256)), dim3(256), 0, s, A, n, n,
                               (uint64_t)0);
            if (what == 8) potrf_blocked<T>(A, n, n, n, Li, info, ex);
            (void)hipStreamSynchronize(s);
            hipGraph_t g = nullptr;
            hipGraphExec_t ge = nullptr;
            GPRX_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed));
            if (what == 8) launch_backsolve<T>(A, n, n - DB, 1, Li, z, al, s);
            else potrf_blocked<T>(A, n, n, n, Li, info, ex);
            GPRX_HIP(hipStreamEndCapture(s, &g));
            GPRX_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            double total = 0;
            for (int it = 0; it < iters + 1; it++) {
                if (what == 7) {
                    hipLaunchKernelGGL(dev_fill_spd<T>, dim3((unsigned)((n * n + 255) / 256)), dim3(256), 0, s, A, n, n,
                                       (uint64_t)it);
                    (void)hipMemsetD32Async((hipDeviceptr_t)info, INT_MAX, 1, s);
                }
                (void)hipEventRecord(e0, s);
                GPRX_HIP(hipGraphLaunch(ge, s));
                (void)hipEventRecord(e1, s);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&tms, e0, e1);
                if (it > 0) total += tms;
            }
            *ms = total / iters;
            (void)hipGraphExecDestroy(ge);
            (void)hipGraphDestroy(g);
        } else {
            throw Error{GPRX_ERR_ARG, "dev bench: unknown case"};
        }
        if (hipDeviceSynchronize() != hipSuccess) throw Error{GPRX_ERR_HIP, "dev bench: device error"};
    } catch (const Error& e) {
        for (void* p : bufs) (void)hipFree(p);
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
        return e.st;
    }
    for (void* p : bufs) (void)hipFree(p);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return GPRX_OK;
}

namespace gprx {
int pt_debug_snapshot(int* out, int max_wg);
int64_t pt_trace_copy(int32_t* tasks, long long* times, int64_t max);
int64_t bs_trace_copy(long long* out, int64_t max_blocks);
}
extern "C" int64_t gprx_dev_bs_trace(int64_t* times, int64_t max_blocks) {
    try {
        return gprx::bs_trace_copy((long long*)times, max_blocks);
    } catch (const Error& e) {
        std::fprintf(stderr, "gprx_dev_bs_trace: %s\n", e.msg.c_str());
        return -1;
    }
}
extern "C" int64_t gprx_dev_pt_trace(int32_t* tasks, int64_t* times, int64_t max) {
    try {
        return gprx::pt_trace_copy(tasks, (long long*)times, max);
    } catch (const gprx::Error& e) {
        std::fprintf(stderr, "gprx_dev_pt_trace: %s\n", e.msg.c_str());
        return -1;
    }
}
extern "C" int32_t gprx_dev_pt_debug(int32_t* out, int32_t max_wg) { return gprx::pt_debug_snapshot(out, max_wg); }

extern "C" gprx_status gprx_dev_schedule(int32_t nc, int32_t nr, int32_t P, int32_t build, double* est_us,
                                         int64_t* ntasks) {
    try {
        // build: bit 0 = fused covariance build, bit 1 = the last nc row blocks are identity,
        // bits 8..15 = chunk rule ratio + 1 (0: the one the simulation picks), bits 16..23 =
        // paired updates' row offset + 1 (0: the simulation's choice, 1: none)
        const int64_t n = potrf_tiles_schedule_stats(nc, nr, P, (build & 1) != 0, est_us, (build & 2) ? nc : 0,
                                                     ((build >> 8) & 0xff) - 1, nullptr, 0, ((build >> 16) & 0xff) - 1);
        if (ntasks) *ntasks = n;
        return GPRX_OK;
    } catch (const Error& e) {
        std::fprintf(stderr, "gprx_dev_schedule: %s\n", e.msg.c_str());
        return e.st;
    }
}

extern "C" int64_t gprx_dev_schedule_list(int32_t nc, int32_t nr, int32_t P, int32_t build, int32_t* out,
                                          int64_t max) {
    try {
        return potrf_tiles_schedule_stats(nc, nr, P, (build & 1) != 0, nullptr, (build & 2) ? nc : 0,
                                          ((build >> 8) & 0xff) - 1, out, max, ((build >> 16) & 0xff) - 1);
    } catch (const Error& e) {
        std::fprintf(stderr, "gprx_dev_schedule_list: %s\n", e.msg.c_str());
        return -1;
    }
}

namespace gprx {
gprx_status gprx_dev_bench_impl(gprx_dtype dtype, int32_t what, int64_t M, int64_t N, int64_t K, int32_t iters,
                                double* ms, Exec* ex) {
    return dtype == GPRX_F64 ? bench_impl<double>(what, M, N, K, iters, ms, *ex)
                             : bench_impl<float>(what, M, N, K, iters, ms, *ex);
}
}  // namespace gprx

extern "C" gprx_status gprx_dev_fexp(gprx_ctx* ctx, const double* x, int64_t n, double* y) {
    (void)ctx;
    if (n <= 0) return GPRX_OK;
    double *dx = nullptr, *dy = nullptr;
    if (hipMalloc(&dx, sizeof(double) * n) != hipSuccess || hipMalloc(&dy, sizeof(double) * n) != hipSuccess)
        return GPRX_ERR_OOM;
    (void)hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(dev_fexp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, dx, n, dy);
    const hipError_t e = hipMemcpy(y, dy, sizeof(double) * n, hipMemcpyDeviceToHost);
    (void)hipFree(dx);
    (void)hipFree(dy);
    return e == hipSuccess ? GPRX_OK : GPRX_ERR_HIP;
}

extern "C" gprx_status gprx_dev_diag_factor(gprx_ctx* ctx, int32_t variant, const double* A, double* L, double* Linv,
                                            int32_t* info_out) {
    (void)ctx;
    if (variant < 0 || variant > 2 || !A || !L || !Linv || !info_out) return GPRX_ERR_ARG;
    double *dA = nullptr, *dLi = nullptr;
    int* di = nullptr;
    long long* pr = nullptr;
    const size_t b = sizeof(double) * DB * DB;
    gprx_status st = GPRX_OK;
    if (hipMalloc(&dA, b) != hipSuccess || hipMalloc(&dLi, b) != hipSuccess || hipMalloc(&di, sizeof(int)) != hipSuccess ||
        hipMalloc(&pr, sizeof(long long) * 8) != hipSuccess) {
        st = GPRX_ERR_OOM;
    } else {
        const int big = 0x7fffffff;
        (void)hipMemcpy(dA, A, b, hipMemcpyHostToDevice);
        (void)hipMemcpy(di, &big, sizeof(int), hipMemcpyHostToDevice);
        pt::launch_diag_bench<double>(variant, dA, DB, dLi, di, pr, 1, 0);
        if (hipMemcpy(L, dA, b, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(Linv, dLi, b, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(info_out, di, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess)
            st = GPRX_ERR_HIP;
    }
    (void)hipFree(dA);
    (void)hipFree(dLi);
    (void)hipFree(di);
    (void)hipFree(pr);
    return st;
}

extern "C" gprx_status gprx_dev_dist_schedule(int32_t nc, int32_t P, int32_t g, int32_t gb, int32_t ww, int32_t flags,
                                              double* est_us, int32_t* chunk_w, int64_t* ntasks) {
    if (nc < 1 || P < 1 || g < 1 || g > 32 || gb < 1 || ww < 1 || !est_us) return GPRX_ERR_ARG;
    try {
        // flags bits 8..15: the update-chunk rule's ratio + 1 (0: the fixed rule)
        const DistSched S = potrf_dist_schedule(nc, g, gb, ww, P, (flags & 1) != 0, (flags & 2) != 0,
                                                std::max(0, ((flags >> 8) & 0xff) - 1));
        *est_us = S.est_us;
        if (chunk_w) *chunk_w = S.W;
        if (ntasks) {
            int64_t t = 0;
            for (const auto& l : S.lists) t += (int64_t)l.size();
            *ntasks = t;
        }
    } catch (...) {
        return GPRX_ERR_ARG;
    }
    return GPRX_OK;
}
