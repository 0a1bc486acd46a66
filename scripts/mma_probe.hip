// Standalone microbenchmark of the 128x128 tile mainloop (k_mma.h tile_mma): one 512-thread
// workgroup per CU, each running `reps` tile products of depth K.  Operands either stay
// L2-resident (mode 0: every workgroup reads the same 128-row blocks) or come from a 32768-row
// matrix, each workgroup its own row blocks (mode 1: HBM/MALL-fed, the factorisation's regime).
// Reports cycles per stage against the MFMA bound (2 waves/SIMD x BK/4 k-steps x 8 MFMAs x
// 64 (f64) or 32 (f32) cycles = 4096 at the shipped depths), the TF/s and the clock.
//   hipcc -O3 --offload-arch=gfx950 -I. scripts/mma_probe.hip -o tools/probe/mma_probe
//   /tmp/mma_probe f32|f64 K reps mode
#include "gpr_amd/csrc/k_mma.h"
#include <cstdio>
#include <cstring>
#include <vector>
using namespace gprx;
using namespace gprx::mm;

constexpr int64_t MROWS = 32768;

template <typename T>
__global__ __launch_bounds__(NT) void probe(const T* M, int64_t ld, int K, int reps, int mode, T* out, long long* cyc) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    T* smem = reinterpret_cast<T*>(smem_raw);
    const int64_t ra = mode ? (int64_t)(blockIdx.x % 256) * 128 : 0;
    const int64_t rb = mode ? (int64_t)((blockIdx.x * 7 + 3) % 256) * 128 : 512;
    typename Mfma<T>::acc_t acc[2][4];
    T s = 0;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; r++) {
        tile_mma<T>(acc, M + ra, ld, M + rb, ld, K, K, smem, threadIdx.x);
#pragma unroll
        for (int x = 0; x < 2; x++)
#pragma unroll
            for (int y = 0; y < 4; y++) s += acc[x][y][0] + acc[x][y][1] + acc[x][y][2] + acc[x][y][3];
        __syncthreads();
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * NT + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename T>
int run(int K, int reps, int mode) {
    const int ncu = 256;
    const int64_t ld = MROWS;
    T *M, *out;
    long long* cyc;
    if (hipMalloc(&M, sizeof(T) * ld * K) != hipSuccess) return 1;
    hipMemset(M, 0, sizeof(T) * ld * K);
    hipMalloc(&out, sizeof(T) * ncu * NT);
    hipMalloc(&cyc, sizeof(long long) * ncu);
    const size_t lds = gemm_lds<T>() + 16;
    hipFuncSetAttribute((const void*)probe<T>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    probe<T><<<ncu, NT, lds>>>(M, ld, K, 2, mode, out, cyc);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float best = 1e30f;
    double avg = 0;
    for (int it = 0; it < 3; it++) {
        hipEventRecord(e0);
        probe<T><<<ncu, NT, lds>>>(M, ld, K, reps, mode, out, cyc);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) {
            best = ms;
            std::vector<long long> h(ncu);
            hipMemcpy(h.data(), cyc, sizeof(long long) * ncu, hipMemcpyDeviceToHost);
            avg = 0;
            for (auto v : h) avg += v;
            avg /= ncu;
        }
    }
    constexpr int BK = BkOf<T>::v;
    const double stages = (double)reps * K / BK;
    const double bound = 2.0 * (BK / 4) * 8 * (sizeof(T) == 8 ? 64 : 32);
    const double flops = 2.0 * 128 * 128 * K * reps * ncu;
    printf("{\"dtype\": \"%s\", \"K\": %d, \"reps\": %d, \"mode\": %d, \"BK\": %d, \"NB\": %d, "
           "\"cycles_per_stage\": %.0f, \"mfma_bound_frac\": %.4f, \"tflops\": %.2f, \"ghz\": %.3f}\n",
           sizeof(T) == 8 ? "f64" : "f32", K, reps, mode, BK, Stage<T>::NB, avg / stages,
           bound / (avg / stages), flops / (best * 1e9), avg / (best * 1e6));
    hipFree(M);
    hipFree(out);
    hipFree(cyc);
    return 0;
}

int main(int argc, char** argv) {
    const bool f32 = argc > 1 && !strcmp(argv[1], "f32");
    const int K = argc > 2 ? atoi(argv[2]) : 4096, reps = argc > 3 ? atoi(argv[3]) : 10;
    const int mode = argc > 4 ? atoi(argv[4]) : 0;
    return f32 ? run<float>(K, reps, mode) : run<double>(K, reps, mode);
}
