// Standalone microbenchmark of the 128x128 f64 tile mainloop (k_mma.h tile_mma): one
// 512-thread workgroup per CU, each running `reps` tile products of depth K from operands that
// stay L2-resident (every workgroup of an XCD reads the same 2 MiB), cycles per 16-deep stage
// against the MFMA bound (2 waves/SIMD x 32 MFMA x 64 cycles = 4096).
//   hipcc -O3 --offload-arch=gfx950 -I. scripts/mma_probe.hip -o /tmp/mma_probe
#include "gpr_amd/csrc/k_mma.h"
#include <cstdio>
#include <vector>
using namespace gprx;
using namespace gprx::mm;

__global__ __launch_bounds__(NT) void probe(const double* A, const double* B, int64_t ld, int K, int reps, double* out,
                                            long long* cyc, int distinct) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    double* smem = reinterpret_cast<double*>(smem_raw);
    const int64_t off = distinct ? (int64_t)(blockIdx.x % 64) * 128 : 0;
    Mfma<double>::acc_t acc[2][4];
    double s = 0;
    __syncthreads();
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; r++) {
        tile_mma<double>(acc, A + off, ld, B + off, ld, K, K, smem, threadIdx.x);
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

int main(int argc, char** argv) {
    const int K = argc > 1 ? atoi(argv[1]) : 2048, reps = argc > 2 ? atoi(argv[2]) : 20;
    const int distinct = argc > 3 ? atoi(argv[3]) : 0;
    const int ncu = 256;
    const int64_t ld = 128 * 64 + 64;  // distinct: 64 row blocks side by side
    double *A, *out;
    long long* cyc;
    hipMalloc(&A, sizeof(double) * ld * K + 4096);
    hipMemset(A, 0, sizeof(double) * ld * K);
    hipMalloc(&out, sizeof(double) * ncu * NT);
    hipMalloc(&cyc, sizeof(long long) * ncu);
    const size_t lds = gemm_lds<double>() + 16;
    hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    probe<<<ncu, NT, lds>>>(A, A + 4 * 128, ld, K, 2, out, cyc, distinct);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    probe<<<ncu, NT, lds>>>(A, A + 4 * 128, ld, K, reps, out, cyc, distinct);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> h(ncu);
    hipMemcpy(h.data(), cyc, sizeof(long long) * ncu, hipMemcpyDeviceToHost);
    double avg = 0;
    for (auto v : h) avg += v;
    avg /= ncu;
    const double stages = (double)reps * K / BKS;
    const double flops = 2.0 * 128 * 128 * K * reps * ncu;
    printf("K=%d reps=%d distinct=%d BKS=%d NBUF=%d: %.0f cycles/stage (MFMA bound 4096: %.1f%%), %.2f TF/s, clock %.2f GHz\n",
           K, reps, distinct, BKS, NBUF, avg / stages, 100.0 * 4096 / (avg / stages), flops / (ms * 1e9), avg / (ms * 1e6));
    return 0;
}
