// Standalone microbenchmark: f64 MFMA issue rate on gfx950 (cycles per v_mfma_f64_16x16x4f64
// per SIMD), one and two waves per SIMD, independent accumulators, no memory traffic.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(512) void mfma_loop(double* out, long long* cyc, int iters) {
    d4 acc[NACC];
    for (int i = 0; i < NACC; i++) acc[i] = d4{0, 0, 0, 0};
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int i = 0; i < NACC; i++) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
    for (int i = 0; i < NACC; i++) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}
int main() {
    int ncu = 256;
    double* out; long long* cyc;
    hipMalloc(&out, sizeof(double) * ncu * 512);
    hipMalloc(&cyc, sizeof(long long) * ncu);
    long long h[256];
    const int iters = 4000;
    for (int threads : {256, 512}) {
        hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
        mfma_loop<8><<<ncu, threads>>>(out, cyc, 10);
        hipEventRecord(e0);
        mfma_loop<8><<<ncu, threads>>>(out, cyc, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
        double avg = 0; for (int i = 0; i < ncu; i++) avg += h[i]; avg /= ncu;
        const double waves_per_simd = threads / 256.0;
        const double mfma_per_simd = waves_per_simd * 8.0 * iters;
        const double flops = (double)ncu * threads / 64 * 8.0 * iters * 2048;
        printf("threads %d: %.1f cycles/MFMA/SIMD (memtime), %.3f ms, %.1f TF/s, clock %.2f GHz\n", threads,
               avg / mfma_per_simd, ms, flops / ms / 1e9, avg / (ms * 1e6));
    }
    return 0;
}
