// coexec_probe.hip — does f64 MFMA from one wave overlap f64 VALU FMAs from another wave on the
// same SIMD (gfx950)?  One workgroup of 8 waves per CU (waves w and w + 4 share a SIMD).
// mode 0: every wave runs the MFMA loop; 1: every wave the VALU loop; 2: waves 0-3 MFMA,
// waves 4-7 VALU.  If the units co-issue, mode 2 takes ~max of half of modes 0 and 1.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(512) void probe(double* out, int iters, int mode) {
    const int w = threadIdx.x >> 6;
    const bool mf = (mode == 0) || (mode == 2 && w < 4);
    double a = threadIdx.x * 1e-3, b = 1.0 + threadIdx.x * 1e-4;
    if (mf) {
        d4 acc[8];
        for (int u = 0; u < 8; u++) acc[u] = d4{0, 0, 0, 0};
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int u = 0; u < 8; u++) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[u], 0, 0, 0);
        }
        double s = 0;
        for (int u = 0; u < 8; u++) s += acc[u][0] + acc[u][3];
        out[blockIdx.x * 512 + threadIdx.x] = s;
    } else {
        // 8 MFMAs of 16x16x4 = 8 x 2048 flops per wave-iteration = 256 f64 FMAs per lane: match it
        double v[16];
        for (int u = 0; u < 16; u++) v[u] = a + u;
        for (int it = 0; it < iters; it++) {
#pragma unroll
            for (int r = 0; r < 16; r++)
#pragma unroll
                for (int u = 0; u < 16; u++) v[u] = fma(v[u], b, 1e-9);
        }
        double s = 0;
        for (int u = 0; u < 16; u++) s += v[u];
        out[blockIdx.x * 512 + threadIdx.x] = s;
    }
}
int main() {
    int ncu = 0;
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    double* out;
    hipMalloc(&out, sizeof(double) * 512 * ncu);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 4000;
    for (int mode = 0; mode < 3; mode++) {
        hipLaunchKernelGGL(probe, dim3(ncu), dim3(512), 0, 0, out, 10, mode);
        hipEventRecord(e0);
        hipLaunchKernelGGL(probe, dim3(ncu), dim3(512), 0, 0, out, iters, mode);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double flops_wave = 8.0 * 2048 * iters;  // per wave (MFMA) = 256 FMA/lane x 2 x 64 (VALU)
        printf("{\"mode\": %d, \"ms\": %.3f, \"tflops\": %.2f}\n", mode, ms, flops_wave * 8 * ncu / (ms * 1e-3) / 1e12);
    }
    return 0;
}
