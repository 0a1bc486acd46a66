// Which physical CU (XCC, SE, CU) does each bit of a HIP stream CU mask select on this GPU?
// Launches on streams whose mask holds a few bits and records where the workgroups ran.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void where(unsigned* out) {
    if (threadIdx.x == 0) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | 20);  // HW_REG_XCC_ID[3:0]
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_REG_HW_ID
        // spin briefly so the workgroups overlap and spread over the masked CUs
        const long long t0 = wall_clock64();
        while (wall_clock64() - t0 < 20000) __builtin_amdgcn_s_sleep(1);
        out[2 * blockIdx.x] = xcc;
        out[2 * blockIdx.x + 1] = hw;
    }
}

static void run(const char* name, const std::vector<uint32_t>& mask, unsigned* d, int nwg) {
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()) != hipSuccess) { std::printf("mask stream failed\n"); return; }
    (void)hipMemset(d, 0xff, 4096 * sizeof(unsigned));
    hipLaunchKernelGGL(where, dim3(nwg), dim3(64), 0, s, d);
    (void)hipStreamSynchronize(s);
    std::vector<unsigned> h(2 * nwg);
    (void)hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
    std::vector<int> seen(8 * 8 * 16, 0);
    int per[8] = {0}, distinct = 0;
    for (int w = 0; w < nwg; w++) {
        const unsigned x = h[2 * w] & 7, hw = h[2 * w + 1];
        const int key = (x * 8 + ((hw >> 13) & 7)) * 16 + ((hw >> 8) & 15);
        if (!seen[key]++) { distinct++; per[x]++; }
    }
    std::printf("%-28s %4d workgroups -> %3d distinct CUs; per XCC:", name, nwg, distinct);
    for (int x = 0; x < 8; x++) std::printf(" %d", per[x]);
    std::printf("\n");
    (void)hipStreamDestroy(s);
}

int main() {
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    std::printf("CUs %d\n", ncu);
    unsigned* d;
    (void)hipMalloc(&d, 4096 * sizeof(unsigned));
    const int nw = (ncu + 31) / 32;
    auto range = [&](int a, int b) { std::vector<uint32_t> m(nw, 0u); for (int i = a; i < b; i++) m[i / 32] |= 1u << (i % 32); return m; };
    auto stride = [&](int st, int off) { std::vector<uint32_t> m(nw, 0u); for (int i = off; i < ncu; i += st) m[i / 32] |= 1u << (i % 32); return m; };
    run("bit 0", range(0, 1), d, 1024);
    run("bits 0-3", range(0, 4), d, 1024);
    run("bits 0-7", range(0, 8), d, 1024);
    run("bits 0-31", range(0, 32), d, 1024);
    run("bits 0-127", range(0, 128), d, 1024);
    run("bits 248-255", range(248, 256), d, 1024);
    run("every 8th bit from 0", stride(8, 0), d, 1024);
    run("every 32nd bit from 0", stride(32, 0), d, 1024);
    run("all", range(0, ncu), d, 1024);
    return 0;
}
