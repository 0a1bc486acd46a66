// ipc_probe.hip — can two processes on one MI355X exchange data through IPC-mapped
// fine-grained device memory with device-side stores and flags only (no host in the loop)?
//
// The distributed fit (gpr_amd/csrc/gprx_dist.cpp) pushes factored tiles straight into the
// peers' receive windows; across processes the windows are hipIpcOpenMemHandle mappings.
// This probe checks the three things that rests on, on the one-GPU box:
//   1. hipIpcGetMemHandle works on hipExtMallocWithFlags(hipDeviceMallocFinegrained) memory
//      (dmabuf IPC, HSA_ENABLE_IPC_MODE_LEGACY=0);
//   2. a kernel of process B can store into it and a kernel of process A, resident at the same
//      time on the same GPU, sees the data after a system-scope release/acquire on a flag;
//   3. both directions, several rounds (slot reuse with epoch-valued flags).
// Usage: ipc_probe server <file> & ipc_probe client <file>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(2);                                                                      \
        }                                                                                      \
    } while (0)

constexpr int NE = 1 << 16;  // doubles per message (512 KB)
constexpr int ROUNDS = 8;

// mailbox: [ROUNDS slots of NE doubles][flag (uint64)]; each side owns one mailbox and writes
// the peer's, one slot per round (no slot is rewritten while the peer may still read it)
__global__ void ping(double* my, unsigned long long* myflag, double* peer, unsigned long long* peerflag, int side,
                     int* result, long long tlimit) {
    __shared__ int s_ok;
    const int t = threadIdx.x;
    int bad = 0;
    for (int r = 0; r < ROUNDS; r++) {
        const unsigned long long ep = (unsigned long long)(r + 1);
        // side 0 sends first in even rounds, side 1 answers; odd rounds the other way
        const bool send_first = ((r & 1) == side);
        for (int phase = 0; phase < 2; phase++) {
            const bool sending = (phase == 0) == send_first;
            if (sending) {
                for (int e = t; e < NE; e += blockDim.x) peer[(int64_t)r * NE + e] = (double)(r * 1000003 + e * 7 + side);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                __syncthreads();
                if (t == 0) __hip_atomic_store(peerflag, ep, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                if (t == 0) {
                    const long long t0 = wall_clock64();
                    int ok = 1;
                    while (__hip_atomic_load(myflag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < ep) {
                        if (wall_clock64() - t0 > tlimit) {
                            ok = 0;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(2);
                    }
                    s_ok = ok;
                }
                __syncthreads();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                if (!s_ok) {
                    if (t == 0) result[1] = r + 1;  // timed out in round r
                    return;
                }
                for (int e = t; e < NE; e += blockDim.x)
                    if (my[(int64_t)r * NE + e] != (double)(r * 1000003 + e * 7 + (1 - side))) bad++;
                __syncthreads();
            }
        }
    }
    atomicAdd(result, bad);
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: ipc_probe server|client <file>\n");
        return 2;
    }
    const bool server = std::strcmp(argv[1], "server") == 0;
    const std::string base = argv[2];
    const size_t bytes = sizeof(double) * NE * ROUNDS + 256;
    CK(hipSetDevice(0));
    void* mine = nullptr;
    CK(hipExtMallocWithFlags(&mine, bytes, hipDeviceMallocFinegrained));
    CK(hipMemset(mine, 0, bytes));
    hipIpcMemHandle_t h;
    CK(hipIpcGetMemHandle(&h, mine));
    const std::string myfile = base + (server ? ".s" : ".c"), peerfile = base + (server ? ".c" : ".s");
    {
        const std::string tmp = myfile + ".tmp";
        FILE* f = std::fopen(tmp.c_str(), "wb");
        std::fwrite(&h, sizeof(h), 1, f);
        std::fclose(f);
        std::rename(tmp.c_str(), myfile.c_str());
    }
    hipIpcMemHandle_t ph;
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        FILE* f = std::fopen(peerfile.c_str(), "rb");
        if (f) {
            const size_t got = std::fread(&ph, sizeof(ph), 1, f);
            std::fclose(f);
            if (got == 1) break;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(30)) {
            std::fprintf(stderr, "no peer handle\n");
            return 3;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(20));
    }
    void* peer = nullptr;
    CK(hipIpcOpenMemHandle(&peer, ph, hipIpcMemLazyEnablePeerAccess));
    int* res = nullptr;
    CK(hipMalloc(&res, 2 * sizeof(int)));
    CK(hipMemset(res, 0, 2 * sizeof(int)));
    double* myd = (double*)mine;
    double* pd = (double*)peer;
    auto* myf = (unsigned long long*)(myd + (size_t)NE * ROUNDS);
    auto* pf = (unsigned long long*)(pd + (size_t)NE * ROUNDS);
    hipLaunchKernelGGL(ping, dim3(1), dim3(256), 0, 0, myd, myf, pd, pf, server ? 0 : 1, res, (long long)(1e8 * 10));
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    int hr[2];
    CK(hipMemcpy(hr, res, sizeof(hr), hipMemcpyDeviceToHost));
    std::printf("ipc_probe %s: %d rounds, mismatches %d, timeout-round %d -> %s\n", server ? "server" : "client", ROUNDS,
                hr[0], hr[1], (hr[0] == 0 && hr[1] == 0) ? "OK" : "FAIL");
    std::fflush(stdout);
    // keep the mapping alive until the peer has finished reading our writes
    std::this_thread::sleep_for(std::chrono::milliseconds(500));
    CK(hipIpcCloseMemHandle(peer));
    CK(hipFree(mine));
    return (hr[0] == 0 && hr[1] == 0) ? 0 : 1;
}
