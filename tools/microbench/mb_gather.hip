// Scattered 4-byte gathers from an L2-resident table: lookups per second per
// CU with all lanes active and with a quarter of the lanes active (the decode
// level-2 pattern). Each lane issues `ilp` independent chains of dependent
// lookups (index = f(previous value)), like a decoder chain.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int ILP, bool INDEP>
__global__ __launch_bounds__(1024) void gather(const uint32_t* tab, uint32_t mask, int iters, uint32_t active_mod, uint32_t* sink) {
    uint32_t v[ILP];
    const uint32_t lane = threadIdx.x & 63;
    for (int c = 0; c < ILP; ++c) v[c] = (blockIdx.x * 7919u + threadIdx.x * 104729u + c * 31u) & mask;
    const bool act = (lane % active_mod) == 0;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < ILP; ++c) {
            if (act) {
                const uint32_t idx = INDEP ? ((v[c] * 2654435761u + i) & mask) : (v[c] & mask);
                v[c] = tab[idx] + (INDEP ? 0u : (uint32_t)i);
            }
        }
    }
    uint32_t s = 0;
    for (int c = 0; c < ILP; ++c) s ^= v[c];
    if (s == 0x12345678u) sink[0] = s;
}

int main() {
    const uint32_t entries = 64 * 1024;  // 256 KB table
    std::vector<uint32_t> h(entries);
    for (uint32_t i = 0; i < entries; ++i) h[i] = (i * 2654435761u) >> 7;
    uint32_t *tab, *sink;
    CK(hipMalloc(&tab, entries * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemcpy(tab, h.data(), entries * 4, hipMemcpyHostToDevice));
    hipDevice_t dev; hipDeviceProp_t prop; CK(hipGetDevice(&dev)); CK(hipGetDeviceProperties(&prop, dev));
    const int cus = prop.multiProcessorCount;
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    const int iters = 256;
    struct Cfg { int ilp; bool indep; uint32_t mod; };
    for (Cfg c : {Cfg{4, false, 1}, Cfg{4, false, 4}, Cfg{8, false, 1}, Cfg{4, true, 1}, Cfg{4, true, 4}, Cfg{1, false, 1}}) {
        for (int rep = 0; rep < 2; ++rep) {
            CK(hipEventRecord(e0));
            for (int k = 0; k < 4; ++k) {
                if (c.ilp == 4 && !c.indep) hipLaunchKernelGGL((gather<4, false>), dim3(cus), dim3(1024), 0, 0, tab, entries - 1, iters, c.mod, sink);
                if (c.ilp == 8) hipLaunchKernelGGL((gather<8, false>), dim3(cus), dim3(1024), 0, 0, tab, entries - 1, iters, c.mod, sink);
                if (c.ilp == 4 && c.indep) hipLaunchKernelGGL((gather<4, true>), dim3(cus), dim3(1024), 0, 0, tab, entries - 1, iters, c.mod, sink);
                if (c.ilp == 1) hipLaunchKernelGGL((gather<1, false>), dim3(cus), dim3(1024), 0, 0, tab, entries - 1, iters, c.mod, sink);
            }
            CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1));
            const double lookups = 4.0 * cus * 1024.0 / c.mod * iters * c.ilp;
            if (rep) printf("ilp %d indep %d active 1/%u: %.3f ms, %.3f G lane-lookups/s total, %.3f per CU per ns\n",
                            c.ilp, c.indep, c.mod, ms, lookups / ms / 1e6, lookups / ms / 1e6 / cus);
        }
    }
    return 0;
}
