// Gather instruction cost by lane pattern (the decoder's level-2 lookups):
//   dummy : every lane issues; a fraction `frac` of the lanes read random table
//           words, the rest read word 0 (one line) -- the decoder's pattern
//   masked: only that fraction of the lanes is active (exec mask), the rest skip
//   random: every lane reads a random word
// Independent gathers (8 per lane per iteration), 16 waves per CU, an
// L2-resident 256 KB table: instruction throughput, not latency.
// build: hipcc --offload-arch=gfx950 -O3 mb_gather_mask.hip -o mbgm
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int MODE>  // 0 dummy, 1 masked, 2 random
__global__ __launch_bounds__(1024) void gather(const uint32_t* tab, uint32_t mask, int iters, uint32_t thresh,
                                               uint32_t* sink) {
    constexpr int ILP = 8;
    uint32_t acc = 0, seed = blockIdx.x * 7919u + threadIdx.x * 104729u;
    for (int i = 0; i < iters; ++i) {
        uint32_t v[ILP];
#pragma unroll
        for (int c = 0; c < ILP; ++c) {
            seed = seed * 1664525u + 1013904223u;
            const bool need = MODE == 2 || (seed >> 8) % 1000u < thresh;
            const uint32_t idx = (seed >> 4) & mask;
            if (MODE == 1) {
                v[c] = need ? tab[idx] : 0u;
            } else {
                v[c] = tab[need ? idx : 0u];
            }
        }
#pragma unroll
        for (int c = 0; c < ILP; ++c) acc += v[c];
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    const uint32_t entries = 64 * 1024;
    std::vector<uint32_t> h(entries);
    for (uint32_t i = 0; i < entries; ++i) h[i] = (i * 2654435761u) >> 7;
    uint32_t *tab, *sink;
    CK(hipMalloc(&tab, entries * 4));
    CK(hipMalloc(&sink, 64));
    CK(hipMemcpy(tab, h.data(), entries * 4, hipMemcpyHostToDevice));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int iters = 512;
    for (uint32_t thresh : {75u, 250u, 1000u}) {
        for (int mode = 0; mode < 3; ++mode) {
            if (mode == 2 && thresh != 1000u) continue;
            float best = 1e9f;
            for (int rep = 0; rep < 3; ++rep) {
                CK(hipEventRecord(e0));
                if (mode == 0) hipLaunchKernelGGL(gather<0>, dim3(cus), dim3(1024), 0, 0, tab, entries - 1, iters, thresh, sink);
                if (mode == 1) hipLaunchKernelGGL(gather<1>, dim3(cus), dim3(1024), 0, 0, tab, entries - 1, iters, thresh, sink);
                if (mode == 2) hipLaunchKernelGGL(gather<2>, dim3(cus), dim3(1024), 0, 0, tab, entries - 1, iters, thresh, sink);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            const double insts = (double)cus * 16 * iters * 8;  // wave-instructions
            printf("mode %s frac %.3f: %.3f ms, %.2f cycles/wave-instruction/CU at 2.1 GHz\n",
                   mode == 0 ? "dummy " : mode == 1 ? "masked" : "random", thresh / 1000.0, best,
                   best * 1e-3 * 2.1e9 / (insts / cus));
        }
    }
    return 0;
}
