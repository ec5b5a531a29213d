// Design probe (not part of the product): LDS atomic add rate on gfx950, returning
// (ds_add_rtn_u32, what the histogram's wrap accounting needs) against non-returning
// (ds_add_u32). One 1024-thread workgroup per CU over a 128 KiB LDS image, as k_hist16.
// Addresses come from a per-lane hash (no HBM traffic); `mask` narrows them to model hot bins.
// Build: hipcc --offload-arch=gfx950 -O3 -o mbl mb_lds_atomic.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

template <int MODE>  // 0: ds_add_rtn, 1: ds_add (no return), 2: ds_read + ds_write (no atomicity)
__global__ __launch_bounds__(1024) void k_lds(uint32_t iters, uint32_t mask, uint32_t* sink) {
  extern __shared__ uint32_t lds[];
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) lds[i] = 0;
  __syncthreads();
  uint32_t x = (blockIdx.x * 1024u + threadIdx.x) * 0x9E3779B9u + 1u, acc = 0;
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      x ^= x << 13; x ^= x >> 17; x ^= x << 5;
      const uint32_t a = (x >> 7) & mask;
      if (MODE == 0) acc += atomicAdd(&lds[a], 1u);
      else if (MODE == 1) __hip_atomic_fetch_add(&lds[a], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else { lds[a] = lds[a] + 1u; }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) acc += lds[i];
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  int dev = 0, ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  uint32_t* sink;
  CK(hipMalloc(&sink, 4));
  const uint32_t iters = 4096;
  CK(hipFuncSetAttribute((const void*)k_lds<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_lds<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)k_lds<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const char* names[3] = {"ds_add_rtn", "ds_add", "read+write"};
  const uint32_t masks[3] = {32767u, 1023u, 31u};
  for (uint32_t m : masks) {
    for (int mode = 0; mode < 3; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(e0));
        if (mode == 0) hipLaunchKernelGGL(k_lds<0>, dim3(ncu), dim3(1024), 131072, 0, iters, m, sink);
        else if (mode == 1) hipLaunchKernelGGL(k_lds<1>, dim3(ncu), dim3(1024), 131072, 0, iters, m, sink);
        else hipLaunchKernelGGL(k_lds<2>, dim3(ncu), dim3(1024), 131072, 0, iters, m, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double ops = (double)ncu * 1024.0 * iters * 8.0;
        if (rep) printf("mask %5u %-11s %8.3f ms  %7.1f G lane-ops/s  %.2f lanes/clk/CU @2.4GHz\n", m, names[mode], ms,
                        ops / ms / 1e6, ops / (ms * 1e-3) / ncu / 2.4e9);
      }
    }
  }
  CK(hipGetLastError());
  return 0;
}
