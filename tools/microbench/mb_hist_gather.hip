// Design-probe microbenchmarks for the Huffman hot path on gfx950 (MI355X).
// Not part of the product. Measures, on 16-bit symbol streams resident in HBM:
//   copy      : 16 B/lane read + write (HBM ceiling for this access shape)
//   read      : 16 B/lane read-only reduction
//   hist_lds16: 65 536-bin histogram, two u16 counters per LDS dword, wrap accounting
//   gat_glb4  : one 4-B gather per symbol from a 256 KiB global table (L2 resident)
//   gat_glb8  : one 8-B gather per symbol from a 512 KiB global table
//   gat_lds4  : one 4-B gather per symbol from a 128 KiB LDS table (sym & 0x7fff)
//   gat_ldsu8 : one 1-B gather per symbol from a 64 KiB LDS table
// Build: hipcc --offload-arch=gfx950 -O3 -o mb mb_hist_gather.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cmath>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ void gen_kernel(uint8_t* out, uint64_t n, const uint64_t* thr, int zipf) {
  __shared__ uint64_t t[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) t[i] = thr[i];
  __syncthreads();
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n / 8; i += stride) {
    uint64_t w = 0;
    for (int k = 0; k < 8; ++k) {
      uint64_t u = splitmix64(42ull ^ (i * 8 + k));
      uint32_t b;
      if (zipf) {
        int lo = 0, hi = 255;
        while (lo < hi) { int m = (lo + hi) >> 1; if (u < t[m]) hi = m; else lo = m + 1; }
        b = lo;
      } else b = u & 0xff;
      w |= (uint64_t)b << (8 * k);
    }
    ((uint64_t*)out)[i] = w;
  }
}

__global__ void copy_kernel(const uint4* __restrict__ in, uint4* __restrict__ out, uint64_t n16) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += stride) out[i] = in[i];
}

__global__ void read_kernel(const uint4* __restrict__ in, uint64_t n16, uint32_t* sink) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += stride) {
    uint4 v = in[i]; acc ^= v.x + v.y + v.z + v.w;
  }
  if (acc == 0x12345678) sink[0] = acc;
}

// Packed u16 histogram: word w = sym>>1 (swizzled), half = sym&1. Exact via wrap accounting.
template <int SWZ>
__global__ __launch_bounds__(1024) void hist_lds16(const uint4* __restrict__ in, uint64_t n16,
                                                    unsigned long long* __restrict__ hist) {
  extern __shared__ uint32_t lds[];
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) lds[i] = 0;
  __syncthreads();
  uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  uint64_t beg = blockIdx.x * per, end = beg + per; if (end > n16) end = n16;
  for (uint64_t i = beg + threadIdx.x; i < end; i += blockDim.x) {
    uint4 v = in[i];
    uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint32_t s = (words[k >> 1] >> (16 * (k & 1))) & 0xffff;
      uint32_t w = s >> 1;
      if (SWZ) w = w ^ (((w >> 5) * 0x9E3779B1u) >> 27);
      uint32_t inc = (s & 1) ? 0x10000u : 1u;
      uint32_t old = atomicAdd(&lds[w], inc);
      uint32_t nw = old + inc;
      if (__builtin_expect(nw < old, 0)) atomicAdd(&hist[s | 1], 65536ull);  // high half wrapped
      if (__builtin_expect(!(s & 1) && (old & 0xffff) == 0xffff, 0)) {
        atomicAdd(&hist[s], 65536ull);
        uint32_t o2 = atomicSub(&lds[w], 0x10000u);
        if (o2 < 0x10000u) atomicAdd(&hist[s | 1], (unsigned long long)(-65536ll));
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) {
    uint32_t w = i;
    if (SWZ) w = w ^ (((w >> 5) * 0x9E3779B1u) >> 27);
    uint32_t v = lds[w];
    if (v & 0xffff) atomicAdd(&hist[2 * i], (unsigned long long)(v & 0xffff));
    if (v >> 16) atomicAdd(&hist[2 * i + 1], (unsigned long long)(v >> 16));
  }
}

// v2: UNR 16-B loads in flight per thread, atomics batched, wrap checks batched.
template <int UNR, int RTN>
__global__ __launch_bounds__(1024) void hist_v2(const uint4* __restrict__ in, uint64_t n16,
                                                 unsigned long long* __restrict__ hist) {
  extern __shared__ uint32_t lds[];
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) lds[i] = 0;
  __syncthreads();
  uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  per = (per + 1023) & ~1023ull;
  uint64_t beg = blockIdx.x * per, end = beg + per; if (end > n16) end = n16;
  uint32_t sinkacc = 0;
  for (uint64_t i = beg + threadIdx.x; i < end; i += (uint64_t)blockDim.x * UNR) {
    uint4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      uint64_t j = i + (uint64_t)u * blockDim.x;
      v[u] = j < end ? in[j] : make_uint4(0, 0, 0, 0);
    }
    uint32_t old[UNR * 8];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      uint32_t words[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
      bool valid = (i + (uint64_t)u * blockDim.x) < end;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        uint32_t s = (words[k >> 1] >> (16 * (k & 1))) & 0xffff;
        uint32_t inc = valid ? ((s & 1) ? 0x10000u : 1u) : 0u;
        if (RTN) old[u * 8 + k] = atomicAdd(&lds[s >> 1], inc);
        else { __hip_atomic_fetch_add(&lds[s & 0x7fff], valid ? 1u : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
      }
    }
    if (RTN) {
      bool any = false;
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        uint32_t words[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          uint32_t s = (words[k >> 1] >> (16 * (k & 1))) & 0xffff;
          uint32_t o = old[u * 8 + k];
          uint32_t inc = (s & 1) ? 0x10000u : 1u;
          any |= (o + inc < o) | (!(s & 1) && ((o & 0xffff) == 0xffff));
        }
      }
      if (__builtin_expect(any, 0)) {
        for (int u = 0; u < UNR; ++u) {
          if (i + (uint64_t)u * blockDim.x >= end) continue;
          uint32_t words[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
          for (int k = 0; k < 8; ++k) {
            uint32_t s = (words[k >> 1] >> (16 * (k & 1))) & 0xffff;
            uint32_t o = old[u * 8 + k];
            uint32_t inc = (s & 1) ? 0x10000u : 1u;
            if (o + inc < o) atomicAdd(&hist[s | 1], 65536ull);
            if (!(s & 1) && (o & 0xffff) == 0xffff) {
              atomicAdd(&hist[s], 65536ull);
              uint32_t o2 = atomicSub(&lds[s >> 1], 0x10000u);
              if (o2 < 0x10000u) atomicAdd(&hist[s | 1], (unsigned long long)(-65536ll));
            }
          }
        }
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) {
    uint32_t v = lds[i];
    if (RTN) {
      if (v & 0xffff) atomicAdd(&hist[2 * i], (unsigned long long)(v & 0xffff));
      if (v >> 16) atomicAdd(&hist[2 * i + 1], (unsigned long long)(v >> 16));
    } else if (v) atomicAdd(&hist[i], (unsigned long long)v);
  }
}

// LDS table lookups, UNR loads in flight, results accumulated.
template <int UNR>
__global__ __launch_bounds__(1024) void gat_lds4_v2(const uint4* __restrict__ in, uint64_t n16, const uint32_t* tab, uint32_t* sink) {
  extern __shared__ uint32_t lds[];
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) lds[i] = tab[i];
  __syncthreads();
  uint64_t per = (n16 + gridDim.x - 1) / gridDim.x;
  per = (per + 1023) & ~1023ull;
  uint64_t beg = blockIdx.x * per, end = beg + per; if (end > n16) end = n16;
  uint32_t acc = 0;
  for (uint64_t i = beg + threadIdx.x; i < end; i += (uint64_t)blockDim.x * UNR) {
    uint4 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      uint64_t j = i + (uint64_t)u * blockDim.x;
      v[u] = j < end ? in[j] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      uint32_t words[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += lds[(words[k >> 1] >> (16 * (k & 1))) & 0x7fff];
    }
  }
  if (acc == 0x12345678) sink[0] = 1;
}

__global__ void hist_naive(const uint4* __restrict__ in, uint64_t n16, unsigned long long* hist) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += stride) {
    uint4 v = in[i];
    uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) atomicAdd(&hist[(words[k >> 1] >> (16 * (k & 1))) & 0xffff], 1ull);
  }
}

template <typename T>
__global__ void gat_glb(const uint4* __restrict__ in, uint64_t n16, const T* __restrict__ tab, uint32_t* sink) {
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  T acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += stride) {
    uint4 v = in[i];
    uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += tab[(words[k >> 1] >> (16 * (k & 1))) & 0xffff];
  }
  if ((uint32_t)acc == 0x12345678) sink[0] = 1;
}

__global__ __launch_bounds__(1024) void gat_lds4(const uint4* __restrict__ in, uint64_t n16, const uint32_t* tab, uint32_t* sink) {
  extern __shared__ uint32_t lds[];
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) lds[i] = tab[i];
  __syncthreads();
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += stride) {
    uint4 v = in[i];
    uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += lds[(words[k >> 1] >> (16 * (k & 1))) & 0x7fff];
  }
  if (acc == 0x12345678) sink[0] = 1;
}

__global__ void gat_ldsu8(const uint4* __restrict__ in, uint64_t n16, const uint8_t* tab, uint32_t* sink) {
  extern __shared__ uint8_t l8[];
  for (int i = threadIdx.x; i < 65536; i += blockDim.x) l8[i] = tab[i];
  __syncthreads();
  uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n16; i += stride) {
    uint4 v = in[i];
    uint32_t words[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += l8[(words[k >> 1] >> (16 * (k & 1))) & 0xffff];
  }
  if (acc == 0x12345678) sink[0] = 1;
}

struct Timer {
  hipEvent_t a, b;
  Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
  void start() { CK(hipEventRecord(a)); }
  float stop() { CK(hipEventRecord(b)); CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); return ms; }
};

int main(int argc, char** argv) {
  uint64_t n = (argc > 1 ? strtoull(argv[1], 0, 0) : (4ull << 30));
  int reps = 5;
  std::vector<uint64_t> thr(256);
  {
    double H = 0; for (int r = 1; r <= 256; ++r) H += pow(r, -1.1);
    double c = 0;
    for (int r = 1; r <= 256; ++r) { c += pow(r, -1.1) / H; thr[r - 1] = (r == 256) ? ~0ull : (uint64_t)(c * 18446744073709551616.0); }
  }
  uint64_t *d_thr; CK(hipMalloc(&d_thr, 256 * 8)); CK(hipMemcpy(d_thr, thr.data(), 2048, hipMemcpyHostToDevice));
  uint8_t *d_in, *d_out; CK(hipMalloc(&d_in, n)); CK(hipMalloc(&d_out, n));
  unsigned long long* d_hist; CK(hipMalloc(&d_hist, 65536 * 8));
  uint32_t *d_sink; CK(hipMalloc(&d_sink, 64));
  uint32_t* d_tab4; CK(hipMalloc(&d_tab4, 65536 * 4)); CK(hipMemset(d_tab4, 1, 65536 * 4));
  uint64_t* d_tab8; CK(hipMalloc(&d_tab8, 65536 * 8)); CK(hipMemset(d_tab8, 1, 65536 * 8));
  uint8_t* d_tab1; CK(hipMalloc(&d_tab1, 65536)); CK(hipMemset(d_tab1, 1, 65536));
  CK(hipFuncSetAttribute((const void*)hist_lds16<0>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)hist_lds16<1>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  CK(hipFuncSetAttribute((const void*)gat_lds4, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
  Timer t;
  uint64_t n16 = n / 16;
  for (int zipf = 1; zipf >= 0; --zipf) {
    gen_kernel<<<4096, 256>>>(d_in, n, d_thr, zipf);
    CK(hipDeviceSynchronize());
    const char* dn = zipf ? "zipf" : "unif";
    auto run = [&](const char* name, double bytes, auto fn) {
      fn(); CK(hipDeviceSynchronize());
      float best = 1e30f, sum = 0;
      for (int r = 0; r < reps; ++r) { t.start(); fn(); float ms = t.stop(); best = fminf(best, ms); sum += ms; }
      printf("%s %-10s n=%llu best %.3f ms avg %.3f ms -> %.1f GB/s (best)\n", dn, name, (unsigned long long)n, best, sum / reps, bytes / best / 1e6);
      fflush(stdout);
    };
    run("copy", 2.0 * n, [&] { copy_kernel<<<256 * 8, 256>>>((const uint4*)d_in, (uint4*)d_out, n16); });
    run("read", 1.0 * n, [&] { read_kernel<<<256 * 8, 256>>>((const uint4*)d_in, n16, d_sink); });
    for (int g : {256, 512}) {
      char nm[32];
      snprintf(nm, 32, "hist0_g%d", g);
      run(nm, 1.0 * n, [&] { (void)hipMemsetAsync(d_hist, 0, 65536 * 8); hist_lds16<0><<<g, 1024, 131072>>>((const uint4*)d_in, n16, d_hist); });
      snprintf(nm, 32, "hist1_g%d", g);
      run(nm, 1.0 * n, [&] { (void)hipMemsetAsync(d_hist, 0, 65536 * 8); hist_lds16<1><<<g, 1024, 131072>>>((const uint4*)d_in, n16, d_hist); });
    }
    // verify histogram against naive global-atomic histogram
    {
      std::vector<unsigned long long> h(65536), h2(65536);
      CK(hipMemcpy(h.data(), d_hist, 65536 * 8, hipMemcpyDeviceToHost));
      run("hist_naive", 1.0 * n, [&] { (void)hipMemsetAsync(d_hist, 0, 65536 * 8); hist_naive<<<256 * 8, 256>>>((const uint4*)d_in, n16, d_hist); });
      CK(hipMemcpy(h2.data(), d_hist, 65536 * 8, hipMemcpyDeviceToHost));
      unsigned long long s = 0; int bad = 0; for (int i = 0; i < 65536; ++i) { s += h[i]; bad += h[i] != h2[i]; }
      printf("%s hist total %llu expect %llu h[0]=%llu mismatching bins vs naive: %d\n", dn, s, (unsigned long long)(n / 2), h[0], bad);
    }
    for (int rtn = 1; rtn >= 0; --rtn) {
      auto k2 = rtn ? hist_v2<2, 1> : hist_v2<2, 0>;
      auto k4 = rtn ? hist_v2<4, 1> : hist_v2<4, 0>;
      CK(hipFuncSetAttribute((const void*)k2, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
      CK(hipFuncSetAttribute((const void*)k4, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
      run(rtn ? "h2u2rtn" : "h2u2norn", 1.0 * n, [&] { (void)hipMemsetAsync(d_hist, 0, 65536 * 8); k2<<<256, 1024, 131072>>>((const uint4*)d_in, n16, d_hist); });
      run(rtn ? "h2u4rtn" : "h2u4norn", 1.0 * n, [&] { (void)hipMemsetAsync(d_hist, 0, 65536 * 8); k4<<<256, 1024, 131072>>>((const uint4*)d_in, n16, d_hist); });
      if (rtn) {
        std::vector<unsigned long long> h(65536), h2(65536);
        CK(hipMemcpy(h.data(), d_hist, 65536 * 8, hipMemcpyDeviceToHost));
        (void)hipMemsetAsync(d_hist, 0, 65536 * 8); hist_lds16<0><<<256, 1024, 131072>>>((const uint4*)d_in, n16, d_hist);
        CK(hipMemcpy(h2.data(), d_hist, 65536 * 8, hipMemcpyDeviceToHost));
        int bad = 0; for (int i = 0; i < 65536; ++i) bad += h[i] != h2[i];
        printf("%s v2 mismatching bins vs v1: %d\n", dn, bad);
      }
    }
    CK(hipFuncSetAttribute((const void*)gat_lds4_v2<2>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    CK(hipFuncSetAttribute((const void*)gat_lds4_v2<4>, hipFuncAttributeMaxDynamicSharedMemorySize, 131072));
    run("glds4u2", 1.0 * n, [&] { gat_lds4_v2<2><<<256, 1024, 131072>>>((const uint4*)d_in, n16, d_tab4, d_sink); });
    run("glds4u4", 1.0 * n, [&] { gat_lds4_v2<4><<<256, 1024, 131072>>>((const uint4*)d_in, n16, d_tab4, d_sink); });
    run("gat_glb4", 1.0 * n, [&] { gat_glb<uint32_t><<<256 * 8, 256>>>((const uint4*)d_in, n16, d_tab4, d_sink); });
    run("gat_glb8", 1.0 * n, [&] { gat_glb<uint64_t><<<256 * 8, 256>>>((const uint4*)d_in, n16, d_tab8, d_sink); });
    run("gat_lds4", 1.0 * n, [&] { gat_lds4<<<256, 1024, 131072>>>((const uint4*)d_in, n16, d_tab4, d_sink); });
    run("gat_ldsu8", 1.0 * n, [&] { gat_ldsu8<<<256 * 2, 512, 65536>>>((const uint4*)d_in, n16, d_tab1, d_sink); });
  }
  return 0;
}
