// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access shapes the
// Huffman path uses (MI355X_MICROARCH.md: only 16-B/lane coalesced reads and
// stores are calibrated; other widths must be calibrated on a known byte
// count). Each kernel touches exactly 1 GiB (4x the Infinity Cache):
//   rd_coalesced : lane-consecutive uint4 loads            (k_hist16)
//   rd_lane64    : lane reads 64 contiguous B as 4 x uint4 (k_pack_count, k_pack_write input)
//   rd_chunk64   : lane streams its own region in 64-B chunks (k_decode payload reader)
//   wr_u32       : lane-consecutive u32 stores             (k_pack_write output words)
//   wr_uint4_b32 : lane writes 32 symbols (64 B) as 4 uint4 (k_decode output burst)
// Build: hipcc --offload-arch=gfx950 -O3 -o mbc mb_pmc_calib.hip
// Run:   rocprofv3 --pmc FETCH_SIZE -d D -o run --output-format csv -- ./mbc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

constexpr uint64_t kBytes = 1ull << 30;

__global__ __launch_bounds__(256) void rd_coalesced(const uint4* in, uint32_t* sink) {
    const uint64_t n = kBytes / 16, stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint4 v = in[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void rd_lane64(const uint4* in, uint32_t* sink) {
    const uint64_t n = kBytes / 64, stride = (uint64_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const uint4* p = in + 4 * i;
#pragma unroll
        for (int q = 0; q < 4; ++q) { const uint4 v = p[q]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void rd_chunk64(const uint4* in, uint32_t* sink) {
    const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t per = kBytes / 64 / lanes;  // chunks per lane
    const uint64_t lane = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t acc = 0;
    for (uint64_t c = 0; c < per; ++c) {
        const uint4* p = in + 4 * (lane * per + c);
#pragma unroll
        for (int q = 0; q < 4; ++q) { const uint4 v = p[q]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ __launch_bounds__(256) void wr_u32(uint32_t* out) {
    const uint64_t n = kBytes / 4, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = (uint32_t)i;
}

__global__ __launch_bounds__(256) void wr_uint4_b32(uint4* out) {
    const uint64_t n = kBytes / 64, stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        uint4* p = out + 4 * i;
#pragma unroll
        for (int q = 0; q < 4; ++q) p[q] = make_uint4((uint32_t)i, q, 1, 2);
    }
}

int main() {
    uint8_t* buf;
    uint32_t* sink;
    CK(hipMalloc(&buf, kBytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(buf, 1, kBytes));
    const int grid = 256 * 16;
    rd_coalesced<<<grid, 256>>>((const uint4*)buf, sink);
    rd_lane64<<<grid, 256>>>((const uint4*)buf, sink);
    rd_chunk64<<<grid, 256>>>((const uint4*)buf, sink);
    wr_u32<<<grid, 256>>>((uint32_t*)buf);
    wr_uint4_b32<<<grid, 256>>>((uint4*)buf);
    CK(hipDeviceSynchronize());
    printf("calibration kernels done: each touches %llu bytes\n", (unsigned long long)kBytes);
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}
