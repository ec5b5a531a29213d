// Cost of one chain-walk step at the walk's occupancy (1024 threads, 16 waves per CU, 64 KiB byte
// table + ring rows in LDS). Each lane runs a dependent chain of steps:
//   two_lds : window from two ring words (ds_read2st64_b32) + table byte (ds_read_u8)  (k_chain_walk)
//   one_lds : window from registers (alignbit of two VGPRs updated by selects) + table byte
//   tab_only: the table read alone (the bare LDS round trip)
// Prints ns and clocks per step (clock: 2.4 GHz assumed) for each, from hipEvent timings.
// Build: hipcc --offload-arch=gfx950 -O3 -o mbw mb_walk_step.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)
constexpr int kSteps = 1 << 14;
constexpr uint32_t kRow = 1024;

__device__ __forceinline__ void fill(uint8_t* tab, uint32_t* ring) {
    for (uint32_t i = threadIdx.x; i < 65536; i += blockDim.x) tab[i] = (uint8_t)(1 + ((i * 2654435761u) >> 27) % 22);
    for (uint32_t i = threadIdx.x; i < 17 * kRow; i += blockDim.x) ring[i] = i * 2246822519u + 0x9e3779b9u;
    __syncthreads();
}

// half-rounds of 7 steps with the walk's park logic (a code > 20 bits parks the chain until the
// half's end) and its limit test; ESC: the parked chains resolve through a global byte table
// (4 MiB, L2-resident lines) with a wait, as k_chain_walk does
template <bool ESC>
__global__ __launch_bounds__(1024) void k_half(uint32_t* sink, const uint8_t* esc) {
    __shared__ __attribute__((aligned(16))) uint8_t tab[65536];
    __shared__ __attribute__((aligned(16))) uint32_t ringa[17 * kRow];
    fill(tab, ringa);
    const uint32_t* ring = ringa + threadIdx.x;
    uint32_t m = 0x7fffffe0u - 37u * threadIdx.x, acc = 0;
    const uint32_t mlim = 0x10000000u;
    bool pk = false;
    uint32_t pW = 0;
    for (int s = 0; s < kSteps / 7; ++s) {
        uint32_t q[7], na = 0;
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            const bool ok = !pk & (m > mlim);
            const uint32_t i = (m >> 5) & 15u;
            const uint32_t* w = ring + i * kRow;
            const uint32_t W = __builtin_amdgcn_alignbit(w[kRow], w[0], m);
            uint32_t e = tab[W >> 16];
            e = e > 20u ? 0u : e;  // ~9 % escapes (the walk: ~1.4 % of codewords, ~0.6 per wave-step)
            __builtin_amdgcn_sched_barrier(0);
            const bool adv = ok & (e != 0u), park = ok ^ adv;
            na += adv ? 1u : 0u;
            m -= adv ? e : 0u;
            pk |= park;
            pW = park ? W : pW;
            q[t] = m;
        }
        if (pk) {
            m -= ESC ? (uint32_t)esc[(pW >> 10) & ((1u << 22) - 1u) & ~63u] | 1u : 21u;
            pk = false;
        }
        acc += na + q[na & 3];
    }
    if (acc == 0x12345u) sink[0] = m;
}

// k_half<true> with the park logic as VGPR arithmetic: 0 / ~0 masks from sign shifts (positions and
// limits stay below 2^31), L = e & ok (an escape reads 0), the parked window by v_bfi: no lane masks,
// no SALU on the step's dependency chain
__global__ __launch_bounds__(1024) void k_half_v(uint32_t* sink, const uint8_t* esc) {
    __shared__ __attribute__((aligned(16))) uint8_t tab[65536];
    __shared__ __attribute__((aligned(16))) uint32_t ringa[17 * kRow];
    fill(tab, ringa);
    const uint32_t* ring = ringa + threadIdx.x;
    uint32_t m = 0x7fffffe0u - 37u * threadIdx.x, acc = 0;
    const uint32_t mlim = 0x10000000u;
    uint32_t pkv = 0;  // ~0: parked
    uint32_t pW = 0;
    for (int s = 0; s < kSteps / 7; ++s) {
        uint32_t q[7], na = 0;
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            const uint32_t okv = ~pkv & (uint32_t)((int32_t)(mlim - m) >> 31);  // m > mlim and not parked
            const uint32_t i = (m >> 5) & 15u;
            const uint32_t* w = ring + i * kRow;
            const uint32_t W = __builtin_amdgcn_alignbit(w[kRow], w[0], m);
            uint32_t e = tab[W >> 16];
            e = e > 20u ? 0u : e;
            __builtin_amdgcn_sched_barrier(0);
            const uint32_t L = e & okv;
            m -= L;
            const uint32_t parkv = okv & (uint32_t)((int32_t)(e - 1u) >> 31);  // ok and e == 0
            pkv |= parkv;
            pW = __builtin_amdgcn_ubfe(0, 0, 0) | ((W & parkv) | (pW & ~parkv));
            na -= (uint32_t)((int32_t)(0u - L) >> 31);  // + (L != 0)
            q[t] = m;
        }
        if (pkv) {
            m -= (uint32_t)esc[(pW >> 10) & ((1u << 22) - 1u) & ~63u] | 1u;
            pkv = 0;
        }
        acc += na + q[na & 3];
    }
    if (acc == 0x12345u) sink[0] = m;
}

// k_half<true> without park flags: a lane past its limit reads an out-of-range LDS byte (0), an escape
// reads 0 from the table; either way it stays put (and reads 0 again), so the advancing steps are a
// prefix with no mask logic; the parked window is the half's last one. 4 VALU + the window per step.
__global__ __launch_bounds__(1024) void k_half_z(uint32_t* sink, const uint8_t* esc) {
    __shared__ __attribute__((aligned(16))) uint8_t tab[65536];
    __shared__ __attribute__((aligned(16))) uint32_t ringa[17 * kRow];
    fill(tab, ringa);
    for (uint32_t i = threadIdx.x; i < 65536; i += blockDim.x) tab[i] = tab[i] > 20 ? 0 : tab[i];
    __syncthreads();
    const uint32_t* ring = ringa + threadIdx.x;
    uint32_t m = 0x7fffffe0u - 37u * threadIdx.x, acc = 0;
    const uint32_t mlim = 0x10000000u;
    for (int s = 0; s < kSteps / 7; ++s) {
        uint32_t q[7], na = 0, W = 0, e = 0;
        bool ok = false;
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            ok = m > mlim;
            const uint32_t i = (m >> 5) & 15u;
            const uint32_t* w = ring + i * kRow;
            W = __builtin_amdgcn_alignbit(w[kRow], w[0], m);
            e = tab[ok ? (W >> 16) : 0x7ffffu];  // past the workgroup's LDS: reads 0
            __builtin_amdgcn_sched_barrier(0);
            m -= e;
            na += e != 0u;
            q[t] = m;
        }
        if (ok & (e == 0u)) m -= (uint32_t)esc[(W >> 10) & ((1u << 22) - 1u) & ~63u] | 1u;
        acc += na + q[na & 3];
    }
    if (acc == 0x12345u) sink[0] = m;
}

template <int MODE>
__global__ __launch_bounds__(1024) void k_step(uint32_t* sink) {
    __shared__ __attribute__((aligned(16))) uint8_t tab[65536];
    __shared__ __attribute__((aligned(16))) uint32_t ringa[17 * kRow];
    fill(tab, ringa);
    const uint32_t* ring = ringa + threadIdx.x;
    uint32_t m = 0x7fffffe0u - 37u * threadIdx.x;
    uint32_t w0 = ring[0], w1 = ring[kRow], acc = 0;
    for (int s = 0; s < kSteps; ++s) {
        uint32_t W;
        if (MODE == 0) {
            const uint32_t i = (m >> 5) & 15u;
            const uint32_t* w = ring + i * kRow;
            W = __builtin_amdgcn_alignbit(w[kRow], w[0], m);
        } else if (MODE == 1) {
            W = __builtin_amdgcn_alignbit(w0, w1, m);
        } else {
            W = m << 11;
        }
        const uint32_t e = tab[W >> 16];
        m -= e;
        if (MODE == 1) {  // a crossing shifts the register words (selects, as a register window would)
            const bool cr = (m & 31u) < e;
            w0 = cr ? w1 : w0;
            w1 = cr ? (w1 * 0x01000193u) ^ e : w1;
        }
        acc += e;
    }
    if (acc == 0x12345u) sink[0] = m ^ w0 ^ w1;
}

int main() {
    uint32_t* sink;
    uint8_t* esc;
    CK(hipMalloc(&sink, 64));
    CK(hipMalloc(&esc, 4 << 20));
    CK(hipMemset(esc, 3, 4 << 20));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grid = 256;
    const char* names[7] = {"two_lds", "one_lds", "tab_only", "half", "half_esc", "half_esc_v", "half_esc_z"};
    for (int rep = 0; rep < 2; ++rep) {
        for (int mode = 0; mode < 7; ++mode) {
            CK(hipEventRecord(a));
            if (mode == 0) k_step<0><<<grid, 1024>>>(sink);
            if (mode == 1) k_step<1><<<grid, 1024>>>(sink);
            if (mode == 2) k_step<2><<<grid, 1024>>>(sink);
            if (mode == 3) k_half<false><<<grid, 1024>>>(sink, esc);
            if (mode == 4) k_half<true><<<grid, 1024>>>(sink, esc);
            if (mode == 5) k_half_v<<<grid, 1024>>>(sink, esc);
            if (mode == 6) k_half_z<<<grid, 1024>>>(sink, esc);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            const double ns = ms * 1e6 / kSteps;
            printf("%-9s %8.3f ms  %7.1f ns/step  %6.0f clk/step (2.4 GHz)\n", names[mode], ms, ns, ns * 2.4);
        }
    }
    CK(hipFree(sink));
    CK(hipFree(esc));
    return 0;
}
