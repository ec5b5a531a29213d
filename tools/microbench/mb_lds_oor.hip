// What an LDS read past the workgroup's allocation returns on this part (the decoders read such
// addresses for lanes whose entry is already final). Fills 32 KiB of dynamic LDS with nonzero words,
// then every lane reads at byte offsets past the allocation; prints how many reads were nonzero.
// Build: hipcc --offload-arch=gfx950 -O3 -o mbo mb_lds_oor.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void k_oor(uint32_t* nonzero, uint32_t* sample) {
    extern __shared__ uint32_t lds[];
    for (uint32_t i = threadIdx.x; i < 8192; i += blockDim.x) lds[i] = 0x80000000u | (i * 2654435761u);
    __syncthreads();
    const uint32_t offs[6] = {32768u, 32772u, 65536u, 262144u, 4u << 20, 0x7ffffffcu};
    uint32_t nz = 0;
    for (int k = 0; k < 6; ++k) {
        const uint32_t byte = offs[k] + 4u * threadIdx.x;
        uint32_t v;
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(byte));
        nz += v != 0u;
        if (blockIdx.x == 0 && threadIdx.x == 0) sample[k] = v;
    }
    if (nz) atomicAdd(nonzero, nz);
}

int main() {
    uint32_t *nz, *sm;
    hipMalloc(&nz, 4);
    hipMalloc(&sm, 64);
    hipMemset(nz, 0, 4);
    hipMemset(sm, 0xff, 64);
    k_oor<<<1024, 256, 32768>>>(nz, sm);
    uint32_t h = 0, s[6];
    hipMemcpy(&h, nz, 4, hipMemcpyDeviceToHost);
    hipMemcpy(s, sm, 24, hipMemcpyDeviceToHost);
    printf("out-of-range LDS reads that returned nonzero: %u of %u\n", h, 1024u * 256u * 6u);
    for (int k = 0; k < 6; ++k) printf("  sample %d: 0x%08x\n", k, s[k]);
    return 0;
}
