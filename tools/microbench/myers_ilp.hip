// Microbenchmark: issue efficiency of the 64-bit Myers column step on gfx950 as a function of
// independent chains per lane (ILP) and waves per SIMD.  Each lane runs STEPS steps on CH chains
// with pseudo-random match masks from registers (no memory in the loop).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../nanopore-barcoding-orc_amd/csrc/dmx_device.h"
using namespace dmx;

template <int CH>
__global__ __launch_bounds__(256) void kern(uint32_t* out, int steps, uint32_t seed) {
    uint32_t pvl[CH], pvh[CH], mvl[CH], mvh[CH];
    int d[CH];
    uint32_t x = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
    extern __shared__ uint32_t dyn[];
    if (steps < 0) dyn[threadIdx.x] = x;   // keeps the dynamic LDS allocation (occupancy knob)
#pragma unroll
    for (int c = 0; c < CH; ++c) { pvl[c] = ~0u; pvh[c] = ~0u; mvl[c] = 0; mvh[c] = 0; d[c] = 59; }
    const uint32_t e0 = x * 7u, e1 = x * 13u, e2 = x * 17u, e3 = x * 19u;
    for (int s = 0; s < steps; s += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t el = (u & 1) ? e0 : e1, eh = (u & 2) ? e2 : e3;
#pragma unroll
            for (int c = 0; c < CH; ++c)
                myers_step_hw<1>(el ^ c, eh + c, pvl[c], pvh[c], mvl[c], mvh[c], d[c], 58);
        }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) acc += d[c] + pvl[c] + mvh[c];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <int CH>
void run(uint32_t* d_out, int blocks, int steps, int waves_per_simd) {
    const size_t lds = (160 * 1024) / waves_per_simd - 1024;
    hipFuncSetAttribute((const void*)kern<CH>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    hipLaunchKernelGGL((kern<CH>), dim3(blocks), dim3(256), lds, 0, d_out, steps, 1u);
    hipEventRecord(a);
    hipLaunchKernelGGL((kern<CH>), dim3(blocks), dim3(256), lds, 0, d_out, steps, 2u);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double lane_steps = (double)blocks * 256 * steps * CH;
    printf("chains %d waves/SIMD %d: %.3f ms  %.1f G lane-steps/s\n", CH, waves_per_simd, ms,
           lane_steps / ms / 1e6);
}

__global__ __launch_bounds__(256) void addloop(uint32_t* out, int steps) {
    uint32_t a = threadIdx.x, b = blockIdx.x, c = a ^ b, d = a + b;
    for (int s = 0; s < steps; ++s) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            a = __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
            b = __builtin_amdgcn_bitop3_b32(b, c, d, 0x96);
            c = __builtin_amdgcn_bitop3_b32(c, d, a, 0x96);
            d = __builtin_amdgcn_bitop3_b32(d, a, b, 0x96);
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = a + b + c + d;
}

int main() {
    uint32_t* d_out;
    hipMalloc(&d_out, 256u * 65536 * 4);
    const int steps = 2048, blocks = 8192;
    {
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipLaunchKernelGGL(addloop, dim3(blocks), dim3(256), 0, 0, d_out, 512);
        hipEventRecord(a);
        hipLaunchKernelGGL(addloop, dim3(blocks), dim3(256), 0, 0, d_out, 512);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double ops = (double)blocks * 256 * 512 * 64;
        printf("bitop3 chain x4: %.3f ms  %.2f T lane-ops/s\n", ms, ops / ms / 1e9);
    }
    for (int w : {1, 2, 3, 4, 6, 8}) {
        run<1>(d_out, blocks, steps, w);
        run<2>(d_out, blocks, steps / 2, w);
        run<4>(d_out, blocks, steps / 4, w);
    }
    return 0;
}
