// Microbenchmark: issue efficiency of the 64-bit Myers column step on gfx950 as a function of
// independent chains per lane (ILP) and waves per SIMD.  Each lane runs STEPS steps on CH chains
// with pseudo-random match masks from registers (no memory in the loop).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <algorithm>
#include <vector>
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

// Eight independent v_bitop3 chains per lane (each op depends only on its own chain): the VALU
// issue rate without dependency stalls, i.e. the practical peak at 8 waves per SIMD.
__global__ __launch_bounds__(256) void indep8(uint32_t* out, int steps) {
    uint32_t v[8];
    const uint32_t k1 = threadIdx.x * 0x9E3779B9u, k2 = blockIdx.x ^ 0x85EBCA6Bu;
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x + c;
    for (int s = 0; s < steps; ++s) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int c = 0; c < 8; ++c) v[c] = __builtin_amdgcn_bitop3_b32(v[c], k1, k2, 0x96);
    }
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) acc += v[c];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// The same chains with the shader clock stamped around the loop by the first lane of every block
// (MI355X_MICROARCH.md 'DVFS give-back' item 6: clock = d(s_memtime) / d(s_memrealtime) x 100 MHz).
// The stamps go to their own buffer; nothing else reads them.
__global__ __launch_bounds__(256) void addloop_stamped(uint32_t* out, int steps,
                                                       unsigned long long* stamps) {
    uint32_t a = threadIdx.x, b = blockIdx.x, c = a ^ b, d = a + b;
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
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
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
}

int main() {
    uint32_t* d_out;
    hipMalloc(&d_out, 256u * 65536 * 4);
    const int steps = 2048, blocks = 8192;
    {   // clock under load: >= 2 s of back-to-back launches, then one stamped launch
        unsigned long long* d_st;
        hipMalloc(&d_st, 2ull * blocks * 8);
        hipEvent_t a, b, w0, w1;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipEventCreate(&w0);
        hipEventCreate(&w1);
        float warm = 0.f;
        int launches = 0;
        hipEventRecord(w0);
        while (warm < 2000.f) {
            for (int i = 0; i < 8; ++i)
                hipLaunchKernelGGL(addloop, dim3(blocks), dim3(256), 0, 0, d_out, 512);
            launches += 8;
            hipEventRecord(w1);
            hipEventSynchronize(w1);
            hipEventElapsedTime(&warm, w0, w1);
        }
        hipEventRecord(a);
        hipLaunchKernelGGL(addloop_stamped, dim3(blocks), dim3(256), 0, 0, d_out, 512, d_st);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        std::vector<unsigned long long> st(2ull * blocks);
        hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost);
        std::vector<double> mhz;
        for (int i = 0; i < blocks; ++i)
            if (st[2 * i + 1]) mhz.push_back((double)st[2 * i] / (double)st[2 * i + 1] * 100.0);
        std::sort(mhz.begin(), mhz.end());
        const double med = mhz.empty() ? 0.0 : mhz[mhz.size() / 2];
        const double ops = (double)blocks * 256 * 512 * 64;
        printf("stamped bitop3 chain x4 after %.0f ms / %d launches: %.3f ms  %.2f T lane-ops/s  "
               "clock %.0f MHz (median of %zu blocks, p10 %.0f p90 %.0f)\n", warm, launches, ms,
               ops / ms / 1e9, med, mhz.size(), mhz.empty() ? 0.0 : mhz[mhz.size() / 10],
               mhz.empty() ? 0.0 : mhz[mhz.size() * 9 / 10]);
        // the same work unstamped, straight after (the stamps' branch and stores aside, the
        // two launches differ only in when they run)
        hipEventRecord(a);
        hipLaunchKernelGGL(addloop, dim3(blocks), dim3(256), 0, 0, d_out, 512);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        printf("unstamped bitop3 chain x4 right after: %.3f ms  %.2f T lane-ops/s\n", ms,
               ops / ms / 1e9);
        hipEventRecord(a);
        hipLaunchKernelGGL(addloop_stamped, dim3(blocks), dim3(256), 0, 0, d_out, 512, d_st);
        hipEventRecord(b);
        hipEventSynchronize(b);
        hipEventElapsedTime(&ms, a, b);
        hipMemcpy(st.data(), d_st, st.size() * 8, hipMemcpyDeviceToHost);
        mhz.clear();
        for (int i = 0; i < blocks; ++i)
            if (st[2 * i + 1]) mhz.push_back((double)st[2 * i] / (double)st[2 * i + 1] * 100.0);
        std::sort(mhz.begin(), mhz.end());
        printf("stamped again: %.3f ms  %.2f T lane-ops/s  clock %.0f MHz\n", ms, ops / ms / 1e9,
               mhz.empty() ? 0.0 : mhz[mhz.size() / 2]);
        hipFree(d_st);
    }
    {   // independent chains
        hipEvent_t a, b;
        hipEventCreate(&a);
        hipEventCreate(&b);
        hipLaunchKernelGGL(indep8, dim3(blocks), dim3(256), 0, 0, d_out, 2048);
        hipEventRecord(a);
        hipLaunchKernelGGL(indep8, dim3(blocks), dim3(256), 0, 0, d_out, 2048);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        const double ops = (double)blocks * 256 * 2048 * 64;
        printf("bitop3 independent x8: %.3f ms  %.2f T lane-ops/s\n", ms, ops / ms / 1e9);
    }
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
