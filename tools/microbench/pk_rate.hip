// Microbenchmark: issue rate of the packed 16-bit integer ops the filter prescan is built from
// (v_pk_add_u16, v_pk_lshlrev_b16, v_pk_min_u16) against a 32-bit op (v_add_u32), and the whole
// packed Myers step (two 16-row blocks per 32-bit word) with its match words from registers and
// from a 16-entry LDS table (the prescan's inner loop).  8 independent chains per lane, 8192 x 256
// threads; prints T lane-ops/s (ops) or G lane-steps/s (Myers steps).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef uint16_t u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_pk(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t as_u32(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }

template <int OP>
__global__ __launch_bounds__(256) void ops(uint32_t* out, int steps) {
    uint32_t v[8];
    const uint32_t k = threadIdx.x * 0x9E3779B9u + blockIdx.x;
#pragma unroll
    for (int c = 0; c < 8; ++c) v[c] = threadIdx.x + c * 77u;
    for (int s = 0; s < steps; ++s) {
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                if (OP == 0) v[c] = v[c] + k;
                if (OP == 1) v[c] = as_u32(as_pk(v[c]) + as_pk(k));
                if (OP == 2) v[c] = as_u32(as_pk(v[c]) << (uint16_t)1) ^ k;
                if (OP == 3) v[c] = as_u32(__builtin_elementwise_min(as_pk(v[c]), as_pk(k))) + 1u;
            }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) acc += v[c];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

__device__ __forceinline__ void myers_step_pk(uint32_t eq, uint32_t& pv, uint32_t& mv, u16x2& d) {
    const uint32_t xv = eq | mv;
    const uint32_t s = as_u32(as_pk(eq & pv) + as_pk(pv));
    const uint32_t ph = mv | ~(s | pv | eq);
    const uint32_t mh = pv & ((s ^ pv) | eq);
    d = d + (as_pk(ph) >> (uint16_t)15) - (as_pk(mh) >> (uint16_t)15);
    const uint32_t ph2 = as_u32(as_pk(ph) << (uint16_t)1);
    const uint32_t mh2 = as_u32(as_pk(mh) << (uint16_t)1);
    pv = mh2 | ~(xv | ph2);
    mv = ph2 & xv;
}

// CH chains; LDS = true: match words from a 16-entry LDS table indexed by bytes of a register
template <int CH, bool LDS>
__global__ __launch_bounds__(256) void steps_pk(uint32_t* out, int steps, uint32_t seed) {
    __shared__ uint32_t tab[16];
    if (threadIdx.x < 16) tab[threadIdx.x] = (threadIdx.x * 0x01234567u) ^ seed;
    __syncthreads();
    uint32_t pv[CH], mv[CH];
    u16x2 d[CH], m[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        pv[c] = ~0u;
        mv[c] = 0u;
        d[c] = as_pk(0x00100010u);
        m[c] = as_pk(0xFFFFFFFFu);
    }
    uint32_t x = seed ^ (blockIdx.x * 256 + threadIdx.x) * 2654435761u;
    for (int s = 0; s < steps; s += 16) {
        x = x * 1664525u + 1013904223u;
        const uint32_t by[4] = {x & 0x3C3C3C3Cu, (x >> 2) & 0x3C3C3C3Cu, (x << 2) & 0x3C3C3C3Cu,
                                (x >> 4) & 0x3C3C3C3Cu};
        uint32_t eq[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const uint32_t off = __builtin_amdgcn_ubfe(by[q & 3], 8 * (q >> 2), 8);
            eq[q] = LDS ? *reinterpret_cast<const uint32_t*>(
                              reinterpret_cast<const char*>(tab) + off)
                        : (x ^ (off * 0x9E3779B9u));
        }
#pragma unroll
        for (int q = 0; q < 16; ++q)
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                myers_step_pk(eq[q] ^ (uint32_t)c, pv[c], mv[c], d[c]);
                m[c] = __builtin_elementwise_min(m[c], d[c]);
            }
    }
    uint32_t acc = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) acc += pv[c] + mv[c] + as_u32(m[c]);
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

template <class F>
float timed(F launch) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    launch();
    hipEventRecord(a);
    launch();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    uint32_t* d_out;
    hipMalloc(&d_out, 256u * 8192 * 4);
    const int blocks = 8192, steps = 512;
    const double lane_ops = (double)blocks * 256 * steps * 64;
    const char* names[4] = {"v_add_u32", "v_pk_add_u16", "v_pk_lshlrev_b16 + v_xor",
                            "v_pk_min_u16 + v_add"};
    float ms[4];
    ms[0] = timed([&] { hipLaunchKernelGGL(ops<0>, dim3(blocks), dim3(256), 0, 0, d_out, steps); });
    ms[1] = timed([&] { hipLaunchKernelGGL(ops<1>, dim3(blocks), dim3(256), 0, 0, d_out, steps); });
    ms[2] = timed([&] { hipLaunchKernelGGL(ops<2>, dim3(blocks), dim3(256), 0, 0, d_out, steps); });
    ms[3] = timed([&] { hipLaunchKernelGGL(ops<3>, dim3(blocks), dim3(256), 0, 0, d_out, steps); });
    for (int i = 0; i < 4; ++i)
        printf("%s: %.3f ms  %.2f T lane-ops/s (x%d ops per chain step)\n", names[i], ms[i],
               lane_ops * (i >= 2 ? 2 : 1) / ms[i] / 1e9, i >= 2 ? 2 : 1);
    const int ps = 4096;
    auto pk = [&](auto kern, int ch, const char* what) {
        const float t = timed([&] {
            hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, 0, d_out, ps, 7u);
        });
        printf("packed Myers step %s chains %d: %.3f ms  %.2f G lane-steps/s (2 columns each)\n",
               what, ch, t, (double)blocks * 256 * ps * ch / t / 1e6);
    };
    pk(steps_pk<1, false>, 1, "regs");
    pk(steps_pk<2, false>, 2, "regs");
    pk(steps_pk<4, false>, 4, "regs");
    pk(steps_pk<1, true>, 1, "lds");
    pk(steps_pk<2, true>, 2, "lds");
    return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
