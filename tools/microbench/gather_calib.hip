// Calibration of rocprofv3 FETCH_SIZE for GATHERS on gfx950.
//
// MI355X_MICROARCH.md: FETCH_SIZE = TCC_EA0_RDREQ x 64 B reports exactly half of the bytes of a
// wide coalesced streaming read (128-B requests tallied at 64 B); other widths are
// uncalibrated.  The verify and band kernels gather 4-16 B per lane from unrelated lines, so
// their traffic needs its own factor.  Each kernel below touches every line of a 2 GiB buffer
// (far beyond L2 and the 256 MiB Infinity Cache) exactly once, in a scattered order (line =
// i * odd constant mod 2^24, a bijection), so the fabric must deliver each line once:
//   line4    : 4 B at offset 0 of the line (one lane per line)
//   line4x2  : 4 B at offset 0 and 4 B at offset 64 of the line (both 64-B halves)
//   line8    : 8 B at offset 0
//   line16   : 16 B at offset 0
//   stream16 : the documented case (16 B per lane, consecutive), for the ½ check
// If a request is one 64-B half (tallied exactly), line4 reports 64 B per line and line4x2 128;
// if a request is the whole 128-B line (tallied as 64), both report 64 B per line.  Run under
// `rocprofv3 --pmc FETCH_SIZE` and `--pmc TCC_EA0_RDREQ_sum` (separate passes); the program
// prints each kernel's line count and time (HIP events).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr uint32_t kLines = 1u << 24;   // 2 GiB of 128-B lines
constexpr uint32_t kMul = 0x9E3779B1u;  // odd: i -> i * kMul mod 2^24 is a bijection

__global__ void line4(const uint32_t* __restrict__ a, uint32_t* out) {
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < kLines; i += gridDim.x * blockDim.x) {
        const uint32_t l = (i * kMul) & (kLines - 1);
        acc ^= a[(size_t)l * 32];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void line4x2(const uint32_t* __restrict__ a, uint32_t* out) {
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < kLines; i += gridDim.x * blockDim.x) {
        const uint32_t l = (i * kMul) & (kLines - 1);
        acc ^= a[(size_t)l * 32] + a[(size_t)l * 32 + 16];
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void line8(const uint2* __restrict__ a, uint32_t* out) {
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < kLines; i += gridDim.x * blockDim.x) {
        const uint32_t l = (i * kMul) & (kLines - 1);
        const uint2 v = a[(size_t)l * 16];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void line16(const uint4* __restrict__ a, uint32_t* out) {
    uint32_t acc = 0;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < kLines; i += gridDim.x * blockDim.x) {
        const uint32_t l = (i * kMul) & (kLines - 1);
        const uint4 v = a[(size_t)l * 8];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void stream16(const uint4* __restrict__ a, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t bytes = (size_t)kLines * 128;
    void* a;
    uint32_t* out;
    if (hipMalloc(&a, bytes + 4096) != hipSuccess || hipMalloc((void**)&out, 64) != hipSuccess)
        return 1;
    hipMemset(a, 1, bytes + 4096);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const dim3 grid(256 * 16), block(256);
    auto timed = [&](const char* name, auto launch) {
        launch();   // warm-up (page tables)
        hipEventRecord(e0, 0);
        launch();
        hipEventRecord(e1, 0);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%s lines %u ms %.3f lines_per_s %.4g\n", name, kLines, ms, kLines / (ms * 1e-3));
    };
    timed("line4", [&] { hipLaunchKernelGGL(line4, grid, block, 0, 0, (const uint32_t*)a, out); });
    timed("line4x2", [&] { hipLaunchKernelGGL(line4x2, grid, block, 0, 0, (const uint32_t*)a, out); });
    timed("line8", [&] { hipLaunchKernelGGL(line8, grid, block, 0, 0, (const uint2*)a, out); });
    timed("line16", [&] { hipLaunchKernelGGL(line16, grid, block, 0, 0, (const uint4*)a, out); });
    timed("stream16", [&] {
        hipLaunchKernelGGL(stream16, grid, block, 0, 0, (const uint4*)a, bytes / 16, out);
    });
    printf("stream16 bytes %zu\n", bytes);
    return hipDeviceSynchronize() == hipSuccess ? 0 : 2;
}
