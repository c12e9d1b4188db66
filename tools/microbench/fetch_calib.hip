// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the filter kernel's access patterns on
// gfx950 (MI355X_MICROARCH.md: FETCH_SIZE is exact-half for 16-B/lane streaming reads; other
// widths uncalibrated).  Each kernel moves a known number of bytes once from HBM (buffers of
// 2 GiB, far beyond the 256 MiB Infinity Cache):
//   stream16  : 16 B per lane, consecutive lanes consecutive 16-B words (the documented case)
//   stream8   : 8 B per lane, consecutive
//   seg       : the filter's pattern — lane i of a wave reads five aligned 64-nt blocks
//               (16 B of codes + 8 B of no-match bits each) starting at its segment,
//               segments of 234 nt, consecutive lanes consecutive segments
//   write40   : 40-B records written by consecutive lanes (the window records)
// Run under `rocprofv3 --pmc FETCH_SIZE` (then WRITE_SIZE) and compare with the printed bytes.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void stream16(const uint4* __restrict__ a, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void stream8(const uint2* __restrict__ a, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint2 v = a[i];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// seq: 2-bit codes (16 B per 64 nt), nm: 1-bit mask (8 B per 64 nt); nseg segments of 234 nt.
__global__ void seg(const uint4* __restrict__ seq, const uint2* __restrict__ nm, size_t nseg,
                    uint32_t* out) {
    uint32_t acc = 0;
    for (size_t s = blockIdx.x * (size_t)blockDim.x + threadIdx.x; s < nseg;
         s += (size_t)gridDim.x * blockDim.x) {
        const size_t g = s * 234;          // first nt of the segment
        const size_t blk = g >> 6;
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint4 c = seq[blk + k];
            const uint2 m = nm[blk + k];
            acc ^= c.x ^ c.y ^ c.z ^ c.w ^ m.x ^ m.y;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

struct Rec40 {
    uint32_t w[10];
};

__global__ void write40(Rec40* __restrict__ o, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        Rec40 r;
        for (int k = 0; k < 10; ++k) r.w[k] = (uint32_t)(i * 10 + k);
        o[i] = r;
    }
}

int main() {
    const size_t bytes = (size_t)2 << 30;
    void *a, *b;
    uint32_t* out;
    if (hipMalloc(&a, bytes + 4096) != hipSuccess || hipMalloc(&b, bytes / 2 + 4096) != hipSuccess ||
        hipMalloc((void**)&out, 64) != hipSuccess)
        return 1;
    hipMemset(a, 1, bytes + 4096);
    hipMemset(b, 2, bytes / 2 + 4096);
    const dim3 grid(256 * 16), block(256);
    hipLaunchKernelGGL(stream16, grid, block, 0, 0, (const uint4*)a, bytes / 16, out);
    hipLaunchKernelGGL(stream8, grid, block, 0, 0, (const uint2*)a, bytes / 8, out);
    // seq region: 2 GiB = 8 Gnt; mask region (1/2 of it) covers the same nt
    const size_t nt = bytes * 4;
    const size_t nseg = (nt - 320) / 234;
    hipLaunchKernelGGL(seg, grid, block, 0, 0, (const uint4*)a, (const uint2*)b, nseg, out);
    const size_t nrec = bytes / 40;
    hipLaunchKernelGGL(write40, grid, block, 0, 0, (Rec40*)a, nrec);
    hipDeviceSynchronize();
    printf("stream16 read bytes %zu\n", bytes);
    printf("stream8 read bytes %zu\n", bytes);
    printf("seg read bytes (unique) %zu seq + %zu mask = %zu\n", nt / 4, nt / 8, nt / 4 + nt / 8);
    printf("write40 write bytes %zu\n", nrec * 40);
    return 0;
}
