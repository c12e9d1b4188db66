// Resident set (anonymous / file) of a HIP process at each step of bringing up a device:
// runtime init, a device allocation, a memset, the first kernel launch, a second module's
// launch, a pageable H2D copy.  tools/rss_probe.py found ~1 GB anonymous after libdmx's first
// run; this separates the runtime's share from libdmx's.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

static void rss(const char* at) {
    FILE* f = fopen("/proc/self/status", "r");
    char line[256];
    long anon = 0, file = 0, hwm = 0;
    while (f && fgets(line, sizeof line, f)) {
        if (!strncmp(line, "RssAnon:", 8)) anon = atol(line + 8);
        if (!strncmp(line, "RssFile:", 8)) file = atol(line + 8);
        if (!strncmp(line, "VmHWM:", 6)) hwm = atol(line + 6);
    }
    if (f) fclose(f);
    printf("%-28s anon %6ld MB  file %6ld MB  hwm %6ld MB\n", at, anon >> 10, file >> 10, hwm >> 10);
}

__global__ void touch(uint32_t* p, size_t n) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i < n) p[i] = (uint32_t)i;
}

int main() {
    rss("start");
    hipFree(nullptr);
    rss("runtime init");
    uint32_t* d = nullptr;
    const size_t n = 256u << 20;   // 1 GiB of u32
    if (hipMalloc(&d, n * 4) != hipSuccess) return 1;
    rss("hipMalloc 1 GiB");
    hipMemset(d, 0, n * 4);
    hipDeviceSynchronize();
    rss("hipMemset");
    touch<<<(unsigned)((n + 255) / 256), 256>>>(d, n);
    hipDeviceSynchronize();
    rss("first kernel");
    std::vector<uint32_t> h(64u << 20, 1u);
    rss("host vector 256 MB");
    hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    rss("pageable H2D 256 MB");
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    rss("pageable D2H 256 MB");
    hipFree(d);
    rss("hipFree");
    return 0;
}
