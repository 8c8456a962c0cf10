// Microbenchmark: a kernel reading a 1 MB body from registered host memory (mapped) into HBM, by
// grid size and loads in flight per lane, against hipMemcpyAsync; and writing a 128 KB reply back.
// Build: hipcc --offload-arch=gfx950 -O3 tools/pciebench.hip -o tools/pciebench.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

template <int ITEMS>
__global__ void pull(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t words) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t w = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; w < words; w += stride * ITEMS) {
        uint4 v[ITEMS];
#pragma unroll
        for (int j = 0; j < ITEMS; j++) v[j] = w + j * stride < words ? src[w + j * stride] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int j = 0; j < ITEMS; j++) if (w + j * stride < words) dst[w + j * stride] = v[j];
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main() {
    const size_t bytes = 1 << 20, words = bytes / 16;
    void* host = aligned_alloc(4096, bytes);
    memset(host, 1, bytes);
    CK(hipHostRegister(host, bytes, hipHostRegisterMapped));
    void* dhost;
    CK(hipHostGetDevicePointer(&dhost, host, 0));
    void* pinned;
    CK(hipHostMalloc(&pinned, bytes, hipHostMallocCoherent | hipHostMallocMapped));
    void* dpinned;
    CK(hipHostGetDevicePointer(&dpinned, pinned, 0));
    uint4* dev;
    CK(hipMalloc(&dev, bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float ms;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    for (int rep = 0; rep < 2; rep++) {
        CK(hipEventRecord(a, s));
        CK(hipMemcpyAsync(dev, host, bytes, hipMemcpyHostToDevice, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("hipMemcpyAsync 1 MB registered: %.1f us (%.1f GB/s)\n", ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    }
    const int grids[] = {32, 64, 128, 256, 512, 1024};
    for (int which = 0; which < 2; which++) {
        const uint4* src = (const uint4*)(which ? dpinned : dhost);
        for (int g : grids) {
            for (int items : {1, 4, 8}) {
                float best = 1e9;
                for (int rep = 0; rep < 3; rep++) {
                    CK(hipEventRecord(a, s));
                    if (items == 1) hipLaunchKernelGGL(pull<1>, dim3(g), dim3(256), 0, s, src, dev, words);
                    if (items == 4) hipLaunchKernelGGL(pull<4>, dim3(g), dim3(256), 0, s, src, dev, words);
                    if (items == 8) hipLaunchKernelGGL(pull<8>, dim3(g), dim3(256), 0, s, src, dev, words);
                    CK(hipEventRecord(b, s));
                    CK(hipEventSynchronize(b));
                    CK(hipEventElapsedTime(&ms, a, b));
                    best = ms < best ? ms : best;
                }
                printf("%s grid %4d items %d: %.1f us (%.1f GB/s)\n", which ? "hostmalloc-coherent" : "registered",
                       g, items, best * 1e3, bytes / (best * 1e-3) / 1e9);
            }
        }
    }
    return 0;
}
