// Microbenchmark: the HBM write ceiling for record-sized output (the AccountEvents emit writes 256-B
// records, 2.56 GB per 10M-event step). 16-byte stores over a 2.56 GB buffer, grid-stride, with
// non-temporal and plain stores, at several grid shapes; and a copy (read + write) for reference.
// Usage: ./writebench  (hipcc --offload-arch=gfx950 -O3 tools/writebench.hip -o writebench)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

__global__ void write_nt(v4u* p, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += stride) {
        const v4u v = {uint32_t(i), uint32_t(i >> 32), 1u, 2u};
        __builtin_nontemporal_store(v, &p[i]);
    }
}
__global__ void write_plain(v4u* p, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += stride) {
        const v4u v = {uint32_t(i), uint32_t(i >> 32), 1u, 2u};
        p[i] = v;
    }
}
__global__ void copy_nt(const v4u* s, v4u* d, uint64_t n) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n; i += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(&s[i]), &d[i]);
}

int main() {
    const uint64_t bytes = 2560ull << 20, n = bytes / 16;
    v4u *a = nullptr, *b = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    hipMemset(a, 0, bytes);
    hipMemset(b, 0, bytes);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int grids[] = {256, 1024, 4096, 16384};
    const int blocks[] = {256, 1024};
    for (int kind = 0; kind < 3; kind++) {
        for (int bl : blocks)
            for (int g : grids) {
                float best = 1e9f;
                for (int rep = 0; rep < 5; rep++) {
                    hipEventRecord(e0);
                    if (kind == 0) hipLaunchKernelGGL(write_nt, dim3(g), dim3(bl), 0, 0, a, n);
                    else if (kind == 1) hipLaunchKernelGGL(write_plain, dim3(g), dim3(bl), 0, 0, a, n);
                    else hipLaunchKernelGGL(copy_nt, dim3(g), dim3(bl), 0, 0, b, a, n);
                    hipEventRecord(e1);
                    hipEventSynchronize(e1);
                    float ms = 0;
                    hipEventElapsedTime(&ms, e0, e1);
                    if (ms < best) best = ms;
                }
                const double moved = kind == 2 ? 2.0 * bytes : double(bytes);
                printf("%-11s grid %5d x %4d: %.3f ms  %.2f TB/s\n",
                       kind == 0 ? "write_nt" : kind == 1 ? "write_plain" : "copy_nt", g, bl, best,
                       moved / (best * 1e-3) / 1e12);
            }
    }
    hipFree(a);
    hipFree(b);
    return 0;
}
