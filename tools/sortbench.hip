// Micro-benchmark of the workgroup sorts (prims.hpp block_bitonic_sort): pulse_sort_chunks on
// random (expires_at, row) candidates, and a u32 key sort of ae_dense_emit's shape; checks the
// output order. Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/sortbench.hip -o /tmp/sortbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#include "../tigerbeetle_amd/csrc/pulse.hpp"

using namespace tbg;

template <uint32_t N, uint32_t T>
__global__ void __launch_bounds__(T) pk_msort(uint64_t* keys, uint32_t reps) {
    __shared__ PulseKey lds[N * T];
    PulseKey k[N];
    uint64_t* base = keys + uint64_t(blockIdx.x) * N * T;
    for (uint32_t rep = 0; rep < reps; rep++) {
#pragma unroll
        for (uint32_t m = 0; m < N; m++) k[m] = PulseKey{base[m * T + threadIdx.x] ^ rep, m * T + threadIdx.x, 0};
        block_merge_sort<N, T>(k, lds);
    }
#pragma unroll
    for (uint32_t m = 0; m < N; m++) base[threadIdx.x * N + m] = k[m].e;
}
template <uint32_t N, uint32_t T, bool MERGE>
__global__ void __launch_bounds__(T) u64_sort(uint64_t* keys, uint32_t reps) {
    __shared__ uint64_t lds[N * T];
    uint64_t k[N];
    uint64_t* base = keys + uint64_t(blockIdx.x) * N * T;
    for (uint32_t rep = 0; rep < reps; rep++) {
#pragma unroll
        for (uint32_t m = 0; m < N; m++) k[m] = ((base[m * T + threadIdx.x] ^ rep) << 20) | (m * T + threadIdx.x);
        if (MERGE) block_merge_sort<N, T>(k, lds);
        else block_bitonic_sort<N, T>(k, lds);
    }
#pragma unroll
    for (uint32_t m = 0; m < N; m++) base[threadIdx.x * N + m] = k[m];
}
template <uint32_t N, uint32_t T>
__global__ void __launch_bounds__(T) u32_msort(uint32_t* keys, uint32_t reps) {
    __shared__ uint32_t lds[N * T];
    uint32_t k[N];
    uint32_t* base = keys + uint64_t(blockIdx.x) * N * T;
    for (uint32_t rep = 0; rep < reps; rep++) {
#pragma unroll
        for (uint32_t m = 0; m < N; m++) k[m] = (base[m * T + threadIdx.x] & ~0xFFFu) | ((m * T + threadIdx.x) & 0xFFF);
        block_merge_sort<N, T>(k, lds);
    }
#pragma unroll
    for (uint32_t m = 0; m < N; m++) base[threadIdx.x * N + m] = k[m];
}

template <uint32_t N, uint32_t T>
__global__ void __launch_bounds__(T) pk_sort(uint64_t* keys, uint32_t reps) {
    __shared__ PulseKey lds[N * T];
    PulseKey k[N];
    uint64_t* base = keys + uint64_t(blockIdx.x) * N * T;
    for (uint32_t rep = 0; rep < reps; rep++) {
#pragma unroll
        for (uint32_t m = 0; m < N; m++) k[m] = PulseKey{base[m * T + threadIdx.x] ^ rep, m * T + threadIdx.x, 0};
        block_bitonic_sort<N, T>(k, lds);
    }
#pragma unroll
    for (uint32_t m = 0; m < N; m++) base[threadIdx.x * N + m] = k[m].e + k[m].r;
}

template <uint32_t N, uint32_t T>
__global__ void __launch_bounds__(T) u32_sort(uint32_t* keys, uint32_t reps) {
    __shared__ uint32_t lds[N * T];
    uint32_t k[N];
    uint32_t* base = keys + uint64_t(blockIdx.x) * N * T;
    for (uint32_t rep = 0; rep < reps; rep++) {
#pragma unroll
        for (uint32_t m = 0; m < N; m++) k[m] = base[m * T + threadIdx.x] ^ rep;
        block_bitonic_sort<N, T>(k, lds);
    }
#pragma unroll
    for (uint32_t m = 0; m < N; m++) base[threadIdx.x * N + m] = k[m];
}

__global__ void burn(float* out, uint32_t iters) {
    float x = threadIdx.x;
    for (uint32_t i = 0; i < iters; i++) x = x * 0.999f + 1.0f;
    if (x == 12345.f) out[0] = x;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main() {
    const uint32_t runs = 4, C = runs * kPulseSortRun;
    std::vector<uint64_t> he(C), hr(C);
    srand(1);
    for (uint32_t i = 0; i < C; i++) {
        he[i] = (uint64_t(rand()) << 12) ^ rand();
        hr[i] = i;
    }
    uint64_t *de, *dr;
    uint32_t* dl;
    unsigned long long* dc;
    CK(hipMalloc(&de, C * 8));
    CK(hipMalloc(&dr, C * 8));
    CK(hipMalloc(&dl, 64 * 4));
    CK(hipMalloc(&dc, 64));
    unsigned long long hc[5] = {0, C, 0, 0, 0};
    CK(hipMemcpy(dc, hc, sizeof(hc), hipMemcpyHostToDevice));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    float ms = 0;
    for (int it = 0; it < 5; it++) {
        CK(hipMemcpy(de, he.data(), C * 8, hipMemcpyHostToDevice));
        CK(hipMemcpy(dr, hr.data(), C * 8, hipMemcpyHostToDevice));
        CK(hipEventRecord(a));
        hipLaunchKernelGGL(pulse_sort_chunks, dim3(runs), dim3(kPulseSortThreads), 0, 0,
                           PulseRuns{de, dr, dl, kPulseSortRun}, dc, kPulseSortRun,
                           uint64_t(it & 1 ? 1ull << 62 : (1ull << 43) - 1), 20u);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        CK(hipEventElapsedTime(&ms, a, b));
        printf("pulse_sort_chunks x%u runs (%s keys): %.1f us\n", runs, it & 1 ? "two-word" : "packed", ms * 1e3);
    std::vector<uint64_t> oe(C), orr(C);
        CK(hipMemcpy(oe.data(), de, C * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(orr.data(), dr, C * 8, hipMemcpyDeviceToHost));
        bool ok = true;
        for (uint32_t r = 0; r < runs; r++) {
            std::vector<std::pair<uint64_t, uint64_t>> want;
            for (uint32_t i = 0; i < kPulseSortRun; i++) want.push_back({he[r * kPulseSortRun + i], hr[r * kPulseSortRun + i]});
            std::sort(want.begin(), want.end());
            for (uint32_t i = 0; i < kPulseSortRun; i++)
                ok &= want[i].first == oe[r * kPulseSortRun + i] && want[i].second == orr[r * kPulseSortRun + i];
        }
        printf("pulse sort order %s\n", ok ? "ok" : "WRONG");
    }
    // u32 sorts, one workgroup per block, `reps` sorts each
    const uint32_t blocks = 64;
    for (int variant = 0; variant < 2; variant++) {
        const uint32_t n = variant == 0 ? 8 * 512 : 4 * 512;
        std::vector<uint32_t> hk(blocks * n);
        for (auto& x : hk) x = uint32_t(rand());
        uint32_t* dk;
        CK(hipMalloc(&dk, hk.size() * 4));
        for (int it = 0; it < 3; it++) {
            CK(hipMemcpy(dk, hk.data(), hk.size() * 4, hipMemcpyHostToDevice));
            CK(hipEventRecord(a));
            if (variant == 0) hipLaunchKernelGGL((u32_sort<8, 512>), dim3(blocks), dim3(512), 0, 0, dk, 1u);
            else hipLaunchKernelGGL((u32_sort<4, 512>), dim3(blocks), dim3(512), 0, 0, dk, 1u);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("u32 sort %u keys x %u blocks: %.1f us\n", n, blocks, ms * 1e3);
        }
        std::vector<uint32_t> ok2(hk.size());
        CK(hipMemcpy(ok2.data(), dk, hk.size() * 4, hipMemcpyDeviceToHost));
        bool good = true;
        for (uint32_t bl = 0; bl < blocks; bl++) {
            std::vector<uint32_t> w(hk.begin() + bl * n, hk.begin() + (bl + 1) * n);
            std::sort(w.begin(), w.end());
            for (uint32_t i = 0; i < n; i++) good &= w[i] == ok2[bl * n + i];
        }
        printf("u32 sort order %s\n", good ? "ok" : "WRONG");
        CK(hipFree(dk));
    }
    // repeated sorts inside one launch (no launch overhead): per-sort time
    {
        uint32_t* dk;
        uint64_t* dk64;
        CK(hipMalloc(&dk, 64 * 8192 * 4));
        CK(hipMalloc(&dk64, 64 * 8192 * 8));
        CK(hipMemset(dk, 7, 64 * 8192 * 4));
        CK(hipMemset(dk64, 7, 64 * 8192 * 8));
        float* dummy;
        CK(hipMalloc(&dummy, 64));
        for (uint32_t reps : {1u, 11u}) {
            hipLaunchKernelGGL(burn, dim3(2048), dim3(256), 0, 0, dummy, 200000u);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((u32_sort<8, 512>), dim3(1), dim3(512), 0, 0, dk, reps);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("u32 4096 (8x512) reps %u: %.1f us\n", reps, ms * 1e3);
            hipLaunchKernelGGL(burn, dim3(2048), dim3(256), 0, 0, dummy, 200000u);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((u32_sort<8, 1024>), dim3(1), dim3(1024), 0, 0, dk, reps);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("u32 8192 (8x1024) reps %u: %.1f us\n", reps, ms * 1e3);
            hipLaunchKernelGGL(burn, dim3(2048), dim3(256), 0, 0, dummy, 200000u);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((pk_sort<8, 1024>), dim3(1), dim3(1024), 0, 0, dk64, reps);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("pulsekey 8192 (8x1024) reps %u: %.1f us\n", reps, ms * 1e3);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((pk_sort<4, 1024>), dim3(1), dim3(1024), 0, 0, dk64, reps);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("pulsekey 4096 (4x1024) reps %u: %.1f us\n", reps, ms * 1e3);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((pk_msort<8, 1024>), dim3(1), dim3(1024), 0, 0, dk64, reps);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("MERGE pulsekey 8192 (8x1024) reps %u: %.1f us\n", reps, ms * 1e3);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((pk_msort<16, 512>), dim3(1), dim3(512), 0, 0, dk64, reps);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("MERGE pulsekey 8192 (16x512) reps %u: %.1f us\n", reps, ms * 1e3);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((u32_msort<8, 512>), dim3(1), dim3(512), 0, 0, dk, reps);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("MERGE u32 4096 (8x512) reps %u: %.1f us\n", reps, ms * 1e3);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((u32_msort<4, 512>), dim3(1), dim3(512), 0, 0, dk, reps);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("MERGE u32 2048 (4x512) reps %u: %.1f us\n", reps, ms * 1e3);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((u64_sort<8, 1024, false>), dim3(1), dim3(1024), 0, 0, dk64, reps);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("BITONIC u64 8192 (8x1024) reps %u: %.1f us\n", reps, ms * 1e3);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((u64_sort<8, 1024, true>), dim3(1), dim3(1024), 0, 0, dk64, reps);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("MERGE u64 8192 (8x1024) reps %u: %.1f us\n", reps, ms * 1e3);
            CK(hipEventRecord(a));
            hipLaunchKernelGGL((u64_sort<4, 512, false>), dim3(1), dim3(512), 0, 0, dk64, reps);
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            CK(hipEventElapsedTime(&ms, a, b));
            printf("BITONIC u64 2048 (4x512) reps %u: %.1f us\n", reps, ms * 1e3);
        }
    }
    return 0;
}
