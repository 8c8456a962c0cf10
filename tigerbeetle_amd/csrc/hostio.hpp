// Host-buffer calls without DMA-engine hand-offs. A replica's message bodies and replies live in
// host memory (the message pool, tigerbeetle.zig:853-901); registered with the executor
// (tbg_register_host) they are mapped into the GPU's address space, and these kernels move a call's
// body into HBM and its results (plus the call's scalars block) back over PCIe on the call's own
// stream. A hipMemcpyAsync between host and device memory runs on a DMA engine: each hand-off
// between it and the compute queue costs ~8-10 us of idle time per copy, more than the 1 MB body
// takes to cross PCIe (profiles/r03_commit/timeline.txt).
#pragma once

#include "events.hpp"

namespace tbg {

constexpr uint32_t kStageThreads = 256;
constexpr uint32_t kStageWords = 4;  // 16-byte words per lane per pass (all loads issued first)
// A body read across PCIe peaks with few requests in flight: 32 workgroups of 256 lanes read 1 MB
// in ~23 us (45 GB/s); 256 or more workgroups took ~29 us (tools/pciebench.hip).
constexpr uint32_t kStageInGridMax = 32;

struct StageIn {
    const uint4* src;  // mapped host body, or null (the body came by hipMemcpyAsync)
    uint4* dst;
    uint64_t words;    // 16-byte words of the body
    const uint32_t* ends_src;  // mapped pinned staging -> the call's device copies
    uint32_t* ends_dst;
    const uint64_t* ts_src;
    uint64_t* ts_dst;
    uint32_t nb;
    DevScalars* reset;  // the call's scalar words to zero (the first kernel of a call), or null
};

__global__ void __launch_bounds__(kStageThreads) stage_in(StageIn s) {
    const uint64_t tid = uint64_t(blockIdx.x) * kStageThreads + threadIdx.x;
    const uint64_t stride = uint64_t(gridDim.x) * kStageThreads;
    if (tid == 0 && s.reset) reset_call_scalars(s.reset);
    if (blockIdx.x == 0)
        for (uint32_t b = threadIdx.x; b < s.nb; b += kStageThreads) {
            s.ends_dst[b] = s.ends_src[b];
            s.ts_dst[b] = s.ts_src[b];
        }
    if (!s.src) return;
    for (uint64_t w = tid; w < s.words; w += stride * kStageWords) {
        uint4 v[kStageWords];
#pragma unroll
        for (uint32_t j = 0; j < kStageWords; j++) {
            const uint64_t x = w + j * stride;
            v[j] = x < s.words ? s.src[x] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (uint32_t j = 0; j < kStageWords; j++) {
            const uint64_t x = w + j * stride;
            if (x < s.words) s.dst[x] = v[j];
        }
    }
}

struct StageOut {
    const uint4* src;  // the call's results (16 B each), or null
    uint4* dst;        // mapped host destination
    uint32_t n;
    const unsigned long long* scalars_src;  // the scalars block, or null
    unsigned long long* scalars_dst;        // mapped pinned copy
    uint32_t scalar_words;
    // A create_transfers call's first stage_out: tr_commit's fixed failures' id slots become
    // tombstones here (null: none to release).
    const uint32_t* fix_slots;
    unsigned long long* id_slots;
    const DevScalars* scalars;
    // The call's end for a spinning host (null: none): the last workgroup to finish writes `seq`
    // into the pinned word after every workgroup's writes (system-scope fences).
    unsigned int* done;
    unsigned int* host_seq;
    unsigned int seq;
    // The last workgroup (host_seq set) also clears the call's scalar words when nothing after the
    // host's wait reads them -- no replay (stats[0]) and no post/void (pnt_resolve) -- and marks its
    // host copy kFlagStageCleared: tr_reset_scalars' work without its launch.
    bool clear;
    // When *finished == finished_epoch (tr_ingest ended the call: Call::finish_done) the kernel
    // copies nothing and publishes nothing. Null: never.
    const unsigned int* finished;
    unsigned int finished_epoch;
    // A small call's AccountEvents snapshot (ae_snapshot's work, kAeAsyncMax events), taken after
    // the workgroup has been counted: the host's wait does not include it, and it costs no launch
    // of its own. `has_snap` false: none.
    bool has_snap;
    AeSnapJob snap;
    // Workgroups [0, copy_wgs) copy and count for the sequence word; the rest only snapshot (0: all).
    uint32_t copy_wgs;
};

// The end of a stream's work for a spinning host (tbg_pulse): `seq` into the pinned word, a
// system-scope release after every earlier kernel of the stream.
__global__ void host_signal(unsigned int* host_seq, unsigned int seq) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        __threadfence_system();
        __hip_atomic_store(host_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// stage_out's copies and the sequence word (every thread of the grid calls it).
__device__ inline void stage_out_copy(const StageOut& s, uint32_t tid, uint32_t threads) {
    if (s.fix_slots) {
        const uint64_t nfix = s.scalars->fixed;
        for (uint64_t i = tid; i < nfix; i += threads) s.id_slots[s.fix_slots[i]] = kTomb;
    }
    if (s.scalars_src && blockIdx.x == 0)
        for (uint32_t w = threadIdx.x; w < s.scalar_words; w += blockDim.x)
            s.scalars_dst[w] = s.scalars_src[w];
    if (s.src)
        for (uint32_t i = tid; i < s.n; i += threads) s.dst[i] = s.src[i];
    if (s.host_seq) {
        // Every thread releases its own stores at system scope before the barrier (a fence orders
        // only the issuing wave's stores; a workgroup barrier waits at workgroup scope only): the
        // workgroup's count then covers every result and scalar word it wrote.
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t counted = s.copy_wgs ? s.copy_wgs : gridDim.x;
            if (atomicAdd(s.done, 1u) == counted - 1) {
                atomicExch(s.done, 0u);
                // (every workgroup has counted: their reads of the scalar words are done; the
                // snapshot's later reads of stats[0] find 0 either way)
                DevScalars* S = const_cast<DevScalars*>(s.scalars);
                if (s.clear && s.scalars_src && S->stats[0] == 0 && !(S->flags & kFlagPostVoid)) {
                    constexpr uint32_t fw = offsetof(DevScalars, flags) / 8;
                    static_assert(offsetof(DevScalars, flags) % 8 == 0, "flags: a word's low half");
                    s.scalars_dst[fw] = s.scalars_src[fw] | kFlagStageCleared;
                    reset_call_scalars(S);
                }
                __threadfence_system();
                __hip_atomic_store(s.host_seq, s.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
}

__global__ void __launch_bounds__(kStageThreads) stage_out(StageOut s) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t copiers = s.copy_wgs ? s.copy_wgs : gridDim.x;
    if (blockIdx.x < copiers && !(s.finished && *s.finished == s.finished_epoch))
        stage_out_copy(s, tid, copiers * blockDim.x);
    if (s.has_snap && tid < kAeAsyncMax) {
        const AeSnapJob& J = s.snap;
        if (J.speculative && J.T.scalars->stats[0] != 0) J.st.created[tid] = 0;
        else ae_snapshot_one(J, tid);
    }
}

}  // namespace tbg
