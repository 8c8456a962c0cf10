// Pulse and pulse_next_timestamp resolution on hand-written kernels (no library sort or scan, no
// host synchronisation inside a pulse).
//
// Pulse (execute_expire_pending_transfers, state_machine.zig:4511-4628): the reference scans the
// expires_at index in (expires_at, timestamp) order and stops after pulse_batch_max values
// (ExpirePendingTransfers, :4875-5029; scan_lookup.zig:150-175 -- `buffer_finished` after exactly
// batch_max values, and pulse_next_timestamp becomes the last one's expiry). Here pulse_collect
// (kernels.hpp) gathers the expired candidates (expires_at, row) -- rows are appended in timestamp
// order, so (expires_at, row) orders exactly as (expires_at, timestamp) -- and:
//   * pulse_sort_chunks sorts each run of kPulseRun candidates in LDS (bitonic, 128 KB) and keeps
//     its first k (k = the batch);
//   * pulse_merge merges the sorted runs pairwise, keeping only the first k of each pair (merge
//     path: every lane finds its diagonal by binary search, then merges its outputs);
// ceil(log2(runs)) merge rounds leave the first min(candidates, k) in order. pulse_settle then
// sets the index's new length and pulse_next_timestamp on device, pulse_keep_copy compacts the
// index, pulse_apply expires the selected rows.
//
// pulse_next_timestamp of a create_transfers call with post/void (pnt_*): every update was
// recorded at its event -- min(expires_at) or reset-if-equal -- and a reset fires iff the running
// minimum before it (the value at the call's start folded with every earlier min) equals its
// expiry. pnt_tile_min reduces each tile of kPntTile events; pnt_tile_resolve gives every tile the
// minimum before it (the earlier tiles' minima), scans its events in order, and the last tile to
// finish writes the final value (timestamp_min if any reset fired, else the overall minimum).
#pragma once

#include "kernels.hpp"

namespace tbg {

constexpr uint32_t kPulseRun = 8192;      // candidates per LDS-sorted run (the batch is <= this)
constexpr uint32_t kPulseThreads = 1024;

// Sorted runs of (expires_at, row): run r at [r * kPulseRun, r * kPulseRun + len[r]).
struct PulseRuns {
    uint64_t* exp;
    uint64_t* row;
    uint32_t* len;
};

__device__ inline bool pulse_less(uint64_t ea, uint64_t ra, uint64_t eb, uint64_t rb) {
    return ea < eb || (ea == eb && ra < rb);
}

__global__ void pulse_reset_counters(unsigned long long* counters) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        counters[0] = 0;      // kept
        counters[1] = 0;      // candidates
        counters[2] = ~0ull;  // earliest unexpired expiry
        counters[3] = 0;      // expired (pulse_settle)
    }
}

// One workgroup per run: the run's candidates sorted in place, truncated to the first k.
__global__ void __launch_bounds__(kPulseThreads) pulse_sort_chunks(PulseRuns R,
                                                                  const unsigned long long* counters,
                                                                  uint32_t k) {
    __shared__ uint64_t se[kPulseRun];
    __shared__ uint64_t sr[kPulseRun];
    const uint32_t tid = threadIdx.x;
    const uint64_t C = counters[1];
    const uint64_t base = uint64_t(blockIdx.x) * kPulseRun;
    if (base >= C) {
        if (tid == 0) R.len[blockIdx.x] = 0;
        return;
    }
    const uint32_t n = uint32_t(C - base < kPulseRun ? C - base : kPulseRun);
    for (uint32_t i = tid; i < kPulseRun; i += kPulseThreads) {
        se[i] = i < n ? R.exp[base + i] : ~0ull;
        sr[i] = i < n ? R.row[base + i] : ~0ull;
    }
    __syncthreads();
    for (uint32_t size = 2; size <= kPulseRun; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            for (uint32_t t = tid; t < kPulseRun / 2; t += kPulseThreads) {
                const uint32_t lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
                const bool ascending = (lo & size) == 0;
                const uint64_t el = se[lo], rl = sr[lo], eh = se[hi], rh = sr[hi];
                if (pulse_less(eh, rh, el, rl) == ascending) {
                    se[lo] = eh;
                    sr[lo] = rh;
                    se[hi] = el;
                    sr[hi] = rl;
                }
            }
            __syncthreads();
        }
    }
    const uint32_t m = n < k ? n : k;
    for (uint32_t i = tid; i < m; i += kPulseThreads) {
        R.exp[base + i] = se[i];
        R.row[base + i] = sr[i];
    }
    if (tid == 0) R.len[blockIdx.x] = m;
}

// Runs 2r and 2r + 1 of `in` (runs_in of them) -> run r of `out`: the first min(k, sum) in order.
__global__ void __launch_bounds__(kPulseThreads) pulse_merge(PulseRuns in, uint32_t runs_in,
                                                            uint32_t k, PulseRuns out) {
    const uint32_t r = blockIdx.x, tid = threadIdx.x;
    const uint32_t a = 2 * r, b = 2 * r + 1;
    const uint32_t la = a < runs_in ? in.len[a] : 0, lb = b < runs_in ? in.len[b] : 0;
    const uint32_t L = la + lb < k ? la + lb : k;
    const uint64_t* ae = in.exp + uint64_t(a) * kPulseRun;
    const uint64_t* ar = in.row + uint64_t(a) * kPulseRun;
    const uint64_t* be = in.exp + uint64_t(b) * kPulseRun;
    const uint64_t* br = in.row + uint64_t(b) * kPulseRun;
    uint64_t* oe = out.exp + uint64_t(r) * kPulseRun;
    uint64_t* orow = out.row + uint64_t(r) * kPulseRun;
    const uint32_t per = (L + kPulseThreads - 1) / kPulseThreads;
    const uint32_t d0 = tid * per, d1 = d0 + per < L ? d0 + per : L;
    if (d0 < d1) {
        // The number of the first d0 outputs taken from a: the smallest i with a[i] after
        // b[d0 - 1 - i] (keys are distinct: rows are).
        uint32_t lo = d0 > lb ? d0 - lb : 0, hi = d0 < la ? d0 : la;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            const uint32_t j = d0 - 1 - mid;
            if (pulse_less(be[j], br[j], ae[mid], ar[mid])) hi = mid;
            else lo = mid + 1;
        }
        uint32_t i = lo, j = d0 - lo;
        for (uint32_t d = d0; d < d1; d++) {
            const bool take_a = j >= lb || (i < la && pulse_less(ae[i], ar[i], be[j], br[j]));
            if (take_a) {
                oe[d] = ae[i];
                orow[d] = ar[i];
                i++;
            } else {
                oe[d] = be[j];
                orow[d] = br[j];
                j++;
            }
        }
    }
    if (tid == 0) out.len[r] = L;
}

// After the selection (the first min(candidates, k) in order at exp / rows): the number expired,
// the index's new length (the entries still pending) and pulse_next_timestamp -- the k-th expiry
// when the scan filled its batch, else the earliest unexpired one (timestamp_max if none).
__global__ void pulse_settle(Tables T, const uint64_t* exp, unsigned long long* counters,
                             unsigned int* expired_out, uint32_t k) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t C = counters[1];
    const uint64_t expired = C < k ? C : k;
    uint64_t next = counters[2] == ~0ull ? TB_TIMESTAMP_MAX : counters[2];
    if (C >= k && k > 0) next = exp[k - 1];
    T.scalars->pulse_next_timestamp = next;
    T.scalars->expiry_count = counters[0];
    counters[3] = expired;
    *expired_out = uint32_t(expired);
}

// A sharded call's recorded updates for the caller (tbg_pnt_ops): event k's flag.
__global__ void pnt_flags(const uint64_t* ops, uint32_t n, uint8_t* flags) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) flags[k] = ops[k] != 0;
}
// ... and the selected ones as (timestamp, op) pairs, in call order.
__global__ void pnt_gather(Call<tb_transfer_t> c, const uint32_t* list, const unsigned int* count,
                           uint64_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *count) return;
    const uint32_t k = list[i];
    uint64_t ts;
    if (c.event_ts) {
        ts = c.event_ts[k];
    } else {
        uint32_t lo = 0, hi = c.n_batches - 1;  // the batch holding k: the first end > k
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (c.batch_ends[mid] > k) hi = mid;
            else lo = mid + 1;
        }
        ts = c.batch_ts[lo] - c.batch_ends[lo] + k + 1;
    }
    out[2 * i] = ts;
    out[2 * i + 1] = c.pnt_call[k];
}

// The pulse's outcome for the host: the count expired and the index's new length.
__global__ void pulse_report(const unsigned int* expired, const unsigned long long* counters,
                             unsigned long long* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    out[0] = *expired;
    out[1] = counters[0];
    __threadfence_system();
}

// The index keeps the entries still pending (the ones just expired are dropped at the next pulse).
__global__ void pulse_keep_copy(Tables T, const uint64_t* keep, const unsigned long long* counters) {
    const uint64_t n = counters[0];
    for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += uint64_t(gridDim.x) * blockDim.x)
        T.expiry[i] = keep[i];
}

// ---- pulse_next_timestamp of a call with post/void -------------------------------------------

constexpr uint32_t kPntThreads = 256;
constexpr uint32_t kPntItems = 16;
constexpr uint32_t kPntTile = kPntThreads * kPntItems;

__device__ inline uint64_t pnt_min_of(uint64_t op) {
    return (op == 0 || (op & kPntReset)) ? ~0ull : op;
}

__device__ inline uint64_t block_min_u64(uint64_t v, uint64_t* lds) {
    for (int d = 32; d >= 1; d >>= 1) {
        const uint64_t o = __shfl_xor(v, d, 64);
        v = o < v ? o : v;
    }
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) lds[wave] = v;
    __syncthreads();
    uint64_t m = ~0ull;
    for (uint32_t w = 0; w < blockDim.x / 64; w++) m = lds[w] < m ? lds[w] : m;
    __syncthreads();
    return m;
}

__global__ void __launch_bounds__(kPntThreads) pnt_tile_min(const uint64_t* ops, uint32_t n,
                                                           uint64_t* tile_min) {
    __shared__ uint64_t lds[kPntThreads / 64];
    const uint64_t base = uint64_t(blockIdx.x) * kPntTile + uint64_t(threadIdx.x) * kPntItems;
    uint64_t m = ~0ull;
    for (uint32_t i = 0; i < kPntItems; i++)
        if (base + i < n) {
            const uint64_t v = pnt_min_of(ops[base + i]);
            m = v < m ? v : m;
        }
    m = block_min_u64(m, lds);
    if (threadIdx.x == 0) tile_min[blockIdx.x] = m;
}

// words: [0] fired, [1] finished tiles (both zero between calls: the last tile clears them),
// [2] the value at the call's start. `mins_only` (a sharded call): resets are not applied here
// (they compare against the value across all shards: the caller resolves them).
__global__ void __launch_bounds__(kPntThreads) pnt_tile_resolve(Tables T, const uint64_t* ops,
                                                               uint32_t n, const uint64_t* tile_min,
                                                               unsigned long long* words,
                                                               uint32_t mins_only) {
    __shared__ uint64_t lds[kPntThreads / 64];
    __shared__ uint64_t thread_min[kPntThreads];
    __shared__ bool last;
    const uint32_t tid = threadIdx.x, tile = blockIdx.x, tiles = gridDim.x;
    const uint64_t start = T.scalars->pulse_next_timestamp;
    if (tile == 0 && tid == 0) words[2] = start;
    // The minimum before this tile: the value at the call's start and the earlier tiles' minima.
    uint64_t before = ~0ull;
    for (uint32_t t = tid; t < tile; t += kPntThreads) before = tile_min[t] < before ? tile_min[t] : before;
    before = block_min_u64(before, lds);
    before = start < before ? start : before;
    // This lane's items, then the lanes before it in the tile.
    const uint64_t base = uint64_t(tile) * kPntTile + uint64_t(tid) * kPntItems;
    uint64_t ops_l[kPntItems];
    uint64_t mine = ~0ull;
    for (uint32_t i = 0; i < kPntItems; i++) {
        ops_l[i] = base + i < n ? ops[base + i] : 0;
        const uint64_t v = pnt_min_of(ops_l[i]);
        mine = v < mine ? v : mine;
    }
    thread_min[tid] = mine;
    __syncthreads();
    uint64_t run = before;
    for (uint32_t t = 0; t < tid; t++) run = thread_min[t] < run ? thread_min[t] : run;
    bool fired = false;
    for (uint32_t i = 0; i < kPntItems; i++) {
        const uint64_t op = ops_l[i];
        if ((op & kPntReset) && !mins_only) fired |= run == (op & ~kPntReset);
        const uint64_t v = pnt_min_of(op);
        run = v < run ? v : run;
    }
    if (fired) atomicOr(&words[0], 1ull);
    __syncthreads();
    if (tid == 0) {
        __threadfence();
        last = atomicAdd(&words[1], 1ull) == tiles - 1;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    // The last tile: every tile has read the start value and reported; write the final value.
    uint64_t all = ~0ull;
    for (uint32_t t = tid; t < tiles; t += kPntThreads) all = tile_min[t] < all ? tile_min[t] : all;
    all = block_min_u64(all, lds);
    if (tid == 0) {
        const bool any = __hip_atomic_load(&words[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
        uint64_t v = start < all ? start : all;
        if (any) v = TB_TIMESTAMP_MIN;
        T.scalars->pulse_next_timestamp = v;
        words[0] = 0;
        words[1] = 0;
    }
}

}  // namespace tbg
