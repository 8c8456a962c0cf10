// Pulse and pulse_next_timestamp resolution on hand-written kernels (no library sort or scan, no
// host synchronisation inside a pulse).
//
// Pulse (execute_expire_pending_transfers, state_machine.zig:4511-4628): the reference scans the
// expires_at index in (expires_at, timestamp) order and stops after pulse_batch_max values
// (ExpirePendingTransfers, :4875-5029; scan_lookup.zig:150-175 -- `buffer_finished` after exactly
// batch_max values, and pulse_next_timestamp becomes the last one's expiry). Here pulse_collect
// (kernels.hpp) gathers the expired candidates (expires_at, row) -- rows are appended in timestamp
// order, so (expires_at, row) orders exactly as (expires_at, timestamp) -- and:
//   * pulse_sort_chunks sorts each run of kPulseSortRun candidates (prims.hpp block_bitonic_sort:
//     4 keys per lane in registers, shuffles within a wave, LDS across waves; one-word keys when
//     the candidates' expiry span allows, PulsePack) and keeps its first k (k = the batch);
//   * pulse_merge merges the sorted runs pairwise, a launch per level, keeping only the first k of
//     each pair (kPulseSegs workgroups per pair: merge-path diagonals, inputs in LDS, outputs
//     through LDS to coalesced stores);
// ceil(log2(runs)) merge levels leave the first min(candidates, k) in order. The root then sets
// the index's new length and pulse_next_timestamp on device and reports to the host (the kept
// entries, written by pulse_collect, become the index), pulse_apply expires the selected rows.
//
// pulse_next_timestamp of a create_transfers call with post/void (pnt_*): every update was
// recorded at its event -- min(expires_at) or reset-if-equal -- and a reset fires iff the running
// minimum before it (the value at the call's start folded with every earlier min) equals its
// expiry. pnt_tile_min reduces each tile of kPntTile events; pnt_tile_resolve gives every tile the
// minimum before it (the earlier tiles' minima), scans its events in order, and the last tile to
// finish writes the final value (timestamp_min if any reset fired, else the overall minimum).
#pragma once

#include "kernels.hpp"
#include "prims.hpp"

namespace tbg {

constexpr uint32_t kPulseRun = 8192;         // the longest merged run (the batch is <= this)
constexpr uint32_t kPulseThreads = 1024;     // (pulse_merge)
constexpr uint32_t kPulseSortRun = 2048;     // candidates per sorted run (pulse_sort_chunks)
constexpr uint32_t kPulseSortThreads = 512;
constexpr uint32_t kPulseSortItems = kPulseSortRun / kPulseSortThreads;

// Sorted runs of (expires_at, row): run r at [r * stride, r * stride + len[r]).
struct PulseRuns {
    uint64_t* exp;
    uint64_t* row;
    uint32_t* len;
    uint32_t stride;
};

__device__ inline bool pulse_less(uint64_t ea, uint64_t ra, uint64_t eb, uint64_t rb) {
    return ea < eb || (ea == eb && ra < rb);
}

__device__ inline void pulse_counters_clear(unsigned long long* counters) {
    counters[0] = 0;      // kept
    counters[1] = 0;      // candidates
    counters[2] = ~0ull;  // earliest unexpired expiry
    counters[3] = 0;      // expired (pulse_settle)
    counters[4] = ~0ull;  // earliest candidate expiry
}
__global__ void pulse_reset_counters(unsigned long long* counters) {
    if (threadIdx.x == 0 && blockIdx.x == 0) pulse_counters_clear(counters);
}

// A candidate's sort key: (expires_at, row).
struct PulseKey {
    uint64_t e;
    uint32_t r, pad;
};
__device__ inline bool sort_less(const PulseKey& a, const PulseKey& b) {
    return a.e < b.e || (a.e == b.e && a.r < b.r);
}
__device__ inline PulseKey sort_shfl_xor(const PulseKey& k, int mask) {
    return PulseKey{__shfl_xor(k.e, mask, 64), __shfl_xor(k.r, mask, 64), 0};
}

// Candidates expire at or before the pulse's timestamp and after the earliest candidate expiry
// (counters[4], pulse_collect): when that span fits, (expires_at - earliest) << row_bits | row is
// one u64 that orders as (expires_at, row) -- the sorts and merges move and compare one 8-byte
// word (a third of the LDS traffic and shuffles of the two-word key, measured 3x faster:
// tools/sortbench.hip); else they take the two-word key.
struct PulsePack {
    uint64_t base;
    uint32_t row_bits;
    bool packed;
    __device__ uint64_t key(uint64_t e, uint64_t r) const { return ((e - base) << row_bits) | r; }
};
__device__ inline PulsePack pulse_pack(const unsigned long long* counters, uint64_t timestamp,
                                       uint32_t row_bits) {
    const uint64_t lo = counters[4];
    const uint64_t span = timestamp >= lo ? timestamp - lo : ~0ull;
    return PulsePack{lo, row_bits, lo != ~0ull && (span >> (63 - row_bits)) == 0};
}

// A run of candidates sorted in one workgroup (kPulseSortRun keys, 4 per lane, prims.hpp
// block_bitonic_sort), truncated to the first k, in place.
template <typename K, typename Pack, typename Unpack>
__device__ void pulse_sort_run(PulseRuns R, uint64_t base, uint32_t n, uint32_t k, K* lds, K none,
                               Pack pack, Unpack unpack) {
    const uint32_t tid = threadIdx.x;
    K key[kPulseSortItems];
#pragma unroll
    for (uint32_t m = 0; m < kPulseSortItems; m++) {  // (any placement: coalesced loads)
        const uint32_t i = m * kPulseSortThreads + tid;
        key[m] = i < n ? pack(R.exp[base + i], R.row[base + i]) : none;
    }
    block_bitonic_sort<kPulseSortItems, kPulseSortThreads>(key, lds);
#pragma unroll
    for (uint32_t m = 0; m < kPulseSortItems; m++) lds[tid * kPulseSortItems + m] = key[m];
    __syncthreads();
    const uint32_t m_out = n < k ? n : k;
    for (uint32_t i = tid; i < m_out; i += kPulseSortThreads) unpack(lds[i], &R.exp[base + i], &R.row[base + i]);
}

__global__ void __launch_bounds__(kPulseSortThreads) pulse_sort_chunks(PulseRuns R,
                                                                      const unsigned long long* counters,
                                                                      uint32_t k, uint64_t timestamp,
                                                                      uint32_t row_bits) {
    __shared__ union {
        uint64_t u[kPulseSortRun];
        PulseKey p[kPulseSortRun];
    } lds;
    const uint64_t C = counters[1];
    const uint64_t base = uint64_t(blockIdx.x) * kPulseSortRun;
    if (base >= C) {
        if (threadIdx.x == 0) R.len[blockIdx.x] = 0;
        return;
    }
    const uint32_t n = uint32_t(C - base < kPulseSortRun ? C - base : kPulseSortRun);
    const PulsePack P = pulse_pack(counters, timestamp, row_bits);
    if (P.packed) {
        const uint64_t mask = (1ull << row_bits) - 1;
        pulse_sort_run<uint64_t>(
            R, base, n, k, lds.u, ~0ull, [&](uint64_t e, uint64_t r) { return P.key(e, r); },
            [&](uint64_t v, uint64_t* e, uint64_t* r) {
                *e = P.base + (v >> row_bits);
                *r = v & mask;
            });
    } else {
        pulse_sort_run<PulseKey>(
            R, base, n, k, lds.p, PulseKey{~0ull, ~0u, 0},
            [](uint64_t e, uint64_t r) { return PulseKey{e, uint32_t(r), 0}; },
            [](const PulseKey& v, uint64_t* e, uint64_t* r) {
                *e = v.e;
                *r = v.r;
            });
    }
    if (threadIdx.x == 0) R.len[blockIdx.x] = n < k ? n : k;
}

// Runs 2r and 2r + 1 of `in` (runs_in of them) -> run r of `out`: the first L = min(k, sum) in
// order, kPulseSegs workgroups per pair, workgroup s writing outputs [s * kPulseSeg, (s + 1) *
// kPulseSeg) of L. Its two merge-path diagonals are found by 64-ary searches over the runs in
// global memory (a wave per diagonal, one probe per lane: 3 rounds of loads for 8,192 keys), its
// inputs -- at most kPulseSeg keys of the two runs together -- are staged in LDS, every lane merges
// kPulseSegItems outputs from its own diagonal (binary search in LDS) and the outputs go through
// LDS to coalesced stores. Keys are distinct (rows are). (One 1,024-lane workgroup per pair took
// ~12 us a level once the levels were down to a few pairs: a latency chain over 8,192 outputs.)
constexpr uint32_t kPulseSeg = 1024;
constexpr uint32_t kPulseSegThreads = 256;
constexpr uint32_t kPulseSegItems = kPulseSeg / kPulseSegThreads;
constexpr uint32_t kPulseSegs = kPulseRun / kPulseSeg;

// The number of run a's keys among the first d outputs of merging runs a and b: the smallest i in
// [max(0, d - lb), min(d, la)] with B[d - 1 - i] < A[i] (the predicate rises once along i). One
// wave, 64 probes a round.
template <typename K, typename LoadA, typename LoadB>
__device__ __forceinline__ uint32_t pulse_diagonal(uint32_t d, uint32_t la, uint32_t lb, LoadA load_a, LoadB load_b) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t lo = d > lb ? d - lb : 0, hi = d < la ? d : la;
    while (lo < hi) {
        const uint32_t step = (hi - lo + 63) / 64;
        const uint32_t i = lo + lane * step;
        bool p = true;
        if (i < hi) p = sort_less(load_b(d - 1 - i), load_a(i));
        const uint64_t m = __ballot(p);
        if (m == 0) {
            lo = lo + 63 * step + 1;
        } else {
            const uint32_t f = uint32_t(__builtin_ctzll(m));
            const uint32_t nhi = lo + f * step < hi ? lo + f * step : hi;
            if (f > 0) lo = lo + (f - 1) * step + 1;
            hi = nhi;
        }
    }
    return lo;
}

template <typename K, typename Pack, typename Unpack>
__device__ __forceinline__ void pulse_merge_seg(PulseRuns in, uint32_t a, uint32_t b, uint32_t la, uint32_t lb,
                                uint32_t L, PulseRuns out, uint32_t r, uint32_t d0, K* A, K* B, K* O,
                                uint32_t* cut, K none, Pack pack, Unpack unpack) {
    const uint32_t tid = threadIdx.x, wave = tid >> 6;
    const uint64_t* ae = in.exp + uint64_t(a) * in.stride;
    const uint64_t* ar = in.row + uint64_t(a) * in.stride;
    const uint64_t* be = in.exp + uint64_t(b) * in.stride;
    const uint64_t* br = in.row + uint64_t(b) * in.stride;
    const uint32_t d1 = d0 + kPulseSeg < L ? d0 + kPulseSeg : L;
    if (wave < 2) {
        const uint32_t d = wave ? d1 : d0;
        const uint32_t i = pulse_diagonal<K>(
            d, la, lb, [=](uint32_t x) { return pack(ae[x], ar[x]); },
            [=](uint32_t x) { return pack(be[x], br[x]); });
        if ((tid & 63) == 0) cut[wave] = i;
    }
    __syncthreads();
    const uint32_t i0 = cut[0], i1 = cut[1];
    const uint32_t j0 = d0 - i0, j1 = d1 - i1;
    const uint32_t na = i1 - i0, nb = j1 - j0;
    for (uint32_t x = tid; x < na; x += kPulseSegThreads) A[x] = pack(ae[i0 + x], ar[i0 + x]);
    for (uint32_t x = tid; x < nb; x += kPulseSegThreads) B[x] = pack(be[j0 + x], br[j0 + x]);
    __syncthreads();
    const uint32_t n = d1 - d0, dd = tid * kPulseSegItems;
    if (dd < n) {
        uint32_t lo = dd > nb ? dd - nb : 0, hi = dd < na ? dd : na;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sort_less(B[dd - 1 - mid], A[mid])) hi = mid;
            else lo = mid + 1;
        }
        uint32_t i = lo, j = dd - lo;
        K x = i < na ? A[i] : none, y = j < nb ? B[j] : none;
#pragma unroll
        for (uint32_t m = 0; m < kPulseSegItems; m++) {
            if (dd + m >= n) break;
            const bool take_a = j >= nb || (i < na && sort_less(x, y));
            if (take_a) {
                O[dd + m] = x;
                i++;
                if (i < na) x = A[i];
            } else {
                O[dd + m] = y;
                j++;
                if (j < nb) y = B[j];
            }
        }
    }
    __syncthreads();
    uint64_t* oe = out.exp + uint64_t(r) * out.stride + d0;
    uint64_t* orow = out.row + uint64_t(r) * out.stride + d0;
    for (uint32_t q = tid; q < n; q += kPulseSegThreads) unpack(O[q], &oe[q], &orow[q]);
}

// The runs holding candidates, and the merge levels over them.
__device__ inline uint32_t pulse_live_runs(const unsigned long long* counters) {
    return uint32_t((counters[1] + kPulseSortRun - 1) / kPulseSortRun);
}
__device__ inline uint32_t pulse_levels(uint32_t live) {
    return live <= 1 ? 0u : 32u - __builtin_clz(live - 1);  // ceil(log2(live))
}


__device__ void pulse_settle_one(Tables T, const uint64_t* exp, unsigned long long* counters,
                                 unsigned int* expired_out, uint32_t k);
__device__ inline void pulse_report_one(unsigned long long* counters, unsigned long long* report);


// The merge levels, a launch each (levels past the candidates' own runs return at once), and
// pulse_final_copy, which moves the result where the host reads it after all levels and settles
// the pulse. (One launch for the whole tree, the second child of a pair to finish merging it, took
// 77 us against ~45: every hand-off between workgroups paid an agent-scope release and acquire --
// the L2 written back and invalidated -- where a kernel boundary pays it once.)
__global__ void __launch_bounds__(kPulseSegThreads) pulse_merge(PulseRuns in, uint32_t runs_in,
                                                               uint32_t k, PulseRuns out,
                                                               const unsigned long long* counters,
                                                               uint64_t timestamp, uint32_t row_bits,
                                                               uint32_t level) {
    if (level >= pulse_levels(pulse_live_runs(counters))) return;
    __shared__ union {
        uint64_t u[3][kPulseSeg];
        PulseKey p[3][kPulseSeg];
    } lds;
    __shared__ uint32_t cut[2];
    const uint32_t r = blockIdx.x / kPulseSegs, s = blockIdx.x % kPulseSegs;
    const uint32_t a = 2 * r, b = 2 * r + 1;
    const uint32_t la = a < runs_in ? in.len[a] : 0, lb = b < runs_in ? in.len[b] : 0;
    const uint32_t L = la + lb < k ? la + lb : k;
    if (s == 0 && threadIdx.x == 0) out.len[r] = L;
    const uint32_t d0 = s * kPulseSeg;
    if (d0 >= L) return;
    const PulsePack P = pulse_pack(counters, timestamp, row_bits);
    if (P.packed) {
        const uint64_t mask = (1ull << row_bits) - 1;
        pulse_merge_seg<uint64_t>(
            in, a, b, la, lb, L, out, r, d0, lds.u[0], lds.u[1], lds.u[2], cut, ~0ull,
            [=](uint64_t e, uint64_t rw) { return P.key(e, rw); },
            [=](uint64_t v, uint64_t* e, uint64_t* rw) {
                *e = P.base + (v >> row_bits);
                *rw = v & mask;
            });
    } else {
        pulse_merge_seg<PulseKey>(
            in, a, b, la, lb, L, out, r, d0, lds.p[0], lds.p[1], lds.p[2], cut, PulseKey{~0ull, ~0u, 0},
            [](uint64_t e, uint64_t rw) { return PulseKey{e, uint32_t(rw), 0}; },
            [](const PulseKey& v, uint64_t* e, uint64_t* rw) {
                *e = v.e;
                *rw = v.r;
            });
    }
}

// After `levels` merge launches the host reads the result from the first buffers when `levels` is
// even, else from the second: when the levels that ran leave it in the other one, run 0 moves.
// Then the settlement (and, for tbg_pulse, the report).
__global__ void __launch_bounds__(kPulseThreads) pulse_final_copy(PulseRuns first, PulseRuns second,
                                                                 unsigned long long* counters,
                                                                 uint32_t levels, Tables T,
                                                                 unsigned int* expired_out,
                                                                 uint32_t k, uint32_t settle,
                                                                 unsigned long long* report) {
    const uint32_t ran = pulse_levels(pulse_live_runs(counters));
    const PulseRuns dst = (levels & 1) ? second : first;
    if ((ran & 1) != (levels & 1)) {
        const PulseRuns src = (ran & 1) ? second : first;
        const uint32_t n = src.len[0];
        for (uint32_t i = threadIdx.x; i < n; i += kPulseThreads) {
            dst.exp[i] = src.exp[i];
            dst.row[i] = src.row[i];
        }
        if (threadIdx.x == 0) dst.len[0] = n;
        __syncthreads();
    }
    if (settle && threadIdx.x == 0) {
        pulse_settle_one(T, dst.exp, counters, expired_out, k);
        if (report) pulse_report_one(counters, report);
    }
}

// tbg_pulse's last selection launch, in place of pulse_final_copy + pulse_apply: the selection is
// where the merge levels that ran left it (the first buffers after an even number, else the
// second); its first min(candidates, k) rows expire and are copied to `sel` (the expiries'
// AccountEvents read them there), and workgroup 0 settles the pulse (pulse_settle_one's values),
// reports to the host and clears `next_counters`, the set the next pulse takes (tbg_pulse
// alternates two: this pulse's own is still being read here).
__global__ void pulse_apply_root(PulseRuns first, PulseRuns second,
                                 const unsigned long long* counters,
                                 unsigned long long* next_counters, Tables T, uint32_t k,
                                 uint64_t* sel, unsigned int* expired_out,
                                 unsigned long long* report) {
    const uint32_t ran = pulse_levels(pulse_live_runs(counters));
    const PulseRuns src = (ran & 1) ? second : first;
    const uint64_t C = counters[1];
    const uint64_t n = C < k ? C : k;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        uint64_t next = counters[2] == ~0ull ? TB_TIMESTAMP_MAX : counters[2];
        if (C >= k && k > 0) next = src.exp[k - 1];
        T.scalars->pulse_next_timestamp = next;
        T.scalars->expiry_count = counters[0];
        *expired_out = uint32_t(n);
        report[0] = n;
        report[1] = counters[0];
        __threadfence_system();
        pulse_counters_clear(next_counters);
    }
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) {
        const uint64_t row = src.row[i];
        sel[i] = row;
        pulse_apply_one(T, row);
    }
}

// After the selection (the first min(candidates, k) in order at exp / rows): the number expired,
// the index's new length (the entries still pending) and pulse_next_timestamp -- the k-th expiry
// when the scan filled its batch, else the earliest unexpired one (timestamp_max if none).
__device__ void pulse_settle_one(Tables T, const uint64_t* exp, unsigned long long* counters,
                                 unsigned int* expired_out, uint32_t k) {
    const uint64_t C = counters[1];
    const uint64_t expired = C < k ? C : k;
    uint64_t next = counters[2] == ~0ull ? TB_TIMESTAMP_MAX : counters[2];
    if (C >= k && k > 0) next = exp[k - 1];
    T.scalars->pulse_next_timestamp = next;
    T.scalars->expiry_count = counters[0];
    counters[3] = expired;
    *expired_out = uint32_t(expired);
}
// tbg_pulse's end (report != null): the count expired and the index's new length into mapped
// pinned memory for the host, and the counters cleared for the next pulse.
__device__ inline void pulse_report_one(unsigned long long* counters, unsigned long long* report) {
    report[0] = counters[3];
    report[1] = counters[0];
    __threadfence_system();
    pulse_counters_clear(counters);
}
__global__ void pulse_settle(Tables T, const uint64_t* exp, unsigned long long* counters,
                             unsigned int* expired_out, uint32_t k, unsigned long long* report) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    pulse_settle_one(T, exp, counters, expired_out, k);
    if (report) pulse_report_one(counters, report);
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
