// One-launch order-preserving scans and selections (a chained scan with decoupled look-back).
//
// The executor's plans are chains of small passes over a call's events (a few thousand to a few
// million items); each library scan or selection costs 2-3 launches and a temp-storage query, and
// the launches, not the bytes, are what such a pass spends. `chained_scan` is one launch:
//
//   * a workgroup of 256 lanes takes a tile of 4096 consecutive items, 16 per lane (a lane's items
//     are contiguous: a u8 flag tile is one 16-byte load per lane), and reduces the tile's counts;
//   * tiles are numbered by a ticket taken at the workgroup's start (not blockIdx), so every tile a
//     workgroup waits on has already started and waits only on tiles before it: the look-back
//     always progresses, whatever the dispatch order;
//   * each tile publishes its aggregate, then its inclusive prefix, in one 8-byte status word per
//     tile (launch sequence:30 | flag:2 | value:32), written and read with agent-scope atomics on
//     both sides (MI355X_MICROARCH.md, inter-workgroup visibility: the word is its own payload). A
//     word of an earlier launch carries another sequence number and reads as "not ready", so the
//     status array is never cleared;
//   * the first wave looks back 64 tiles at a time: the nearest tile with an inclusive prefix ends
//     the walk, the aggregates of the tiles before it are summed on the way;
//   * the op then emits every item with its exclusive prefix, and the last tile reports the total.
//
// An op supplies: `count(i)` (items i >= n are never asked), `emit(i, prefix)` for every item
// i < n with a nonzero count (scans: every item), and `total(t)` (called once, by the last tile).
#pragma once

#include "device_common.hpp"

namespace tbg {

constexpr uint32_t kScanThreads = 256;
constexpr uint32_t kScanItems = 16;
constexpr uint32_t kScanTile = kScanThreads * kScanItems;
constexpr uint64_t kScanFlagAggregate = 1, kScanFlagInclusive = 2;

struct ScanState {
    unsigned long long* status;  // per tile
    unsigned int* ticket;        // monotone tile ticket counter
    uint32_t ticket_base;        // the ticket of this launch's first tile
    uint32_t seq;                // this launch's sequence number (1 .. 2^30 - 1)
    // The launch does nothing when *skip == skip_if (a queued launch whose work another kernel
    // took over; every launch sharing its status words and ticket must skip alike).
    const unsigned int* skip = nullptr;
    uint32_t skip_if = 0;
};

__device__ inline unsigned long long scan_word(uint32_t seq, uint64_t flag, uint32_t v) {
    return (uint64_t(seq) << 34) | (flag << 32) | v;
}

__device__ inline uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// Inclusive scan across the 64 lanes of a wave.
__device__ inline uint32_t wave_inclusive_u32(uint32_t v, uint32_t lane) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(v, d, 64);
        if (lane >= uint32_t(d)) v += o;
    }
    return v;
}

// One tile of a chained scan: `status` the scan's tile words, `tile` its tile (by ticket).
template <typename Op>
__device__ inline void scan_tile(uint64_t n, const Op& op, unsigned long long* status, uint32_t seq,
                                 uint32_t tile) {
    __shared__ uint32_t s_prefix;
    __shared__ uint32_t s_wave[kScanThreads / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    ScanState st{status, nullptr, 0, seq};
    const uint64_t base = uint64_t(tile) * kScanTile + uint64_t(tid) * kScanItems;
    uint32_t c[kScanItems];
    op.load(base, n, c);
    uint32_t mine = 0;
#pragma unroll
    for (uint32_t i = 0; i < kScanItems; i++) mine += c[i];
    const uint32_t incl = wave_inclusive_u32(mine, lane);
    if (lane == 63) s_wave[wave] = incl;
    __syncthreads();
    uint32_t wave_before = 0, agg = 0;
#pragma unroll
    for (uint32_t w = 0; w < kScanThreads / 64; w++) {
        const uint32_t t = s_wave[w];
        if (w < wave) wave_before += t;
        agg += t;
    }
    if (wave == 0) {
        uint32_t excl = 0;
        if (tile == 0) {
            if (lane == 0)
                __hip_atomic_store(&st.status[0], scan_word(st.seq, kScanFlagInclusive, agg),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            if (lane == 0)
                __hip_atomic_store(&st.status[tile], scan_word(st.seq, kScanFlagAggregate, agg),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            int64_t j = int64_t(tile) - 1;
            while (true) {
                const int64_t idx = j - int64_t(lane);
                uint64_t flag = kScanFlagInclusive;
                uint32_t val = 0;
                if (idx >= 0) {
                    const unsigned long long w = __hip_atomic_load(
                        &st.status[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    flag = (uint32_t(w >> 34) == st.seq) ? ((w >> 32) & 3) : 0;
                    val = uint32_t(w);
                }
                const uint64_t incl_mask = __ballot(flag == kScanFlagInclusive);
                const uint64_t not_ready = __ballot(flag == 0);
                const uint32_t k = incl_mask ? uint32_t(__builtin_ctzll(incl_mask)) : 63u;
                const uint64_t need = k == 63 ? ~0ull : ((2ull << k) - 1);
                if (not_ready & need) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                excl += wave_sum_u32(lane <= k ? val : 0u);
                if (incl_mask) break;
                j -= 64;
            }
            if (lane == 0)
                __hip_atomic_store(&st.status[tile],
                                   scan_word(st.seq, kScanFlagInclusive, excl + agg),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (lane == 0) s_prefix = excl;
    }
    __syncthreads();
    uint32_t p = s_prefix + wave_before + incl - mine;
#pragma unroll
    for (uint32_t i = 0; i < kScanItems; i++) {
        if (base + i < n && (c[i] || Op::kEmitAll)) op.emit(base + i, p);
        p += c[i];
    }
    const uint64_t tiles = n ? (n + kScanTile - 1) / kScanTile : 1;
    if (tid == 0 && tile == tiles - 1) op.total(s_prefix + agg);
}

template <typename Op>
__global__ void __launch_bounds__(kScanThreads) chained_scan(uint64_t n, Op op, ScanState st) {
    __shared__ uint32_t s_tile;
    if (st.skip && *st.skip == st.skip_if) return;
    if (threadIdx.x == 0) s_tile = atomicAdd(st.ticket, 1u) - st.ticket_base;
    __syncthreads();
    scan_tile(n, op, st.status, st.seq, s_tile);
}

// Two independent scans in one launch: tickets [0, tiles1) are the first scan's tiles, the rest
// the second's (its tile words follow the first's). A tile waits only on earlier tiles of its own
// scan, which hold earlier tickets: the look-back progresses as in chained_scan.
template <typename Op1, typename Op2>
__global__ void __launch_bounds__(kScanThreads) chained_scan2(uint64_t n1, Op1 op1, uint64_t n2,
                                                              Op2 op2, uint32_t tiles1,
                                                              ScanState st) {
    __shared__ uint32_t s_tile;
    if (threadIdx.x == 0) s_tile = atomicAdd(st.ticket, 1u) - st.ticket_base;
    __syncthreads();
    const uint32_t t = s_tile;
    if (t < tiles1) scan_tile(n1, op1, st.status, st.seq, t);
    else scan_tile(n2, op2, st.status + tiles1, st.seq, t - tiles1);
}

// ---- workgroup sort in registers -----------------------------------------------------------------
//
// A bitonic network over THREADS * N keys, N per lane, lane-major (lane t holds elements
// t N .. t N + N - 1): strides below N are compare-exchanges between a lane's own registers, strides
// below 64 N between lanes of a wave (one shuffle per key), and only the longer strides go through
// LDS (`lds`: THREADS * N keys), a barrier each. Ascending; on return every lane holds its N sorted
// elements. Every lane of the workgroup must call it (it has barriers). A key type supplies
// sort_less(a, b) and sort_shfl_xor(k, mask).
__device__ inline bool sort_less(uint32_t a, uint32_t b) { return a < b; }
__device__ inline uint32_t sort_shfl_xor(uint32_t k, int mask) { return __shfl_xor(k, mask, 64); }
__device__ inline bool sort_less(uint64_t a, uint64_t b) { return a < b; }
__device__ inline uint64_t sort_shfl_xor(uint64_t k, int mask) { return __shfl_xor(k, mask, 64); }

template <uint32_t N, uint32_t THREADS, typename K>
__device__ void block_bitonic_sort(K (&k)[N], K* lds) {
    static_assert((N & (N - 1)) == 0 && (THREADS & (THREADS - 1)) == 0 && THREADS >= 64);
    constexpr uint32_t kWave = 64 * N, kTotal = N * THREADS;
    const uint32_t tid = threadIdx.x;
    for (uint32_t size = 2; size <= kTotal; size <<= 1) {
        uint32_t stride = size >> 1;
        if (stride >= kWave) {
#pragma unroll
            for (uint32_t m = 0; m < N; m++) lds[tid * N + m] = k[m];
            __syncthreads();
            for (; stride >= kWave; stride >>= 1) {
                for (uint32_t p = tid; p < kTotal / 2; p += THREADS) {
                    const uint32_t lo = 2 * p - (p & (stride - 1)), hi = lo + stride;
                    const bool ascending = (lo & size) == 0;
                    const K a = lds[lo], b = lds[hi];
                    if (sort_less(b, a) == ascending) {
                        lds[lo] = b;
                        lds[hi] = a;
                    }
                }
                __syncthreads();
            }
#pragma unroll
            for (uint32_t m = 0; m < N; m++) k[m] = lds[tid * N + m];
            __syncthreads();  // (the next LDS stage rewrites the array)
        }
        for (; stride >= N; stride >>= 1) {
#pragma unroll
            for (uint32_t m = 0; m < N; m++) {
                const K o = sort_shfl_xor(k[m], int(stride / N));
                const uint32_t i = tid * N + m;
                const bool keep_min = ((i & stride) == 0) == ((i & size) == 0);
                const bool o_less = sort_less(o, k[m]);
                if (keep_min == o_less) k[m] = o;
            }
        }
        // (strides below N: unrolled over constant strides, so the keys stay in registers)
#pragma unroll
        for (uint32_t st = N / 2; st > 0; st >>= 1) {
            if (st > stride) continue;
#pragma unroll
            for (uint32_t m = 0; m < N; m++) {
                if (m & st) continue;
                const uint32_t p = m | st;
                const bool ascending = ((tid * N + m) & size) == 0;
                if (sort_less(k[p], k[m]) == ascending) {
                    const K x = k[m];
                    k[m] = k[p];
                    k[p] = x;
                }
            }
        }
    }
}

// The same contract by merging: every lane sorts its N keys in registers (a bitonic network, no
// communication), then log2(THREADS) rounds merge pairs of sorted runs through LDS -- each lane
// finds where its N outputs start by a merge-path binary search and merges them into registers,
// one barrier before and after the write-back. Keys must be distinct.
template <uint32_t N, typename K>
__device__ inline void lane_sort(K (&k)[N]) {
#pragma unroll
    for (uint32_t size = 2; size <= N; size <<= 1)
#pragma unroll
        for (uint32_t st = size >> 1; st > 0; st >>= 1)
#pragma unroll
            for (uint32_t m = 0; m < N; m++) {
                if (m & st) continue;
                const uint32_t p = m | st;
                const bool ascending = (m & size) == 0;
                if (sort_less(k[p], k[m]) == ascending) {
                    const K x = k[m];
                    k[m] = k[p];
                    k[p] = x;
                }
            }
}

template <uint32_t N, uint32_t THREADS, typename K>
__device__ void block_merge_sort(K (&k)[N], K* lds) {
    constexpr uint32_t kTotal = N * THREADS;
    const uint32_t tid = threadIdx.x;
    lane_sort<N>(k);
#pragma unroll
    for (uint32_t m = 0; m < N; m++) lds[tid * N + m] = k[m];
    __syncthreads();
    for (uint32_t L = N; L < kTotal; L <<= 1) {
        const uint32_t o0 = tid * N, base = o0 & ~(2 * L - 1), d = o0 - base;
        const K* A = lds + base;
        const K* B = lds + base + L;
        uint32_t lo = d > L ? d - L : 0, hi = d < L ? d : L;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (sort_less(B[d - 1 - mid], A[mid])) hi = mid;
            else lo = mid + 1;
        }
        uint32_t i = lo, j = d - lo;
        K a = A[i < L ? i : L - 1], b = B[j < L ? j : L - 1];
#pragma unroll
        for (uint32_t m = 0; m < N; m++) {
            const bool take_a = j >= L || (i < L && sort_less(a, b));
            k[m] = take_a ? a : b;
            if (take_a) {
                i++;
                if (i < L) a = A[i];
            } else {
                j++;
                if (j < L) b = B[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t m = 0; m < N; m++) lds[o0 + m] = k[m];
        __syncthreads();
    }
}

// Ops.

// u8 flags -> the indices of the nonzero ones, in order; the count to *count.
struct SelectFlags8 {
    static constexpr bool kEmitAll = false;
    const uint8_t* flags;
    uint32_t* out;
    unsigned int* count;
    __device__ void load(uint64_t base, uint64_t n, uint32_t* c) const {
        if (base + kScanItems <= n) {
            const uint4 v = *reinterpret_cast<const uint4*>(flags + base);
            const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (uint32_t i = 0; i < kScanItems; i++) c[i] = ((w[i >> 2] >> (8 * (i & 3))) & 0xFF) != 0;
        } else {
#pragma unroll
            for (uint32_t i = 0; i < kScanItems; i++) c[i] = base + i < n && flags[base + i] != 0;
        }
    }
    __device__ void emit(uint64_t i, uint32_t p) const { out[p] = uint32_t(i); }
    __device__ void total(uint32_t t) const { *count = t; }
};

// u32 counts -> their exclusive prefix sums; the total to *total_out (optional).
struct ExclusiveSumU32 {
    static constexpr bool kEmitAll = true;
    const uint32_t* in;
    uint32_t* out;
    unsigned int* total_out;
    __device__ void load(uint64_t base, uint64_t n, uint32_t* c) const {
        if (base + kScanItems <= n) {
            const uint4* q = reinterpret_cast<const uint4*>(in + base);
#pragma unroll
            for (uint32_t i = 0; i < kScanItems / 4; i++) {
                const uint4 v = q[i];
                c[4 * i] = v.x;
                c[4 * i + 1] = v.y;
                c[4 * i + 2] = v.z;
                c[4 * i + 3] = v.w;
            }
        } else {
#pragma unroll
            for (uint32_t i = 0; i < kScanItems; i++) c[i] = base + i < n ? in[base + i] : 0u;
        }
    }
    __device__ void emit(uint64_t i, uint32_t p) const { out[i] = p; }
    __device__ void total(uint32_t t) const {
        if (total_out) *total_out = t;
    }
};

}  // namespace tbg
