// The flow replay: the ordered replay of a create_transfers call executed by many lanes at once,
// with exactly the serial order's outcome.
//
// Units. The replayed events (the replay list, in call order) form units: a linked chain
// (execute_create's scope, state_machine.zig:3033-3043, :3116-3145, :3196-3207) is one unit, every
// other event is a unit of its own. A unit runs start to finish on one lane, which keeps the
// chain's scope (its undo log is the lane's own).
//
// Keys. Everything an event reads or writes that another replayed event can also write is named
// by a key:
//   * id keys: a 32-bit hash of the event's id and, for post/void, of its pending_id. They cover
//     the id slot and its in-call holder's result (groove.get visibility, replay.hpp header), the
//     transfer row behind it, and the pending transfer's TransferPending status. (A collision
//     only adds an ordering the serial order already has.) A call without duplicate ids or
//     post/void takes none: each id's slot and row are then its own event's alone.
//   * account keys: the row of every account the event may read or write -- its debit and credit
//     accounts, or the pending transfer's for post/void, resolved before the replay: the committed
//     pending row's, or the in-call creator's event's. When that creator is not certain (the
//     pending id has several in-call claimants, or is not found at planning in a call with
//     duplicate ids) the unit becomes a barrier.
//     Additive accounts (no replayed event reads their balances or changes their `closed` flag,
//     Replay::additive) get no key: their deltas are u128 atomics, which commute.
// Account existence, ledgers and every FAST delta are fixed before the replay, so
// these keys are the whole in-call state a replayed event depends on, apart from three scalars
// handled in Replay (replay.hpp: key_range, pulse_next_timestamp, the expires_at list).
//
// Order. A unit may execute an event once, for each key of the event, the previous unit holding
// that key (in call order) has finished -- its "predecessor", from the grouping of the (key, unit)
// pairs by key (group.hpp). Waiting on the immediate predecessor is enough: it waited on its own. Units are taken in
// call order, and each waits only on earlier units, so the earliest unfinished unit can always
// run: the replay always progresses and every lane reaches the exit. A barrier unit runs alone:
// every earlier unit has finished and no later unit starts until it has.
//
// The engine's lanes may sit on many CUs: a unit's writes are released (agent scope) before its
// successors learn that it finished, and acquired by the lane that runs a successor.
#pragma once

#include "kernels.hpp"
#include "prims.hpp"

namespace tbg {

constexpr uint32_t kFlowThreads = 512;      // threads of a lanes workgroup (kLanesMax)
// flow_replay's workgroup bound: 4 waves (the default shape) leave a lane 512 VGPRs; at 512
// threads the replay's registers spilled to scratch
constexpr uint32_t kFlowReplayThreads = 256;
constexpr uint32_t kFlowLanesMax = 8192;    // lanes running units, over all engine workgroups
constexpr uint32_t kFlowLanesPerWave = 1;   // default engine shape (TBG_FLOW_LPW / _WAVES / _BLOCKS)
constexpr uint32_t kFlowWaves = 4;
constexpr uint32_t kFlowBlocks = 256;
constexpr uint32_t kFlowDoneShards = 16;    // units_done counter shards (one line each)
constexpr uint32_t kFlowEngineWords = 64 + 32 * kFlowDoneShards;
constexpr uint32_t kFlowChainMax = 256;     // longer chains run as barriers (global undo log)
constexpr uint32_t kFlowUndoPerLane = 3 * kFlowChainMax;  // 2 accounts + 1 status per event
constexpr uint32_t kFlowKeys = 4;           // keys per event
constexpr uint64_t kFlowNoKey = ~0ull;
constexpr uint32_t kFlowUnitBits = 31;
constexpr uint64_t kFlowSpinLimit = 1ull << 18;  // idle polls / 8 while no unit finishes anywhere

struct FlowPlan {
    uint32_t m;                  // replayed events (the replay list's length)
    uint32_t epoch;              // the call's epoch: `done` and `dup_mark` values of this call
    const uint32_t* slow_list;
    uint8_t* head8;              // per position: starts a unit
    uint32_t* heads;             // per unit: its first position
    unsigned int* counts;        // [0] units, [1] barriers, [2] initially ready units
    uint32_t* unit_of;           // per position
    uint8_t* barrier8;           // per unit (positions >= units hold 0)
    uint32_t* barriers;          // barrier units, in order
    uint32_t* dup_mark;          // per event of the call: an in-call holder with later claimants
    uint32_t* succ;              // kFlowKeys per position: successor unit or kNone32
    uint32_t* indeg;             // per unit: predecessors not yet finished
    const uint32_t* indeg0;      // per unit: its predecessors (edges) at the start (SelectReady)
    uint32_t* queue;             // ready units (unit + 1; 0 = not yet pushed)
    uint64_t* pnt_ops;           // post/void calls: Call::pnt_call (per event), else null
    UndoEntry* lane_undo;        // kFlowUndoPerLane per lane
    struct Step* steps;          // per position: what the engine prefetches before it waits
    tb_transfer_t* evs;          // per position: its event (a copy, addressed by position)
    const unsigned int* skip;    // nonzero: the account lanes replayed the call (lanes.hpp)
    uint32_t* exp_flag;          // per position: may append to the expires_at index
    unsigned long long* exp_base;  // expiry_count at the plan's start (flow_heads)
    unsigned int* lane_counts;   // the account lanes' counters (zeroed by flow_heads)
    uint32_t add_epoch;          // nonzero: additive accounts get no key (Replay::additive)
    unsigned int* engine;        // [0] q_head, [32] q_tail, [64 + 32 j] units_done shard j
                                 // (kFlowDoneShards; one 128-byte line each)
    uint32_t lanes_per_wave;     // lanes of each engine wave that run units
    uint32_t xcd_stride;         // only workgroups blockIdx % xcd_stride == 0 run
    uint32_t backoff;            // idle waves sleep longer the longer they find no unit
    unsigned long long* debug;   // optional: [0] loop iterations, [1] events, [2] cycles executing,
                                 // [3] cycles of the engine (lane 0)
    // Doomed debits (group.hpp: flow_credit_pot): null, or per account row the call's credit
    // potential (epoch:32 | sum:32, sum all-ones: unbounded) and a word set to the epoch when the
    // call cannot bound it (a post/void whose pending transfer is uncertain).
    unsigned long long* acc_pot;
    uint32_t* doom_off;
};

// Per position, everything the replay reads that no other unit writes, so the engine loads it
// while the position's keys are still held by earlier units.
struct Step {
    uint64_t ts_event;
    uint32_t batch, flags;  // StepInfo
    uint32_t k, slot, dr, cr;  // the event and its EvRefs
    uint32_t pslot, add;       // EvRefs::pslot, EvRefs::add
};

__device__ inline uint64_t flow_key(uint32_t type, uint32_t index, uint32_t unit) {
    return (uint64_t(type) << 63) | (uint64_t(index) << kFlowUnitBits) | unit;
}

// (The low word: hash_id's high bits are shared by the 16 ids of a home group.)
__device__ inline uint32_t flow_id_key(const tb_uint128_t& id) { return uint32_t(hash_id(id)); }

// Unit heads and duplicate holders.
__global__ void flow_heads(Tables T, Call<tb_transfer_t> c, FlowPlan P) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    // Per-call counters, zeroed here (grid >= kFlowEngineWords): the engine's q_head, q_tail and
    // done shards, the lanes' counters, the grouping's listed segments, pulse_next_timestamp's flag.
    if (s < kFlowEngineWords) P.engine[s] = 0;
    if (s < 4) P.lane_counts[s] = 0;
    if (s == 0) {
        P.counts[5] = P.counts[6] = P.counts[7] = P.counts[8] = 0;
    }
    if (s >= P.m) return;
    const uint32_t k = P.slow_list[s];
    bool head = true;
    if (s > 0 && P.slow_list[s - 1] == k - 1 && (c.events[k - 1].flags & TB_TRANSFER_LINKED)) {
        // k continues k - 1's chain unless k opens a new batch (a chain cannot cross one).
        const uint32_t b = batch_of_guess(c.batch_ends, c.n_batches, c.n, k);
        head = batch_start_of(c, b) == k;
    }
    P.head8[s] = head;
    P.barrier8[s] = 0;  // (units < m: plan_keys sets the barriers)
    P.queue[s] = 0;  // (the ready units are selected into it after the grouping)
    if (s == 0) *P.exp_base = T.scalars->expiry_count;
    const uint32_t slot = c.ev_slot[k];
    if (slot != kNone32) {
        const uint64_t w = T.tr.slots[slot];
        if (w != kEmpty && w != kTomb) {
            const uint64_t r = (w & kRefMask) - 1;
            if (r >= c.row_base && r - c.row_base < k) P.dup_mark[r - c.row_base] = P.epoch;
        }
    }
}

// Unit heads selected in order (heads[u] = the unit's first position) and every position's unit
// (the inclusive count of heads up to it, minus one): one chained scan over head8.
struct SelectHeads {
    static constexpr bool kEmitAll = true;
    const uint8_t* head8;
    uint32_t* heads;
    uint32_t* unit_of;
    unsigned int* count;
    __device__ void load(uint64_t base, uint64_t n, uint32_t* c) const {
        SelectFlags8{head8, nullptr, nullptr}.load(base, n, c);
    }
    __device__ void emit(uint64_t s, uint32_t p) const {
        const bool head = head8[s] != 0;
        if (head) heads[p] = uint32_t(s);
        unit_of[s] = p + (head ? 1u : 0u) - 1u;
    }
    __device__ void total(uint32_t t) const { *count = t; }
};

// The engine: lanes spread over `blocks` workgroups (see the header). A unit is ready once every
// predecessor has finished (indeg 0). Ready units wait in a queue; a lane pops one, runs it, and
// releases its successors -- the first that becomes ready it runs itself next (so a chain of units
// on one hot key stays on one lane, its rows warm in that CU's L1), the others it pushes. Each
// unit's last predecessor makes it ready exactly once, so every unit runs exactly once; the
// earliest unfinished unit's predecessors have all finished, so it is ready or running: the
// replay progresses, and lanes leave when the queue is drained and every unit has finished.
// With a barrier unit in the call, lane 0 replays every unit in order (serial semantics).
//
// Lanes. Only `lanes_per_wave` lanes of each wave run units: the replay of one event is a long
// branchy walk of dependent memory round trips, and lanes of one wave in different branches take
// turns, so a unit's latency grows with the busy lanes of its wave. With `xcd_stride` 8 only every
// 8th workgroup runs (workgroups are dealt round-robin over the 8 XCDs): the engine shares one L2.
// Measured on config 4: one lane per wave over the whole chip halved the replay's time against one
// workgroup of 512 busy lanes (116 -> 56 ms per 300k events, every account keyed); packing onto one
// XCD lost. With additive accounts unkeyed the replay has far more independent units, and more
// lanes won while an event cost ~5 us (8192 lanes, 8 per wave: 7.0 ms per 1M events; 512: 19.9).
// With an event at ~2.8 us (no scratch, one round trip for the row loads and one for the additive
// atomics) the critical path dominates and sharing a wave costs more than lanes gain: 1024 lanes,
// one per wave, is the default (executor.hip, profiles/r02_shapes).
//
// Hand-offs between lanes on different CUs follow the agent-scope model (MI355X_MICROARCH.md,
// inter-workgroup visibility): a finishing unit runs one release fence (L2 write-back) before its
// relaxed decrements of its successors' indeg; a lane that takes a unit -- from its own decrement
// or from a relaxed poll of the queue -- runs one acquire fence (L1 invalidate) before it reads
// anything another unit wrote. The queue counters live in global memory (P.engine).
// (kDbg: TBG_FLOW_DEBUG's counters; the production instance holds none of them)
template <bool kDbg>
__global__ void __launch_bounds__(kFlowReplayThreads) flow_replay(Tables T, Call<tb_transfer_t> c,
                                                           FlowPlan P) {
    if (P.skip && *P.skip) return;
    if (blockIdx.x % P.xcd_stride) return;
    const uint32_t block = blockIdx.x / P.xcd_stride;
    const uint32_t tid = threadIdx.x;
    const uint32_t wave_lane = tid & 63;
    const uint32_t lane = (block * (blockDim.x >> 6) + (tid >> 6)) * P.lanes_per_wave + wave_lane;
    const uint32_t units = P.counts[0];
    unsigned int* q_head = P.engine;
    unsigned int* q_tail = P.engine + 32;
    const uint64_t t_start = kDbg ? wall_clock64() : 0;
    uint64_t it_count = 0, ev_count = 0, exec_cycles = 0, conts = 0;
    bool chain_open = false, chain_broken = false;
    uint32_t chain_start = 0;

    if (P.counts[1] != 0) {  // barrier units: the serial replay, on one lane
        if (block == 0 && tid == 0) {
            Replay R(T);
            R.expiry_planned = true;
            R.pnt_ops = P.pnt_ops;
            for (uint32_t s = 0; s < P.m; s++) {
                replay_chain_step<tb_transfer_t>(R, c, P.slow_list[s], true, chain_open,
                                                 chain_start, chain_broken);
                if (R.overflow) {
                    atomicOr(&T.scalars->flags, kFlagUndoOverflow);
                    break;
                }
            }
            T.scalars->stats[2] = P.m;
        }
        return;
    }

    Replay R(T);
    R.concurrent = true;
    R.pnt_ops = P.pnt_ops;
    R.undo = P.lane_undo + uint64_t(lane) * kFlowUndoPerLane;
    R.undo_cap = kFlowUndoPerLane;
    R.add_epoch = P.add_epoch;
    R.expiry_planned = true;
    uint64_t lane_key_max = 0;
    unsigned int* done_shard = P.engine + 64 + 32 * (lane % kFlowDoneShards);

    // Runs unit u; releases its successors; returns the one this lane runs next (or kNone32).
    auto run_unit = [&](uint32_t u) -> uint32_t {
        const uint32_t begin = P.heads[u];
        const uint32_t end = u + 1 < units ? P.heads[u + 1] : P.m;
        R.undo_len = 0;
        R.key_max = 0;
        const uint64_t t0 = kDbg ? wall_clock64() : 0;
        // Step records and events are addressed by position and never written during the
        // replay: a chain's next pair loads while the current event runs.
        Step st = P.steps[begin];
        tb_transfer_t ev = P.evs[begin];
        for (uint32_t s = begin; s < end; s++) {
            const bool more = s + 1 < end;
            Step st_next;
            tb_transfer_t ev_next;
            if (more) {
                st_next = P.steps[s + 1];
                ev_next = P.evs[s + 1];
            }
            StepInfo si;
            si.ts_event = st.ts_event;
            si.batch = st.batch;
            si.flags = st.flags;
            replay_chain_step_at<tb_transfer_t>(R, c, st.k, ev, si,
                                                EvRefs{st.slot, st.dr, st.cr, st.pslot, st.add},
                                                true, chain_open, chain_start, chain_broken);
            if (R.overflow) {
                atomicOr(&T.scalars->flags, kFlagUndoOverflow);
                R.overflow = false;
            }
            if (more) {
                st = st_next;
                ev = ev_next;
            }
        }
        R.flush_adds();  // (the unit's last carries, before its release)
        if (kDbg) {
            exec_cycles += wall_clock64() - t0;
            ev_count += end - begin;
        }
        // (transfers key_max: read only by imported events, which never take the flow replay;
        // each lane folds its maximum in at the exit.)
        if (R.key_max > lane_key_max) lane_key_max = R.key_max;
        // Release: this unit's writes reach the point of coherence before any decrement. A unit
        // without successors skips it (the L2 write-back is the costliest step of a short unit,
        // and nothing in this kernel reads what it wrote; the kernel's end releases it).
        bool any_succ = false, several = false;
        uint32_t only = kNone32, edges = 0;
        for (uint32_t s = begin; s < end; s++) {
            const uint4 sc = *reinterpret_cast<const uint4*>(P.succ + kFlowKeys * uint64_t(s));
            any_succ |= (sc.x & sc.y & sc.z & sc.w) != kNone32;
            const uint32_t vs[kFlowKeys] = {sc.x, sc.y, sc.z, sc.w};
#pragma unroll
            for (uint32_t q = 0; q < kFlowKeys; q++) {
                if (vs[q] == kNone32) continue;
                if (only == kNone32) only = vs[q];
                if (vs[q] == only) edges++;
                else several = true;
            }
        }
        // A private hand-off: every edge into the one successor v comes from this unit (its
        // in-degree at the start is this unit's edges to it), so no other lane waits on v or on
        // this unit's writes before v has run. This lane runs v next with no release, decrement or
        // acquire: v reads this unit's writes through the lane's own CU and XCD L2, and v's own
        // release (or the kernel's end) publishes both units' writes to their later readers, all
        // of which follow v. (v's in-degree word is reset for the next call's plan.)
        if (any_succ && !several && P.indeg0[only] == edges) {
            P.indeg[only] = 0;
            __hip_atomic_fetch_add(done_shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            conts++;
            return only;
        }
        uint32_t next = kNone32;
        bool pushed = false;
        if (any_succ) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        for (uint32_t s = begin; any_succ && s < end; s++) {
            const uint4 sc = *reinterpret_cast<const uint4*>(P.succ + kFlowKeys * uint64_t(s));
            const uint32_t vs[kFlowKeys] = {sc.x, sc.y, sc.z, sc.w};
#pragma unroll
            for (uint32_t q = 0; q < kFlowKeys; q++) {
                const uint32_t v = vs[q];
                if (v == kNone32) continue;
                const uint32_t old = __hip_atomic_fetch_add(&P.indeg[v], 0xFFFFFFFFu,
                                                            __ATOMIC_RELAXED,
                                                            __HIP_MEMORY_SCOPE_AGENT);
                if (old != 1) continue;
                if (next == kNone32) {
                    // Acquire what every other predecessor of v released.
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    next = v;
                } else {
                    if (!pushed) {
                        // Pass the acquired writes on to the lanes that pop the pushed units.
                        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                        pushed = true;
                    }
                    const uint32_t slot = atomicAdd(q_tail, 1u);
                    __hip_atomic_store(&P.queue[slot], v + 1, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        __hip_atomic_fetch_add(done_shard, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        conts += next != kNone32;
        return next;
    };
    uint32_t u = kNone32;
    uint64_t spins = 0;
    uint32_t last_seen = 0, polls = 0, idle = 0;
    bool alive = wave_lane < P.lanes_per_wave;
    uint32_t pos = alive ? atomicAdd(q_head, 1u) : 0;
    // The loop's exit is wave-uniform (a vote): inside it every lane only takes if/else paths, so
    // a waiting lane and a running lane of the same wave share every iteration. (With per-lane
    // exits the compiler may form an inner loop of the waiting lanes that the running lanes of the
    // wave only re-enter once every waiter has left it -- a waiter that needs a unit of its own
    // wave would never leave.)
    while (__any(alive)) {
        if (alive && u == kNone32) {
            // Pop: the queue entry at `pos`, or leave once every unit has finished.
            if (pos >= units) {
                alive = false;
            } else {
                const uint32_t w = __hip_atomic_load(&P.queue[pos], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT);
                it_count++;
                if (w != 0) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    u = w - 1;
                    pos = atomicAdd(q_head, 1u);
                    spins = 0;
                    idle = 0;
                } else if ((++idle, ++polls & 7) == 0) {  // the shards' sum, every 8th idle poll
                    uint32_t seen = 0;
                    for (uint32_t j = 0; j < kFlowDoneShards; j++)
                        seen += __hip_atomic_load(P.engine + 64 + 32 * j, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_AGENT);
                    if (seen != last_seen) {
                        last_seen = seen;
                        spins = 0;
                    }
                    if (seen == units) {
                        alive = false;
                    } else if (++spins > kFlowSpinLimit) {
                        // Watchdog: a replay that stops progressing is a bug; leave with a flag
                        // (the call fails) instead of holding the GPU.
                        atomicOr(&T.scalars->flags, kFlagFlowStalled);
                        if (kDbg) {
                            P.debug[8] = *q_head;
                            P.debug[9] = *q_tail;
                            P.debug[10] = seen;
                            P.debug[11] = pos;
                        }
                        alive = false;
                    }
                }
            }
        }
        // A wave sleeps only when none of its lanes has a unit to run (s_sleep stalls the whole
        // wave); the longer its lanes have been idle, the longer it sleeps, so that idle waves'
        // polls do not crowd the memory system the running lanes' replays wait on.
        const bool wave_runs = __any(alive && u != kNone32);
        if (alive && u != kNone32) {
            u = run_unit(u);
        } else if (alive && !wave_runs) {
            if (!P.backoff || idle < 16) __builtin_amdgcn_s_sleep(1);
            else if (idle < 128) __builtin_amdgcn_s_sleep(4);
            else __builtin_amdgcn_s_sleep(16);
        }
    }
    if (lane_key_max)
        atomicMax(&T.scalars->transfers_key_max, (unsigned long long)lane_key_max);
    if (kDbg) {
        atomicAdd(&P.debug[0], (unsigned long long)it_count);
        atomicAdd(&P.debug[1], (unsigned long long)ev_count);
        atomicAdd(&P.debug[2], (unsigned long long)exec_cycles);
        atomicAdd(&P.debug[4], (unsigned long long)conts);
    }
    __syncthreads();
    if (block == 0 && tid == 0) {
        T.scalars->stats[2] = P.m;
        if (kDbg) P.debug[3] = wall_clock64() - t_start;
    }
}

}  // namespace tbg
