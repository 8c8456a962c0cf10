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
//     only adds an ordering the serial order already has.)
//   * account keys: the row of every account the event may read or write -- its debit and credit
//     accounts, or the pending transfer's for post/void, resolved before the replay: the committed
//     pending row's, or the in-call creator's event's. When that creator is not certain (the
//     pending id has several in-call claimants, or is not found at planning in a call with
//     duplicate ids) the unit becomes a barrier.
// Account existence, ledgers and every FAST delta are fixed before the replay, so
// these keys are the whole in-call state a replayed event depends on, apart from three scalars
// handled in Replay (replay.hpp: key_range, pulse_next_timestamp, the expires_at list).
//
// Order. A unit may execute an event once, for each key of the event, the previous unit holding
// that key (in call order) has finished -- its "predecessor", from a radix sort of (key, unit)
// pairs. Waiting on the immediate predecessor is enough: it waited on its own. Units are taken in
// call order, and each waits only on earlier units, so the earliest unfinished unit can always
// run: the replay always progresses and every lane reaches the exit. A barrier unit runs alone:
// every earlier unit has finished and no later unit starts until it has.
//
// The engine is one workgroup: all its lanes share one CU's L1, so workgroup-scope release/acquire
// orders a unit's writes before its successors' reads without cache maintenance.
#pragma once

#include "kernels.hpp"

namespace tbg {

constexpr uint32_t kFlowThreads = 512;      // lanes of the engine workgroup
constexpr uint32_t kFlowChainMax = 256;     // longer chains run as barriers (global undo log)
constexpr uint32_t kFlowUndoPerLane = 3 * kFlowChainMax;  // 2 accounts + 1 status per event
constexpr uint32_t kFlowKeys = 4;           // keys per event
constexpr uint64_t kFlowNoKey = ~0ull;
constexpr uint32_t kFlowUnitBits = 31;

struct FlowPlan {
    uint32_t m;                  // replayed events (the replay list's length)
    uint32_t epoch;              // the call's epoch: `done` and `dup_mark` values of this call
    const uint32_t* slow_list;
    uint8_t* head8;              // per position: starts a unit
    uint32_t* heads;             // per unit: its first position
    unsigned int* counts;        // [0] units, [1] barriers
    uint32_t* unit_of;           // per position
    uint8_t* barrier8;           // per unit (positions >= units hold 0)
    uint32_t* barriers;          // barrier units, in order
    uint32_t* dup_mark;          // per event of the call: an in-call holder with later claimants
    uint64_t* keys;              // kFlowKeys per position: (type:1 | index:32 | unit:31)
    uint32_t* vals;              // kFlowKeys * position + j
    uint64_t* keys_sorted;
    uint32_t* vals_sorted;
    uint32_t* pred;              // kFlowKeys per position: predecessor unit or kNone32
    uint32_t* done;              // per unit: epoch once finished
    uint64_t* pnt_ops;           // per position (post/void calls), else null
    uint64_t* pnt_scan;
    unsigned long long* pnt_fired;
    UndoEntry* lane_undo;        // kFlowUndoPerLane per lane
    struct Step* steps;          // per position: what the engine prefetches before it waits
    unsigned long long* debug;   // optional: [0] loop iterations, [1] events, [2] cycles executing,
                                 // [3] cycles of the engine (lane 0)
};

// Per position, everything the replay reads that no other unit writes, so the engine loads it
// while the position's keys are still held by earlier units.
struct Step {
    uint64_t ts_event;
    uint32_t batch, flags;  // StepInfo
    uint32_t k, slot, dr, cr;  // the event and its EvRefs
};

__device__ inline uint64_t flow_key(uint32_t type, uint32_t index, uint32_t unit) {
    return (uint64_t(type) << 63) | (uint64_t(index) << kFlowUnitBits) | unit;
}

// (The low word: hash_id's high bits are shared by the 16 ids of a home group.)
__device__ inline uint32_t flow_id_key(const tb_uint128_t& id) { return uint32_t(hash_id(id)); }

// Unit heads and duplicate holders.
__global__ void flow_heads(Tables T, Call<tb_transfer_t> c, FlowPlan P) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.m) return;
    const uint32_t k = P.slow_list[s];
    bool head = true;
    if (s > 0 && P.slow_list[s - 1] == k - 1 && (c.events[k - 1].flags & TB_TRANSFER_LINKED)) {
        // k continues k - 1's chain unless k opens a new batch (a chain cannot cross one).
        const uint32_t b = batch_of(c.batch_ends, c.n_batches, k);
        head = batch_start_of(c, b) == k;
    }
    P.head8[s] = head;
    const uint32_t slot = c.ev_slot[k];
    if (slot != kNone32) {
        const uint64_t w = T.tr.slots[slot];
        if (w != kEmpty && w != kTomb) {
            const uint64_t r = (w & kRefMask) - 1;
            if (r >= c.row_base && r - c.row_base < k) P.dup_mark[r - c.row_base] = P.epoch;
        }
    }
}

// Positions of each unit; barrier flags of over-long chains.
__global__ void flow_units(FlowPlan P) {
    const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= P.m) return;
    const uint32_t units = P.counts[0];
    if (u >= units) {
        P.barrier8[u] = 0;
        return;
    }
    const uint32_t begin = P.heads[u];
    const uint32_t end = u + 1 < units ? P.heads[u + 1] : P.m;
    for (uint32_t s = begin; s < end; s++) P.unit_of[s] = u;
    P.barrier8[u] = end - begin > kFlowChainMax;
}

// The keys of each replayed event.
__global__ void flow_keys(Tables T, Call<tb_transfer_t> c, FlowPlan P, unsigned int call_flags) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.m) return;
    const uint32_t k = P.slow_list[s];
    const uint32_t u = P.unit_of[s];
    const tb_transfer_t& t = c.events[k];
    uint64_t key[kFlowKeys] = {kFlowNoKey, kFlowNoKey, kFlowNoKey, kFlowNoKey};
    if (!u128_is_zero(t.id) && !u128_is_max(t.id)) key[0] = flow_key(0, flow_id_key(t.id), u);
    if (t.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) {
        if (!u128_is_zero(t.pending_id) && !u128_is_max(t.pending_id)) {
            key[1] = flow_key(0, flow_id_key(t.pending_id), u);
            // The pending transfer's accounts: the committed row's, or its in-call creator's.
            bool certain = true;
            const tb_transfer_t* p = nullptr;
            const uint64_t ps = transfer_slot_find(T, c, t.pending_id);
            if (ps == kNone) {
                // Not found now; with duplicate ids in the call a later claimant may create it.
                certain = !(call_flags & kFlagDuplicate);
            } else {
                const uint64_t w = T.tr.slots[ps];
                const uint64_t r = (w & kRefMask) - 1;
                if (r < c.row_base) {
                    if (!(w & kOrphanBit)) p = &T.tr_rows[r];
                } else {
                    const uint32_t j = uint32_t(r - c.row_base);
                    if (P.dup_mark[j] == P.epoch) certain = false;
                    else p = &c.events[j];
                }
            }
            if (!certain) {
                P.barrier8[u] = 1;
            } else if (p) {
                const uint64_t dr = account_find(T, p->debit_account_id);
                const uint64_t cr = account_find(T, p->credit_account_id);
                if (dr != kNone) key[2] = flow_key(1, uint32_t(dr), u);
                if (cr != kNone) key[3] = flow_key(1, uint32_t(cr), u);
            }
        }
    } else {
        const uint32_t dr = c.ev_dr[k], cr = c.ev_cr[k];
        if (dr != kNone32) key[2] = flow_key(1, dr, u);
        if (cr != kNone32) key[3] = flow_key(1, cr, u);
    }
    const StepInfo si = step_info(c, k, uint16_t(TB_TRANSFER_IMPORTED));
    const EvRefs x = ev_refs(c, k);
    Step st;
    st.ts_event = si.ts_event;
    st.batch = si.batch;
    st.flags = si.flags;
    st.k = k;
    st.slot = x.slot;
    st.dr = x.dr;
    st.cr = x.cr;
    P.steps[s] = st;
#pragma unroll
    for (uint32_t j = 0; j < kFlowKeys; j++) {
        P.keys[kFlowKeys * uint64_t(s) + j] = key[j];
        P.vals[kFlowKeys * uint64_t(s) + j] = kFlowKeys * s + j;
    }
}

// Predecessor of each (key, unit) pair: the unit of the previous pair with the same key, unless
// it is the same unit (a key repeated within a chain) -- then the first occurrence carries it.
__global__ void flow_preds(FlowPlan P) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint64_t n = kFlowKeys * uint64_t(P.m);
    if (i >= n) return;
    const uint64_t key = P.keys_sorted[i];
    uint32_t pred = kNone32;
    if (key != kFlowNoKey && i > 0) {
        const uint64_t prev = P.keys_sorted[i - 1];
        const uint32_t unit = uint32_t(key & ((1u << kFlowUnitBits) - 1));
        const uint32_t prev_unit = uint32_t(prev & ((1u << kFlowUnitBits) - 1));
        if ((prev >> kFlowUnitBits) == (key >> kFlowUnitBits) && prev_unit != unit) pred = prev_unit;
    }
    P.pred[P.vals_sorted[i]] = pred;
}

__device__ inline uint32_t flow_load(const uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// The engine: one workgroup of kFlowThreads lanes (see the header).
__global__ void __launch_bounds__(kFlowThreads) flow_replay(Tables T, Call<tb_transfer_t> c,
                                                           FlowPlan P) {
    __shared__ unsigned int next_unit, done_count, gate_index;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) {
        next_unit = 0;
        done_count = 0;
        gate_index = 0;
    }
    __syncthreads();
    const uint32_t units = P.counts[0];
    const uint32_t n_barriers = P.counts[1];
    UndoEntry* const my_undo = P.lane_undo + uint64_t(tid) * kFlowUndoPerLane;

    Replay R(T);
    R.concurrent = true;
    R.pnt_ops = P.pnt_ops;
    bool chain_open = false, chain_broken = false;
    uint32_t chain_start = 0;

    const uint64_t t_start = wall_clock64();
    uint64_t it_count = 0, ev_count = 0, exec_cycles = 0, blocked[kFlowKeys] = {}, blocked_dist = 0;
    uint32_t u = atomicAdd(&next_unit, 1u);
    uint32_t s = 0, end = 0, need = 0;
    bool barrier = false;
    Step st;
    tb_transfer_t ev;
    uint4 pr;
    // The position's prefetch: its step record, event and predecessors.
    auto load_position = [&]() {
        st = P.steps[s];
        ev = c.events[st.k];
        pr = *reinterpret_cast<const uint4*>(P.pred + kFlowKeys * uint64_t(s));
        need = (pr.x != kNone32 ? 1u : 0u) | (pr.y != kNone32 ? 2u : 0u) |
               (pr.z != kNone32 ? 4u : 0u) | (pr.w != kNone32 ? 8u : 0u);
    };
    auto begin_unit = [&]() {
        if (u >= units) return;
        s = P.heads[u];
        end = u + 1 < units ? P.heads[u + 1] : P.m;
        barrier = P.barrier8[u] != 0;
        R.undo = barrier ? T.undo : my_undo;
        R.undo_cap = barrier ? T.undo_capacity : kFlowUndoPerLane;
        R.undo_len = 0;
        R.key_max = 0;
        load_position();
    };
    begin_unit();
    while (u < units) {
        // The barrier gate: the earliest unfinished barrier unit, or none.
        const uint32_t gi = __hip_atomic_load(&gate_index, __ATOMIC_ACQUIRE,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t gate = gi < n_barriers ? P.barriers[gi] : 0xFFFFFFFFu;
        bool ready;
        if (u > gate) ready = false;
        else if (u == gate)
            ready = __hip_atomic_load(&done_count, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == u;
        else ready = true;
        if (ready && need) {
            // The predecessors still outstanding, loaded together.
            const uint32_t d0 = (need & 1) ? flow_load(&P.done[pr.x]) : P.epoch;
            const uint32_t d1 = (need & 2) ? flow_load(&P.done[pr.y]) : P.epoch;
            const uint32_t d2 = (need & 4) ? flow_load(&P.done[pr.z]) : P.epoch;
            const uint32_t d3 = (need & 8) ? flow_load(&P.done[pr.w]) : P.epoch;
            need &= (d0 != P.epoch ? 1u : 0u) | (d1 != P.epoch ? 2u : 0u) |
                    (d2 != P.epoch ? 4u : 0u) | (d3 != P.epoch ? 8u : 0u);
            if (need) {
                ready = false;
                if (P.debug) {
                    const uint32_t q = __builtin_ctz(need);
                    blocked[q]++;
                    blocked_dist += u - (q == 0 ? pr.x : q == 1 ? pr.y : q == 2 ? pr.z : pr.w);
                }
            }
        }
        it_count++;
        if (!ready) {
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        R.pos = s;
        const uint64_t t0 = P.debug ? wall_clock64() : 0;
        StepInfo si;
        si.ts_event = st.ts_event;
        si.batch = st.batch;
        si.flags = st.flags;
        replay_chain_step_at<tb_transfer_t>(R, c, st.k, ev, si, EvRefs{st.slot, st.dr, st.cr},
                                            true, chain_open, chain_start, chain_broken);
        if (P.debug) {
            exec_cycles += wall_clock64() - t0;
            ev_count++;
        }
        if (R.overflow) {
            atomicOr(&T.scalars->flags, kFlagUndoOverflow);
            R.overflow = false;
        }
        s++;
        if (s < end) {
            load_position();
            continue;
        }
        // The unit is finished: publish its effects, then its completion.
        if (R.key_max) atomicMax(&T.scalars->transfers_key_max, (unsigned long long)R.key_max);
        __hip_atomic_store(&P.done[u], P.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(&done_count, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (barrier)
            __hip_atomic_fetch_add(&gate_index, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        u = atomicAdd(&next_unit, 1u);
        begin_unit();
    }
    if (P.debug) {
        atomicAdd(&P.debug[0], (unsigned long long)it_count);
        atomicAdd(&P.debug[1], (unsigned long long)ev_count);
        atomicAdd(&P.debug[2], (unsigned long long)exec_cycles);
        for (uint32_t q = 0; q < kFlowKeys; q++)
            atomicAdd(&P.debug[4 + q], (unsigned long long)blocked[q]);
        atomicAdd(&P.debug[8], (unsigned long long)blocked_dist);
    }
    __syncthreads();
    if (tid == 0) {
        T.scalars->stats[2] = P.m;
        if (P.debug) P.debug[3] = wall_clock64() - t_start;
    }
}

// pulse_next_timestamp after a flow replay of a call with post/void: the recorded updates in
// replay order. `min` updates lower it; a reset fires when the value before it (the start value
// and every earlier `min`, while no reset has fired) equals its expiry, after which the value is
// timestamp_min, which no later update changes.
__global__ void flow_pnt_prep(FlowPlan P) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.m) return;
    const uint64_t op = P.pnt_ops[s];
    P.pnt_scan[s] = (op == 0 || (op & kPntReset)) ? ~0ull : op;
}

__global__ void flow_pnt_check(Tables T, FlowPlan P, const uint64_t* prefix_min) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.m) return;
    const uint64_t op = P.pnt_ops[s];
    if (!(op & kPntReset)) return;
    uint64_t before = T.scalars->pulse_next_timestamp;
    if (s > 0 && prefix_min[s - 1] < before) before = prefix_min[s - 1];
    if (before == (op & ~kPntReset)) atomicOr(P.pnt_fired, 1ull);
}

__global__ void flow_pnt_final(Tables T, FlowPlan P, const uint64_t* prefix_min) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t v = T.scalars->pulse_next_timestamp;
    if (*P.pnt_fired) v = TB_TIMESTAMP_MIN;
    else if (P.m && prefix_min[P.m - 1] < v) v = prefix_min[P.m - 1];
    T.scalars->pulse_next_timestamp = v;
}

}  // namespace tbg
