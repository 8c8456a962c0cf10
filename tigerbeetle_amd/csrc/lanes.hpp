// Account lanes: the ordered replay of calls whose only order dependence is balance limits
// (BASELINE.json config 3: hot accounts with debits_must_not_exceed_credits), one lane per limited
// account, its balances in registers.
//
// A replayed event is a *limit event* when its outcome can only be created / exceeds_credits /
// exceeds_debits: a single (unlinked) transfer, not post/void, pending, balancing, closing or
// imported, timeout 0, the holder of a fresh id, both accounts found and open, amount < 2^64 and
// every balance of both accounts < 2^126 (no overflow for any interleaving of the call) -- and the
// call has no duplicate ids, post/void, closable accounts or imported events. Such an event passed
// every check of create_transfer (state_machine.zig:3719-3905) up to the limits; what remains is
//   exceeds_credits  dr has debits_must_not_exceed_credits and dpe + dpo + amount > cpo
//   exceeds_debits   cr has credits_must_not_exceed_debits and cpe + cpo + amount > dpo
// (:3907-3913, in that order), else created with dpo(dr) += amount, cpo(cr) += amount.
//
// The accounts with a limit flag ("owners") each get a lane that walks the account's events in
// call order (the flow plan's (key, unit) sort already lists them) with the account's balances in
// registers. An owner *decides* an event when its own limit is the one checked (debit side with
// debits_must_not_exceed_credits, credit side with credits_must_not_exceed_debits); it publishes
// its verdict in the event's mailbox. An event's outcome is known once every deciding owner has
// published; every owner of the event then applies it, and the writer (the debit owner, else the
// credit owner) writes the result and adds the amount to a non-owner side with an atomic (such an
// account's balance is never read in the call; lanes_finish). The earliest undecided event's owners have decided
// all their earlier events, so they can all publish: the lanes always progress.
//
// When a call is not all limit events, or has more owners than lanes, the flow replay runs.
#pragma once

#include <utility>

#include "flow.hpp"

namespace tbg {

constexpr uint32_t kLanesMax = kFlowThreads;

// What an owner lane reads per step (16 bytes; the rest of the event is the post pass's).
struct LaneRec {
    uint64_t amount;
    uint32_t dr, bits;
};
enum : uint32_t {
    kLaneDrOwner = 1, kLaneCrOwner = 2,  // the account has a limit flag
    kLaneDrDecides = 4,                  // dr has debits_must_not_exceed_credits
    kLaneCrDecides = 8,                  // cr has credits_must_not_exceed_debits
    kLaneDrFree = 16, kLaneCrFree = 32,  // the side's owner is free (lanes_free_sums adds it)
};
// mailbox bits per event
enum : uint32_t { kMbDrSet = 1, kMbDrOk = 2, kMbCrSet = 4, kMbCrOk = 8 };
enum : uint8_t { kOutCreated = 0, kOutExceedsCredits = 1, kOutExceedsDebits = 2 };
// LaneRec.bits above kLaneMbShift: the event's LDS mailbox index (events with two owners)
constexpr uint32_t kLaneMbShift = 8;
constexpr uint32_t kLaneMbWords = 16384;              // 64 KB of LDS, 8 events per word
constexpr uint32_t kLaneMbMax = kLaneMbWords * 8;

struct LanePlan {
    uint32_t m;
    const uint64_t* keys_sorted;  // the flow plan's grouped (key, unit) pairs (group.hpp)
    const unsigned int* n_pairs;  // grouped pairs (device)
    const Step* steps;
    const uint32_t* slow_list;
    LaneRec* recs;            // per position
    uint32_t* mailbox;        // per position: 1 when both sides are owned (then its LDS index)
    uint32_t* mb_index;       // exclusive prefix sum of `mailbox` (one-lane mode); the walk's
                              // verdict words (zeroed by plan_keys)
    uint8_t* outcome;         // per position: the writer lane's verdict (kOut*)
    uint32_t* owner_starts;   // per owner: its segment's first grouped pair (any order)
    unsigned int* counts;     // [0] owners, [1] ineligible events, [2] handled (set by the engine)
    uint32_t epoch;
    uint32_t* acc_free;       // per account row: epoch of the call in which it is a free owner
    uint32_t walk_seq;        // lanes_walk: every window event by event (TBG_WALK_SEQ)
};

// The rings' loads are inline asm, so the compiler inserts no wait for them: its wait analysis
// cannot see that a lane consumes slot q only after the other kAhead - 1 slots (the dispatch on
// `phase`), and would wait for (nearly) every outstanding load at each step. The step waits
// instead with vmcnt(kWaitNewer): when slot q is consumed, at least kWaitNewer vector-memory ops
// were issued after its record load and after the pair load that follows it -- steady state 3 per
// other step (outcome store, record load, pair load) = 21 and 22; the first round at least 14
// (the initial fill issues a record and a pair load per slot after one vmcnt(0)). vmcnt counts
// loads and stores in issue order on CDNA. The asm outputs are consumed only after that wait.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kWaitNewer = 14;
__device__ inline u32x4 lane_load16(const void* p) {
    u32x4 r;
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
}
__device__ inline uint64_t lane_load8(const void* p) {
    uint64_t r;
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(r) : "v"(p) : "memory");
    return r;
}

__device__ inline bool lanes_owner(uint16_t flags) {
    return (flags & (TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS |
                     TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS)) != 0;
}

__device__ inline bool lanes_low(const tb_account_t& a) {
    constexpr uint64_t kLim = 1ull << 62;
    return a.debits_pending.hi < kLim && a.debits_posted.hi < kLim && a.credits_pending.hi < kLim &&
           a.credits_posted.hi < kLim;
}

// The LDS mailbox index of each event with two owners (too many: the flow replay runs).
__global__ void lanes_mailboxes(LanePlan L) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= L.m || !L.mailbox[s]) return;
    const uint32_t i = L.mb_index[s];
    if (i >= kLaneMbMax) atomicAdd(&L.counts[1], 1u);
    else L.recs[s].bits |= i << kLaneMbShift;
}

// Free owners. An owner whose limit passes even if every event it checks in the call is created
// and nothing replenishes it -- debits_must_not_exceed_credits: dpe + dpo + (sum of its checked
// debit amounts) <= cpo; credits_must_not_exceed_debits: cpe + cpo + (sum of its checked credit
// amounts) <= dpo, all at the call's start -- passes every check in any order (in a limit-events
// call balances only grow by created amounts, and the checked side's sum bounds them). Its side of
// each event is then as good as unowned: no lane walks it (lanes_free clears its owner bits; the
// post pass adds its amounts with atomics), and an event left without owners is created. Config 3
// (hot accounts funded for most of the stream) needs no lane at all until an account nears its
// limit. The sums are taken per owner segment by the grouping (group.hpp: group_owner_verdict).
__global__ void lanes_free(Tables T, LanePlan L) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= L.m || L.counts[1] != 0) return;
    LaneRec r = L.recs[s];
    const uint32_t cr = L.steps[s].cr;
    uint32_t bits = r.bits;
    if ((bits & kLaneDrOwner) && L.acc_free[r.dr] == L.epoch)
        bits = (bits & ~uint32_t(kLaneDrOwner | kLaneDrDecides)) | kLaneDrFree;
    if ((bits & kLaneCrOwner) && L.acc_free[cr] == L.epoch)
        bits = (bits & ~uint32_t(kLaneCrOwner | kLaneCrDecides)) | kLaneCrFree;
    if (bits == r.bits) return;
    L.recs[s].bits = bits;
    if (!(bits & (kLaneDrOwner | kLaneCrOwner))) L.outcome[s] = kOutCreated;
}

__global__ void __launch_bounds__(kLanesMax) lanes_replay(Tables T, Call<tb_transfer_t> c,
                                                          LanePlan L) {
    __shared__ uint32_t mbox[kLaneMbWords];
    // Steps finished by any lane of the workgroup: the watchdog counts a lane's idle polls only
    // while no lane progresses (a lane waiting on a verdict that sits late in a hot owner's walk
    // may poll for as long as that walk takes).
    __shared__ unsigned int progress;
    const uint32_t owners = L.counts[0];
    if (L.counts[1] != 0 || owners == 0 || owners > kLanesMax) return;  // the flow replay runs
    const uint32_t o = threadIdx.x;
    if (o == 0) {
        L.counts[2] = 1;
        progress = 0;
    }
    for (uint32_t i = o; i < kLaneMbWords; i += blockDim.x) mbox[i] = 0;
    __syncthreads();
    bool alive = o < owners;
    const uint64_t n_pairs = *L.n_pairs;
    uint64_t idx = alive ? L.owner_starts[o] : 0;
    const uint64_t my_key = alive ? (L.keys_sorted[idx] >> kFlowUnitBits) : 0;
    const uint32_t row = uint32_t(my_key & 0xFFFFFFFFu);
    const bool walks = alive && L.acc_free[row] != L.epoch;  // (free owners: lanes_free)
    alive = walks;
    u128 dpe = 0, dpo = 0, cpe = 0, cpo = 0;
    if (alive) {
        const tb_account_t& a = T.acc_rows[row];
        dpe = U(a.debits_pending);
        dpo = U(a.debits_posted);
        cpe = U(a.credits_pending);
        cpo = U(a.credits_posted);
    }
    bool published = false;
    // The account's records in call order: record loads kAhead steps ahead, and the pair loads
    // that name them kAhead further (a step is register arithmetic; neither load chain may be its
    // latency).
    constexpr uint32_t kAhead = 8;
    static_assert(kWaitNewer == 2 * (kAhead - 1), "the rings' wait count (lane_load16)");
    u32x4 ring[kAhead];  // raw LaneRecs (lane_load16)
    bool ring_ok[kAhead];
    uint32_t ring_s[kAhead];
    uint64_t pre_key[kAhead];  // the (key, unit) pairs of the following kAhead steps, raw
    uint64_t fetch_idx = idx;
    // Every load and store of the steady-state step is unconditional (a clamped index, a dummy
    // slot) and no loaded value is used before kAhead steps later: the wait counters then keep
    // the rings in flight instead of draining them every step.
    bool pre_valid[kAhead];
    auto fetch_pair = [&](uint32_t slot) {  // (an unconditional load: no select waits for it)
        const uint64_t at = fetch_idx < n_pairs ? fetch_idx : n_pairs - 1;
        pre_valid[slot] = fetch_idx < n_pairs;
        pre_key[slot] = lane_load8(&L.keys_sorted[at]);
        fetch_idx++;
    };
    auto take_pair = [&](uint32_t slot) {  // pre_key[slot] -> ring[slot]'s record load
        const uint64_t key = pre_key[slot];
        const uint32_t ps = uint32_t(key & ((1u << kFlowUnitBits) - 1));
        return std::pair<bool, uint32_t>(pre_valid[slot] && (key >> kFlowUnitBits) == my_key,
                                         ps < L.m ? ps : 0u);
    };
#pragma unroll
    for (uint32_t q = 0; q < kAhead; q++) fetch_pair(q);
#pragma unroll
    for (uint32_t q = 0; q < kAhead; q++) asm volatile("s_waitcnt vmcnt(0)" : "+v"(pre_key[q]) :: "memory");
#pragma unroll
    for (uint32_t q = 0; q < kAhead; q++) {
        const auto t = take_pair(q);
        ring_ok[q] = t.first;
        ring_s[q] = t.second;
        ring[q] = lane_load16(&L.recs[ring_s[q]]);
        fetch_pair(q);
    }
    alive = alive && ring_ok[0];
    uint64_t spins = 0;
    unsigned int seen_progress = 0;
    // The ring is consumed in place: slot q holds the record of every step t with t % kAhead == q,
    // and the loop body is unrolled over the slots (constant indices keep the rings in registers).
    // Moving ring entries instead would wait for every outstanding load at each step.
    uint32_t phase = 0;  // the slot of this lane's current step
    while (__any(alive)) {
        if (alive && ++spins > kFlowSpinLimit) {
            const unsigned int p = __hip_atomic_load(&progress, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_WORKGROUP);
            if (p != seen_progress) {
                seen_progress = p;
                spins = 0;
            } else {  // watchdog (a bug): no lane progressed for kFlowSpinLimit polls
                atomicOr(&T.scalars->flags, kFlagFlowStalled);
                alive = false;
            }
        }
#pragma unroll
        for (uint32_t q = 0; q < kAhead; q++) {
            if (alive && phase == q) {
                // Slot q's record and the pair after it are the oldest of at least kWaitNewer
                // newer vector-memory ops (see lane_load16).
                // (The registers are operands: no use of them is scheduled above the wait.)
                asm volatile("s_waitcnt vmcnt(%2)"
                             : "+v"(ring[q]), "+v"(pre_key[q])
                             : "n"(kWaitNewer)
                             : "memory");
                LaneRec rec;
                rec.amount = uint64_t(ring[q].x) | (uint64_t(ring[q].y) << 32);
                rec.dr = ring[q].z;
                rec.bits = ring[q].w;
                const uint32_t s = ring_s[q];
                const bool debit = rec.dr == row;
                const bool decides_dr = (rec.bits & kLaneDrDecides) != 0;
                const bool decides_cr = (rec.bits & kLaneCrDecides) != 0;
                const bool mine = debit ? decides_dr : decides_cr;   // this lane's limit is checked
                const bool other = debit ? decides_cr : decides_dr;  // the other owner's is
                const bool other_owner = (rec.bits & (debit ? kLaneCrOwner : kLaneDrOwner)) != 0;
                const u128 amount = rec.amount;
                bool my_ok = true;
                if (mine) my_ok = debit ? !(dpe + dpo + amount > cpo) : !(cpe + cpo + amount > dpo);
                // Verdicts between two owners go through LDS (4 bits per event whose two sides are
                // owned): a memory round trip here would stall the lane on every such event.
                const uint32_t mbi = rec.bits >> kLaneMbShift;
                const uint32_t mb_shift = (mbi & 7) * 4;
                if (mine && other_owner && !published) {
                    // The other owner applies this event too: it needs the verdict.
                    atomicOr(&mbox[mbi >> 3], (debit ? (kMbDrSet | (my_ok ? kMbDrOk : 0u))
                                                     : (kMbCrSet | (my_ok ? kMbCrOk : 0u)))
                                                  << mb_shift);
                }
                published = true;
                const uint32_t mb = other ? (__hip_atomic_load(&mbox[mbi >> 3], __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_WORKGROUP) >>
                                             mb_shift) & 15u
                                          : 0u;
                const bool known = !other || (mb & (debit ? kMbCrSet : kMbDrSet));
                if (known) {
                    const bool other_ok = !other || (mb & (debit ? kMbCrOk : kMbDrOk));
                    const bool dr_fail = debit ? !my_ok : !other_ok;
                    const bool cr_fail = debit ? !other_ok : !my_ok;
                    const bool created = !dr_fail && !cr_fail;
                    if (created) {
                        if (debit) dpo += amount;
                        else cpo += amount;
                    }
                    const bool writer = debit || !(rec.bits & kLaneDrOwner);
                    // (non-writers store to their own dummy byte past the positions)
                    L.outcome[writer ? s : L.m + o] =
                        created ? kOutCreated : (dr_fail ? kOutExceedsCredits : kOutExceedsDebits);
                    published = false;
                    spins = 0;
                    atomicAdd(&progress, 1u);
                    // Refill the slot with the step kAhead later (its pair was loaded kAhead steps
                    // ago) and load the pair of the step 2 * kAhead later.
                    const auto t = take_pair(q);
                    ring_ok[q] = t.first;
                    ring_s[q] = t.second;
                    ring[q] = lane_load16(&L.recs[ring_s[q]]);
                    fetch_pair(q);
                    phase = (q + 1) % kAhead;
                    alive = ring_ok[(q + 1) % kAhead];
                }
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the rings' last loads)
    if (walks) {
        tb_account_t& a = T.acc_rows[row];
        a.debits_posted = W(dpo);
        a.credits_posted = W(cpo);
        const uint16_t h = acc_hazard_of(a);
        if (h) acc_hazard_set(T.acc_index, T.acc_entry_of, row, h);
    }
    if (o == 0) T.scalars->stats[2] = L.m;
}

// The account walk on one wave per walked owner (the default; lanes_replay above is the one-lane
// form, TBG_LANES_ONE_LANE). A wave loads 64 of its owner's (key, unit) pairs and their records
// at a time, coalesced and one window ahead, and resolves the window's events in call order in a
// wave-uniform loop: the owner's balances live in scalar registers, each event is a handful of
// scalar instructions on values read out of the window's lanes. Verdicts between two owners go
// through a u32 word per position in global memory (`mbox`, zeroed by the host): the deciding
// owner publishes with an agent-scope atomic OR, the other owner reads it with an agent-scope
// (sc1) load -- from a snapshot taken when the window's records were fetched, or, when the
// verdict was not there yet, by polling (MI355X_MICROARCH.md: agent atomics on the producer side,
// sc1 loads on the consumer side, no payload besides the word itself). Every owner waits only on
// verdicts of earlier events, whose deciding owners have applied all their own earlier events:
// the walks always progress. `progress` counts finished windows chip-wide; a poll that sees no
// window finish anywhere for kFlowSpinLimit polls raises kFlagFlowStalled (a bug: the call fails).
constexpr uint32_t kWalkWaves = 4;  // waves per workgroup (one owner each)

struct WalkWindow {
    uint32_t s;        // position (unit) of this lane's event
    uint32_t amt_lo, amt_hi;
    uint32_t bits;     // kWalk* flags relative to the walking owner
    uint32_t mb;       // mailbox snapshot
    bool valid;
};
enum : uint32_t {
    kWalkDebit = 1,        // the owner is the event's debit account
    kWalkMine = 2,         // the owner's limit is the one checked on its side
    kWalkOther = 4,        // the other side's limit is checked: wait for its verdict
    kWalkOtherOwner = 8,   // the owner decides and the other side is walked: publish the verdict
    kWalkWriter = 16,      // this owner writes the outcome
};

__device__ inline uint64_t walk_u64(uint32_t lo, uint32_t hi) { return (uint64_t(hi) << 32) | lo; }
__device__ inline uint32_t walk_uniform(uint32_t v) {
    return uint32_t(__builtin_amdgcn_readfirstlane(int(v)));
}
__device__ inline uint64_t walk_uniform64(uint64_t v) {
    return walk_u64(walk_uniform(uint32_t(v)), walk_uniform(uint32_t(v >> 32)));
}
__device__ inline u128 walk_uniform128(const tb_uint128_t& x) {
    return (u128(walk_uniform64(x.hi)) << 64) | walk_uniform64(x.lo);
}
// The window sums of lanes_walk in u64 (narrow owners and amounts) or u128 (wide ones).
// Wave sums on DPP (with every lane active): an inclusive scan within each row of 16 lanes (row
// shifts 1, 2, 4, 8), then the row broadcasts 15 and 31 carry the rows' totals up, and lane 63 holds
// the sum -- six dependent VALU steps. (A __shfl_xor butterfly is an LDS permute round trip per
// step: the walk's per-window sums took ~0.4 us each on it.)
template <int kCtrl, int kRowMask>
__device__ inline uint32_t walk_dpp(uint32_t v) {
    return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), kCtrl, kRowMask, 0xF, true));
}
template <int kCtrl, int kRowMask>
__device__ inline void walk_dpp_add(uint64_t& v) {
    const uint32_t lo = walk_dpp<kCtrl, kRowMask>(uint32_t(v));
    const uint32_t hi = walk_dpp<kCtrl, kRowMask>(uint32_t(v >> 32));
    v += walk_u64(lo, hi);
}
// (the inclusive scan: lane i holds the sum over lanes 0..i)
__device__ inline uint64_t walk_dpp_scan64(uint64_t v) {
    walk_dpp_add<0x111, 0xF>(v);  // row_shr:1
    walk_dpp_add<0x112, 0xF>(v);  // row_shr:2
    walk_dpp_add<0x114, 0xF>(v);  // row_shr:4
    walk_dpp_add<0x118, 0xF>(v);  // row_shr:8
    walk_dpp_add<0x142, 0xA>(v);  // row_bcast:15 into rows 1 and 3
    walk_dpp_add<0x143, 0xC>(v);  // row_bcast:31 into rows 2 and 3
    return v;
}
__device__ inline uint64_t walk_lane(uint64_t v, uint32_t j) {
    return walk_u64(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), j)),
                    uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v >> 32)), j)));
}
__device__ inline u128 walk_lane(u128 v, uint32_t j) {
    return (u128(walk_lane(uint64_t(v >> 64), j)) << 64) | walk_lane(uint64_t(v), j);
}
__device__ inline uint64_t walk_dpp_sum64(uint64_t v) { return walk_lane(walk_dpp_scan64(v), 63); }
__device__ inline uint64_t walk_wave_sum(uint64_t v) { return walk_dpp_sum64(v); }
// u128: each 32-bit limb summed in u64 (64 lanes: < 2^38), then recombined with the carries.
__device__ inline u128 walk_wave_sum(u128 v) {
    const uint64_t lo = uint64_t(v), hi = uint64_t(v >> 64);
    const uint64_t s0 = walk_dpp_sum64(lo & 0xFFFFFFFFull), s1 = walk_dpp_sum64(lo >> 32);
    const uint64_t s2 = walk_dpp_sum64(hi & 0xFFFFFFFFull), s3 = walk_dpp_sum64(hi >> 32);
    return u128(s0) + (u128(s1) << 32) + (u128(s2) << 64) + (u128(s3) << 96);
}
// Exclusive wave scans (lane i: the sum over lanes 0..i-1), u64 or u128 as above.
__device__ inline uint64_t walk_wave_scan_excl(uint64_t v) { return walk_dpp_scan64(v) - v; }
__device__ inline u128 walk_wave_scan_excl(u128 v) {
    const uint64_t lo = uint64_t(v), hi = uint64_t(v >> 64);
    const uint64_t s0 = walk_dpp_scan64(lo & 0xFFFFFFFFull), s1 = walk_dpp_scan64(lo >> 32);
    const uint64_t s2 = walk_dpp_scan64(hi & 0xFFFFFFFFull), s3 = walk_dpp_scan64(hi >> 32);
    return u128(s0) + (u128(s1) << 32) + (u128(s2) << 64) + (u128(s3) << 96) - v;
}

// (kDbg: TBG_FLOW_DEBUG's counters and timers; the production instance holds none of them:
// thirteen 64-bit counters live across the walk were ~26 SGPRs of a kernel that spills SGPRs)
template <bool kDbg>
__global__ void __launch_bounds__(kWalkWaves * 64) lanes_walk(Tables T, Call<tb_transfer_t> c,
                                                               LanePlan L, uint32_t* mbox,
                                                               unsigned long long* dbg) {
    // dbg (TBG_FLOW_DEBUG): [0] windows, [1] events, [2] live polls, [3] poll cycles,
    // [4] max walk cycles, [5] verdicts found in snapshots, [6] walks (100 MHz wall clock)
    const uint64_t t_walk0 = kDbg ? wall_clock64() : 0;
    uint64_t n_win = 0, n_ev = 0, n_poll = 0, t_poll = 0, n_snap = 0, n_iter = 0, n_alla = 0;
    uint64_t n_refresh = 0, t_refresh = 0, t_fetch = 0, t_b = 0, t_tail = 0, t_a = 0;
    const uint32_t owners = L.counts[0];
    const bool run = L.counts[1] == 0 && owners != 0 && owners <= kLanesMax;
    if (blockIdx.x == 0 && threadIdx.x == 0 && run) {
        L.counts[2] = 1;
        T.scalars->stats[2] = L.m;
    }
    if (!run) return;
    const uint32_t lane = threadIdx.x & 63;
    // Everything about the owner is wave-uniform: scalar registers and scalar branches.
    const uint32_t o = walk_uniform(blockIdx.x * kWalkWaves + (threadIdx.x >> 6));
    if (o >= owners) return;
    const uint64_t start = walk_uniform64(L.owner_starts[o]);
    const uint64_t n_pairs = walk_uniform(*L.n_pairs);
    const uint64_t my_key = walk_uniform64(L.keys_sorted[start]) >> kFlowUnitBits;
    const uint32_t row = uint32_t(my_key & 0xFFFFFFFFu);
    if (walk_uniform(L.acc_free[row]) == L.epoch) return;  // a free owner (lanes_free)
    unsigned int* progress = &L.counts[3];

    const tb_account_t& acc0 = T.acc_rows[row];
    const uint32_t oflags = walk_uniform(acc0.flags);
    const bool owner_dm = (oflags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) != 0;
    const bool owner_cm = (oflags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) != 0;
    const bool one_limit = owner_dm != owner_cm && !L.walk_seq;
    const u128 dpe = walk_uniform128(acc0.debits_pending);
    const u128 cpe = walk_uniform128(acc0.credits_pending);
    u128 dpo = walk_uniform128(acc0.debits_posted);
    u128 cpo = walk_uniform128(acc0.credits_posted);

    auto fetch_pairs = [&](uint64_t base, uint64_t* key) {
        const uint64_t p = base + lane;
        *key = p < n_pairs ? L.keys_sorted[p] : ~0ull;
    };
    // A window as loaded: nothing computed from the loads here, so that no load waits for another
    // (the snapshot word is loaded for every valid event, needed or not).
    struct WalkRaw {
        uint32_t s;
        LaneRec r;
        uint32_t mb;
        bool valid;
    };
    auto fetch_recs = [&](uint64_t key, WalkRaw* w) {
        w->valid = key != ~0ull && (key >> kFlowUnitBits) == my_key;
        const uint32_t s = uint32_t(key & ((1u << kFlowUnitBits) - 1));
        w->s = w->valid && s < L.m ? s : 0u;
        w->r = L.recs[w->s];
        w->mb = w->valid ? __hip_atomic_load(&mbox[w->s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                         : 0u;
    };
    auto decode = [&](const WalkRaw& x, WalkWindow* w) {
        w->valid = x.valid;
        w->s = x.s;
        const LaneRec r = x.r;
        const bool debit = r.dr == row;
        const bool dec_dr = (r.bits & kLaneDrDecides) != 0, dec_cr = (r.bits & kLaneCrDecides) != 0;
        const bool mine = debit ? dec_dr : dec_cr;
        const bool other = debit ? dec_cr : dec_dr;
        const bool other_owner = (r.bits & (debit ? kLaneCrOwner : kLaneDrOwner)) != 0;
        const bool writer = debit || !(r.bits & kLaneDrOwner);
        w->bits = (debit ? kWalkDebit : 0u) | (mine ? kWalkMine : 0u) | (other ? kWalkOther : 0u) |
                  (other_owner && mine ? kWalkOtherOwner : 0u) | (writer ? kWalkWriter : 0u);
        w->amt_lo = uint32_t(r.amount);
        w->amt_hi = uint32_t(r.amount >> 32);
        w->mb = other && w->valid ? x.mb : 0u;
    };

    // Super windows of four windows (256 events): the records (and snapshot) of super window W + 1
    // are issued as W starts, their pairs one super window earlier -- one memory round trip per
    // four windows, overlapped with W's work. (Loads whose address is a loaded value wait for
    // everything issued before them: a deeper ring of single windows waits as often.)
    uint64_t base = start;
    WalkRaw b0, b1, b2, b3;
    uint64_t k0, k1, k2, k3;  // the pairs of the next super window
    {
        uint64_t p0, p1, p2, p3;
        fetch_pairs(base, &p0);
        fetch_pairs(base + 64, &p1);
        fetch_pairs(base + 128, &p2);
        fetch_pairs(base + 192, &p3);
        fetch_recs(p0, &b0);
        fetch_recs(p1, &b1);
        fetch_recs(p2, &b2);
        fetch_recs(p3, &b3);
        fetch_pairs(base + 256, &k0);
        fetch_pairs(base + 320, &k1);
        fetch_pairs(base + 384, &k2);
        fetch_pairs(base + 448, &k3);
    }
    uint64_t spins = 0;
    unsigned int seen = 0;
    bool stalled = false;
    bool done = false;
    while (!done) {
        // This super window's records and the next one's pairs arrived during the previous super
        // window: one wait for them here, before the next loads issue. (Without it the compiler's
        // wait at the window loop's head -- its pending-load state merged over the loop -- was a
        // vmcnt(0) that also waited for the loads issued just below: the prefetch never overlapped.
        // A builtin, not inline asm, so that the compiler's wait pass sees it.)
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (gfx9 encoding; expcnt, lgkmcnt not waited)
        const bool more_super = (__ballot(b3.valid) >> 63) & 1;
        WalkRaw n0, n1, n2, n3;
        n0.valid = n1.valid = n2.valid = n3.valid = false;
        uint64_t q0 = ~0ull, q1 = ~0ull, q2 = ~0ull, q3 = ~0ull;
        if (more_super) {
            fetch_recs(k0, &n0);
            fetch_recs(k1, &n1);
            fetch_recs(k2, &n2);
            fetch_recs(k3, &n3);
            fetch_pairs(base + 512, &q0);
            fetch_pairs(base + 576, &q1);
            fetch_pairs(base + 640, &q2);
            fetch_pairs(base + 704, &q3);
        }
      for (uint32_t sub = 0; sub < 4; sub++) {
        const uint64_t tf0 = kDbg ? wall_clock64() : 0;
        // (field by field: a select of whole structs goes through scratch)
        WalkRaw x;
        x.s = sub == 0 ? b0.s : sub == 1 ? b1.s : sub == 2 ? b2.s : b3.s;
        x.r.amount = sub == 0 ? b0.r.amount : sub == 1 ? b1.r.amount : sub == 2 ? b2.r.amount : b3.r.amount;
        x.r.dr = sub == 0 ? b0.r.dr : sub == 1 ? b1.r.dr : sub == 2 ? b2.r.dr : b3.r.dr;
        x.r.bits = sub == 0 ? b0.r.bits : sub == 1 ? b1.r.bits : sub == 2 ? b2.r.bits : b3.r.bits;
        x.mb = sub == 0 ? b0.mb : sub == 1 ? b1.mb : sub == 2 ? b2.mb : b3.mb;
        x.valid = sub == 0 ? b0.valid : sub == 1 ? b1.valid : sub == 2 ? b2.valid : b3.valid;
        WalkWindow cur;
        decode(x, &cur);
        // The window as scalar masks (one bit per event, in call order).
        const uint64_t vmask = __ballot(cur.valid);
        if (vmask == 0) {
            done = true;
            break;
        }
        const uint64_t debit_m = __ballot(cur.valid && (cur.bits & kWalkDebit));
        const uint64_t mine_m = __ballot(cur.valid && (cur.bits & kWalkMine));
        const uint64_t other_m = __ballot(cur.valid && (cur.bits & kWalkOther));
        const uint64_t pub_m = __ballot(cur.valid && (cur.bits & kWalkOtherOwner));
        const bool my_debit = (cur.bits & kWalkDebit) != 0;
        const uint64_t snap_set =
            __ballot((cur.mb & (my_debit ? kMbCrSet : kMbDrSet)) != 0);
        const uint64_t snap_ok = __ballot((cur.mb & (my_debit ? kMbCrOk : kMbDrOk)) != 0);
        if (kDbg) t_fetch += wall_clock64() - tf0;
        const bool more = (vmask >> 63) & 1;  // the segment continues past this window
        const uint32_t cnt = uint32_t(__popcll(vmask));
        uint64_t created_m = 0, drfail_m = 0, myok_m = 0, published = 0;
        // Verdicts this owner owes are published with one vector atomic per flush: before any
        // poll (an owner it waits on may wait on them) and at the window's end.
        uint64_t decided = 0;  // events this owner has decided (mine) so far in the window
        auto publish = [&]() {
            const uint64_t due = pub_m & decided & ~published;
            if (due == 0) return;
            if ((due >> lane) & 1) {
                const bool ok = (myok_m >> lane) & 1;
                const uint32_t v = my_debit ? (kMbDrSet | (ok ? kMbDrOk : 0u))
                                            : (kMbCrSet | (ok ? kMbCrOk : 0u));
                atomicOr(&mbox[cur.s], v);
            }
            published |= due;
        };
        // The events in call order. When the owner's balances are < 2^62 and the window's amounts
        // < 2^56 (no sum below can wrap 64 bits), the checks run on u64 (Balances64), else on u128;
        // amounts are read with one readlane when the window's fit in 32 bits.
        const bool amt32 = __ballot(cur.valid && cur.amt_hi != 0) == 0;
        const bool narrow = __ballot(cur.valid && cur.amt_hi >= (1u << 24)) == 0 &&
                            (dpe >> 62) == 0 && (dpo >> 62) == 0 && (cpe >> 62) == 0 &&
                            (cpo >> 62) == 0;
        // The other side's verdict of window event j (not in the snapshot): poll its word.
        auto wait_verdict = [&](uint32_t j, bool debit) -> bool {
            const uint64_t tp0 = kDbg ? wall_clock64() : 0;
            n_poll++;
            publish();  // (an owner this one waits on may wait on these)
            const uint32_t sj = __builtin_amdgcn_readlane(cur.s, j);
            const uint32_t need = debit ? kMbCrSet : kMbDrSet;
            uint32_t mb = 0;
            while (!stalled) {
                mb = walk_uniform(__hip_atomic_load(&mbox[sj], __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT));
                if (mb & need) break;
                __builtin_amdgcn_s_sleep(1);
                if ((++spins & 255) == 0) {
                    const unsigned int p = walk_uniform(__hip_atomic_load(
                        progress, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    if (p != seen) {
                        seen = p;
                        spins = 0;
                    } else if (spins > kFlowSpinLimit) {
                        stalled = true;
                    }
                }
            }
            if (kDbg) t_poll += wall_clock64() - tp0;
            return (mb & (debit ? kMbCrOk : kMbDrOk)) != 0;
        };
        auto walk_events = [&](auto dpe_v, auto& dpo_v, auto cpe_v, auto& cpo_v) {
            using V = decltype(dpe_v);
            for (uint32_t j = 0; j < cnt; j++) {
                const uint64_t bit = 1ull << j;
                const uint32_t lo = __builtin_amdgcn_readlane(cur.amt_lo, j);
                const V amt = amt32 ? V(lo) : V(walk_u64(lo, __builtin_amdgcn_readlane(cur.amt_hi, j)));
                const bool debit = (debit_m & bit) != 0;
                bool my_ok = true;
                if (mine_m & bit) {
                    my_ok = debit ? !(dpe_v + dpo_v + amt > cpo_v) : !(cpe_v + cpo_v + amt > dpo_v);
                    decided |= bit;
                    if (my_ok) myok_m |= bit;
                    if (pub_m & bit) {  // an owner may be waiting on this verdict: publish now
                        if (lane == j) {
                            const uint32_t v = debit ? (kMbDrSet | (my_ok ? kMbDrOk : 0u))
                                                     : (kMbCrSet | (my_ok ? kMbCrOk : 0u));
                            atomicOr(&mbox[cur.s], v);
                        }
                        published |= bit;
                    }
                }
                bool other_ok = true;
                if (other_m & bit) {
                    if (snap_set & bit) {
                        other_ok = (snap_ok & bit) != 0;
                        n_snap++;
                    } else {
                        other_ok = wait_verdict(j, debit);
                    }
                }
                const bool dr_fail = debit ? !my_ok : !other_ok;
                const bool cr_fail = debit ? !other_ok : !my_ok;
                if (!dr_fail && !cr_fail) {
                    created_m |= bit;
                    // (value selects: an if / else here becomes a store through a selected
                    // pointer, and the balances then live in scratch -- whose loads wait, in order,
                    // for every memory operation issued before them, the prefetched windows
                    // included)
                    dpo_v += debit ? amt : V(0);
                    cpo_v += debit ? V(0) : amt;
                } else if (dr_fail) {
                    drfail_m |= bit;
                }
            }
        };
        // An owner with one limit flag resolves its window in wave-wide steps, on u64 when its
        // balances and the window's amounts are narrow (no sum below can wrap), else on u128.
        auto one_limit_window = [&](auto zero) {
            using V = decltype(zero);
            // An owner with one limit flag: its checked ("mine") events all test used + amount <=
            // cap -- debits_must_not_exceed_credits: used = dpe + dpo, cap = cpo; credits_must_
            // not_exceed_debits: used = cpe + cpo, cap = dpo -- a created mine event adds to
            // `used`, a created other event to `cap`. The window resolves in wave-wide steps:
            // (A) if used + (every mine amount) <= cap, every mine check passes whatever the
            // other events do; (B) else the window resolves in speculative steps (below): steps
            // are disagreements + polls, not events.
            V used = owner_dm ? V(dpe) + V(dpo) : V(cpe) + V(cpo);
            V cap = owner_dm ? V(cpo) : V(dpo);
            const V used0 = used, cap0 = cap;
            const V amt = cur.valid ? V(walk_u64(cur.amt_lo, cur.amt_hi)) : V(0);
            const bool l_mine = (mine_m >> lane) & 1, l_other = (other_m >> lane) & 1;
            uint64_t known = snap_set & other_m, known_ok = snap_ok & other_m;
            n_snap += __popcll(known);
            // The words of the window events in `want` read again, all at once (the snapshot is
            // two windows old): one round trip instead of a poll per event.
            auto refresh = [&](uint64_t want) {
                const uint64_t tr0 = kDbg ? wall_clock64() : 0;
                n_refresh++;
                publish();
                const bool w = (want >> lane) & 1;
                const uint32_t mb2 = w ? __hip_atomic_load(&mbox[cur.s], __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT)
                                       : 0u;
                const uint64_t set = __ballot(w && (mb2 & (my_debit ? kMbCrSet : kMbDrSet)));
                const uint64_t ok = __ballot(w && (mb2 & (my_debit ? kMbCrOk : kMbDrOk)));
                known |= set;
                known_ok |= ok & set;
                if (kDbg) t_refresh += wall_clock64() - tr0;
            };
            const V mine_sum = walk_wave_sum(l_mine ? amt : V(0));
            if (used + mine_sum <= cap) {
                n_alla++;
                decided = mine_m;
                myok_m = mine_m;
                publish();
                if (other_m & ~known) refresh(other_m & ~known);
                for (uint64_t u = other_m & ~known; u != 0; u &= u - 1) {
                    const uint32_t j = uint32_t(__builtin_ctzll(u));
                    known |= 1ull << j;
                    if (wait_verdict(j, (debit_m >> j) & 1)) known_ok |= 1ull << j;
                }
                created_m = vmask & (~other_m | known_ok);
                drfail_m = vmask & ~created_m & ~debit_m;  // (credit events: the debit side failed)
                used += walk_wave_sum(((created_m & mine_m) >> lane) & 1 ? amt : V(0));
                cap += walk_wave_sum(((created_m & ~mine_m) >> lane) & 1 ? amt : V(0));
            } else {
                const uint64_t tb0 = kDbg ? wall_clock64() : 0;
                uint64_t rem = vmask;
                // Each step decides every remaining event on the state at the step's start (the
                // single-event rule below), then checks each again against that state plus the
                // amounts of the events so created before it (exclusive wave scans): up to the
                // first event the two disagree on, or that waits on an unknown verdict with its
                // own check passing, the speculation is the serial outcome, and the step applies
                // all of it. Steps are disagreements + polls, not created events (wide amounts:
                // most events pass, a few huge ones fail -- a step per created event was ~11 a
                // window).
                while (rem != 0 && !stalled) {
                    n_iter++;
                    const bool in = (rem >> lane) & 1;
                    const bool kok = ((known_ok >> lane) & 1) != 0;
                    const bool l_debit = ((debit_m >> lane) & 1) != 0;
                    const bool unknown = l_other && !((known >> lane) & 1);
                    const bool ok0 = !l_mine || used + amt <= cap;
                    const bool cr0 = in && ok0 && (!l_other || kok);
                    const V am = cr0 && l_mine ? amt : V(0), ao = cr0 && !l_mine ? amt : V(0);
                    const V pm = walk_wave_scan_excl(am), po = walk_wave_scan_excl(ao);
                    const bool ok1 = !l_mine || used + pm + amt <= cap + po;
                    const bool cr1 = ok1 && (!l_other || kok);
                    const uint64_t stop = __ballot(in && (cr1 != cr0 || (unknown && ok1)));
                    const uint64_t before = stop ? ((stop & (0 - stop)) - 1) & rem : rem;
                    const uint64_t crm = __ballot(in && cr1);
                    const uint64_t okm = __ballot(in && l_mine && ok1);
                    // (not created: as in the single-event rule)
                    const uint64_t drf = __ballot(in && ((l_mine && !ok1 && l_debit) ||
                                                         (l_other && !l_debit && !kok)));
                    created_m |= before & crm;
                    decided |= before & mine_m;
                    myok_m |= before & okm;
                    drfail_m |= before & drf;
                    rem &= ~before;
                    // the state after `before`: the sums up to the stop (or over the window)
                    const uint32_t j = stop ? uint32_t(__builtin_ctzll(stop)) : 63u;
                    used += walk_lane(stop ? pm : pm + am, j);
                    cap += walk_lane(stop ? po : po + ao, j);
                    if (stop == 0) break;
                    const uint64_t bit = 1ull << j;
                    if ((other_m & bit) && !(known & bit) && ((okm >> j) & 1 || !(mine_m & bit))) {
                        // Its own check first (the state is final up to j): the other owner may
                        // be waiting on this very verdict.
                        if (mine_m & bit) {
                            decided |= bit;
                            myok_m |= bit;
                        }
                        refresh(other_m & ~known & rem);
                        if (!(known & bit)) {
                            known |= bit;
                            if (wait_verdict(j, (debit_m & bit) != 0)) known_ok |= bit;
                        }
                        continue;
                    }
                    publish();  // (j disagreed: the next step starts at it, on the new state)
                }
                if (kDbg) t_b += wall_clock64() - tb0;
            }
            const u128 d_used = u128(used - used0), d_cap = u128(cap - cap0);
            dpo += owner_dm ? d_used : d_cap;
            cpo += owner_dm ? d_cap : d_used;
        };
        const uint64_t ta0 = kDbg ? wall_clock64() : 0;
        if (one_limit && narrow) {
            one_limit_window(uint64_t(0));
        } else if (one_limit) {
            one_limit_window(u128(0));
        } else if (narrow) {
            uint64_t dpo64 = uint64_t(dpo), cpo64 = uint64_t(cpo);
            walk_events(uint64_t(dpe), dpo64, uint64_t(cpe), cpo64);
            dpo = dpo64;
            cpo = cpo64;
        } else {
            walk_events(dpe, dpo, cpe, cpo);
        }
        const uint64_t tt0 = kDbg ? wall_clock64() : 0;
        if (kDbg) t_a += tt0 - ta0;
        publish();
        if (stalled) {
            if (lane == 0) atomicOr(&T.scalars->flags, kFlagFlowStalled);
            return;
        }
        if (cur.valid && (cur.bits & kWalkWriter)) {
            const uint8_t out = ((created_m >> lane) & 1) ? kOutCreated
                                : ((drfail_m >> lane) & 1) ? kOutExceedsCredits
                                                           : kOutExceedsDebits;
            L.outcome[cur.s] = out;
        }
        if (lane == 0) atomicAdd(progress, 1u);
        if (kDbg) t_tail += wall_clock64() - tt0;
        n_win++;
        n_ev += cnt;
        if (!more) {
            done = true;
            break;
        }
      }
        if (done) break;
        base += 256;
        b0 = n0;
        b1 = n1;
        b2 = n2;
        b3 = n3;
        k0 = q0;
        k1 = q1;
        k2 = q2;
        k3 = q3;
    }
    if (lane == 0) {
        tb_account_t& acc = T.acc_rows[row];
        acc.debits_posted = W(dpo);
        acc.credits_posted = W(cpo);
        const uint16_t h = acc_hazard_of(acc);
        if (h) acc_hazard_set(T.acc_index, T.acc_entry_of, row, h);
        if (kDbg) {
            atomicAdd(&dbg[0], n_win);
            atomicAdd(&dbg[1], n_ev);
            atomicAdd(&dbg[2], n_poll);
            atomicAdd(&dbg[3], t_poll);
            atomicMax(&dbg[4], wall_clock64() - t_walk0);
            atomicAdd(&dbg[5], n_snap);
            atomicAdd(&dbg[6], 1ull);
            atomicAdd(&dbg[7], n_refresh);
            atomicAdd(&dbg[8], t_refresh);
            atomicAdd(&dbg[9], t_fetch);
            if (o < 1000) {  // per owner: events, polls, poll time, walk time, windows, step
                             // B iterations, all-pass windows
                unsigned long long* w = &dbg[16 + 8 * o];
                w[0] = n_ev;
                w[1] = n_poll;
                w[2] = t_poll;
                w[3] = wall_clock64() - t_walk0;
                w[4] = n_win | (t_fetch << 24);
                w[5] = n_iter | (t_b << 24);
                w[6] = n_alla | (t_tail << 24);
                w[1] = n_poll | (t_a << 24);
                w[7] = (n_refresh << 32) | (t_refresh & 0xFFFFFFFFull);
            }
        }
    }
}

// After the lanes, one lane per event: the result (timestamp, verdict), the sides of created
// events that no lane owns (u128 atomics: their balances are never read in the call), and the
// transfers key_max.
// Adds `amount` to balance field `key` (kNone32: nothing) with u128 atomics: the lanes sharing the
// key of the first pending lane are summed first (`rounds` times; a key that dominates the wave
// takes one atomic), the rest add their own. Every lane of the wave calls it.
__device__ inline void wave_add_field(const BalTarget& B, uint32_t key, uint64_t amount,
                                      int rounds = 64) {
    const uint32_t lane = threadIdx.x & 63;
    for (int r = 0; r < rounds; r++) {
        const uint64_t pend = __ballot(key != kNone32);
        if (pend == 0) break;
        const int leader = __ffsll((unsigned long long)pend) - 1;
        const uint32_t lkey = __shfl(key, leader);
        const bool mine = key == lkey;
        uint64_t lo = mine ? amount : 0, hi = 0;
        for (int off = 32; off > 0; off >>= 1) {
            const uint64_t olo = __shfl_xor(lo, off);
            const uint64_t ohi = __shfl_xor(hi, off);
            const uint64_t nlo = lo + olo;
            hi = hi + ohi + (nlo < lo ? 1u : 0u);
            lo = nlo;
        }
        if (lane == uint32_t(leader)) add_field(B, lkey, (u128(hi) << 64) | lo, true);
        if (mine) key = kNone32;
    }
    if (key != kNone32) add_field(B, key, u128(amount), true);
}

// Free owners' sides (lanes_free): every created event's amount on the owner's posted field, one
// u128 atomic per run of the owner's grouped pairs in a wave (the pairs are grouped by account, so
// a segmented sum over 64 consecutive pairs; config 3's hottest free owner takes ~20k events per
// call on one field -- as per-event atomics, contention).
__global__ void lanes_free_sums(Tables T, LanePlan L, uint64_t pairs) {
    const uint64_t p = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const uint32_t lane = threadIdx.x & 63;
    uint64_t run = ~0ull;  // the account key (tag | row) of the pair; ~0: none
    uint64_t dlo = 0, dhi = 0, clo = 0, chi = 0;
    const bool ok = L.counts[2] && !(T.scalars->flags & kFlagFlowStalled);
    if (ok && p < pairs && p < *L.n_pairs) {
        const uint64_t key = L.keys_sorted[p];
        run = key >> kFlowUnitBits;
        const uint32_t row = uint32_t(run & 0xFFFFFFFFu);
        if ((run >> 32) == 1 && L.acc_free[row] == L.epoch) {
            const uint32_t s = uint32_t(key & ((1u << kFlowUnitBits) - 1));
            if (s < L.m && L.outcome[s] == kOutCreated) {
                const LaneRec r = L.recs[s];
                if (r.dr == row && (r.bits & kLaneDrFree)) dlo = r.amount;
                else if (r.dr != row && (r.bits & kLaneCrFree)) clo = r.amount;
            }
        }
    }
    // Segmented inclusive sums over the wave (runs of equal `run` are contiguous).
    for (int off = 1; off < 64; off <<= 1) {
        const uint64_t orun = __shfl_up(run, off);
        const uint64_t odlo = __shfl_up(dlo, off), odhi = __shfl_up(dhi, off);
        const uint64_t oclo = __shfl_up(clo, off), ochi = __shfl_up(chi, off);
        if (lane >= uint32_t(off) && orun == run) {
            const uint64_t nd = dlo + odlo, nc = clo + oclo;
            dhi += odhi + (nd < dlo ? 1u : 0u);
            chi += ochi + (nc < clo ? 1u : 0u);
            dlo = nd;
            clo = nc;
        }
    }
    const uint64_t next = __shfl_down(run, 1);
    const bool last = lane == 63 || next != run;
    if (last && run != ~0ull) {
        const BalTarget B{T.acc_rows, T.acc_index, T.acc_entry_of};
        const uint32_t row = uint32_t(run & 0xFFFFFFFFu);
        add_field(B, row * 4 + 1, (u128(dhi) << 64) | dlo, true);
        add_field(B, row * 4 + 3, (u128(chi) << 64) | clo, true);
    }
}

__global__ void lanes_finish(Tables T, Call<tb_transfer_t> c, LanePlan L) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t ts_max = 0;
    uint32_t dr_key = kNone32, cr_key = kNone32;
    uint64_t amount = 0;
    // (a stalled walk fails the call: its outcomes are incomplete)
    if (s < L.m && L.counts[2] && !(T.scalars->flags & kFlagFlowStalled)) {
        const Step st = L.steps[s];
        const LaneRec rec = L.recs[s];
        const uint8_t out = L.outcome[s];
        tb_create_result_t res;
        res.timestamp = st.ts_event;
        res.status = out == kOutCreated ? TB_STATUS_CREATED
                                        : (out == kOutExceedsCredits ? TB_CT_EXCEEDS_CREDITS
                                                                     : TB_CT_EXCEEDS_DEBITS);
        res.reserved = 0;
        c.results[st.k] = res;
        if (out == kOutCreated) {
            ts_max = st.ts_event;
            amount = rec.amount;
            if (!(rec.bits & (kLaneDrOwner | kLaneDrFree))) dr_key = st.dr * 4 + 1;
            if (!(rec.bits & (kLaneCrOwner | kLaneCrFree))) cr_key = st.cr * 4 + 3;
        }
    }
    // (sides of free owners: lanes_free_sums; the unowned sides here are mostly distinct)
    const BalTarget B{T.acc_rows, T.acc_index, T.acc_entry_of};
    wave_add_field(B, dr_key, amount, 2);
    wave_add_field(B, cr_key, amount, 2);
    ts_max = block_reduce(ts_max, OpMax());
    if (threadIdx.x == 0 && ts_max)
        atomicMax(&T.scalars->transfers_key_max, (unsigned long long)ts_max);
}

}  // namespace tbg
