// The flow plan's key grouping: each replayed event's keys (flow.hpp header) grouped by key, every
// group in call order -- what the flow replay's edges and the account lanes' walks are read from.
//
// A library radix sort of the 64-bit (key, unit) words took ~20 launches per call (merge passes)
// and the lanes' pre-passes another ~10; the grouping here is six launches, none of them a sort of
// the whole pair array:
//
//   plan_keys      per replayed event: its keys (flow_keys' rules), its step record, the lanes'
//                  eligibility and record (lanes_check's rules); each key is counted in an LDS
//                  table of the workgroup's distinct keys, and each distinct key then takes its
//                  slot in an HBM hash table (key -> slot, CAS on an empty word) and its range in
//                  the slot with one add -- a hot account's thousands of pairs cost one probe and
//                  one add per workgroup -- and each pair keeps its arrival rank.
//   chained_scan   the slots' exclusive sums: every key's segment in the grouped array.
//   group_scatter  pair -> its segment at its rank (arrival order, not yet call order).
//   group_small    per slot: a segment of <= 16 pairs is sorted in registers by pair index (pair
//                  index 4 * position + j grows with the unit), one of <= 256 by the slot's wave
//                  (a rank sort through LDS), larger ones are listed. Then the
//                  segment's edges (a pair whose predecessor in the segment belongs to another
//                  unit adds to that unit's in-degree; the last pair of a unit's run names the
//                  next unit as its successor), its (key, unit) words, and -- for the account lanes
//                  -- owner segments with their free-owner verdict (lanes.hpp). The slot is
//                  cleared for the next call (the table is never memset).
//   group_sort     per listed segment, one workgroup: bitmaps of up to 2^20 pair indices in LDS
//                  over the segment's range (set bits, prefix popcounts, enumerate).
//   group_chunk    per 2048-pair chunk of a listed segment, one workgroup: the same per-pair work;
//                  an owner segment's last chunk adds up the chunks' contributions.
//
// Segments are disjoint and each is in call order, which is all the consumers read: flow_replay
// (succ / indeg), lanes_walk / lanes_replay (a segment ends where the key changes; the grouped
// pair count bounds the array). The order of the segments themselves is arbitrary.
#pragma once

#include "lanes.hpp"
#include "prims.hpp"

namespace tbg {

constexpr uint32_t kGroupSmall = 16;        // segments sorted in registers
constexpr uint32_t kGroupMid = 256;         // segments sorted by one wave (rank sort, LDS)
constexpr uint32_t kGroupBigThreads = 512;
constexpr uint32_t kGroupLdsWords = 32768;  // 128 KB: one bitmap window
constexpr uint32_t kGroupWindowBits = kGroupLdsWords * 32;
constexpr uint32_t kGroupBigBlocks = 256;
constexpr uint32_t kGroupBatch = 4;         // consecutive pairs per lane (group_chunk)
constexpr uint32_t kGroupChunk = kGroupBigThreads * kGroupBatch;  // pairs per group_chunk workgroup
constexpr uint32_t kGroupChunkBlocks = 512;  // group_chunk grid (grid-stride over the chunks)
constexpr uint32_t kPlanThreads = 256;      // plan_keys workgroup: 1024 pairs
constexpr uint32_t kPlanLdsSlots = 2048;    // LDS aggregation table (load <= 0.5)
// plan_keys' workgroup (512 / 1024 lanes, fewer global adds per hot slot: 46 / 58 us a plan
// against 43, profiles/r05_commit/ab_plan_keys.txt)
constexpr uint32_t kPlanKeysThreads = 256;
constexpr uint32_t kPlanKeysSlots = 8 * kPlanKeysThreads;  // (kFlowKeys per lane, load <= 0.5)

struct GroupPlan {
    uint64_t hmask;                 // hash slots - 1
    unsigned long long* hkeys;      // per slot: key + 1 (0 empty); key = type << 32 | index
    uint32_t* hcnt;                 // per slot: pairs
    uint32_t* hoff;                 // per slot: exclusive sum of hcnt
    uint32_t* loc;                  // per pair: slot (kNone32: no key)
    uint32_t* rank;                 // per pair: arrival rank within its slot
    uint32_t* vals;                 // grouped pair indices (arrival order within a segment)
    uint32_t* vals_sorted;          // large segments: pair indices in order
    uint64_t* keys_sorted;          // grouped (key, unit) words: flow_key(type, index, unit)
    uint4* big;                     // listed segments: {offset, count, key lo, key hi}
    unsigned int* counts;           // [0] grouped pairs, [1] listed segments, [2] / [3] the
                                    // longest id-key / account-key segment (pairs), [4] chunks
                                    // of the listed segments
    uint32_t* chunk_seg;            // per chunk of a listed segment: the segment's entry in big
    unsigned long long* chunk_sum;  // per chunk: u128 {lo, hi} of its owner contributions
    unsigned int* seg_done;         // per listed segment: chunks finished (group_chunk)
    const uint32_t* unit_of;        // per position
    uint32_t* succ;                 // per pair
    uint32_t* indeg;                // per unit
    // account lanes (lanes.hpp): owner segments and free owners; lanes == false: none
    bool lanes;
    bool free_owners;               // free-owner verdicts (TBG_NO_FREE_OWNERS: none)
    bool stats;                     // counts[2] / [3] (TBG_FLOW_DEBUG)
    uint32_t pairs;                 // kFlowKeys * m: every pair index is below it
    uint32_t epoch;
    uint32_t* owner_starts;
    unsigned int* lane_counts;      // [0] owners, [1] ineligible events
    const LaneRec* recs;            // per position
    uint32_t* acc_free;             // per account row
};

__device__ inline uint64_t group_hash(uint64_t key) { return mix64(key ^ 0x94D049BB133111EBull); }

// The slot of `key` in the grouping table (inserting it). Words only go 0 -> key + 1, so a stale 0
// read is settled by the CAS and a nonzero read is final.
__device__ inline uint32_t group_slot(const GroupPlan& G, uint64_t key) {
    const unsigned long long tag = key + 1;
    uint64_t s = group_hash(key) & G.hmask;
    while (true) {
        unsigned long long w = G.hkeys[s];
        if (w == 0) {
            w = atomicCAS(&G.hkeys[s], 0ull, tag);
            if (w == 0) return uint32_t(s);
        }
        if (w == tag) return uint32_t(s);
        s = (s + 1) & G.hmask;
    }
}

// The slots of up to kFlowKeys keys (kFlowNoKey: none): every home word is read, and every empty
// one claimed, before any result is waited on -- one or two round trips for the event instead of
// one per key; equal keys share the first one's slot, collisions continue in group_slot.
template <uint32_t N>
__device__ inline void group_slots(const GroupPlan& G, const uint64_t (&key)[N], uint64_t none,
                                   uint32_t (&slot)[N]) {
    uint64_t h[N];
    unsigned long long w[N];
#pragma unroll
    for (uint32_t j = 0; j < N; j++) {
        h[j] = group_hash(key[j]) & G.hmask;
        w[j] = key[j] != none ? G.hkeys[h[j]] : 1ull;
    }
    bool same[N];
#pragma unroll
    for (uint32_t j = 0; j < N; j++) {
        same[j] = false;
#pragma unroll
        for (uint32_t i = 0; i < j; i++) same[j] |= key[i] == key[j];
        if (key[j] != none && !same[j] && w[j] == 0)
            w[j] = atomicCAS(&G.hkeys[h[j]], 0ull, (unsigned long long)(key[j] + 1));
    }
#pragma unroll
    for (uint32_t j = 0; j < N; j++) {
        slot[j] = kNone32;
        if (key[j] == none) continue;
        if (same[j]) {
            for (uint32_t i = 0; i < j; i++)
                if (key[i] == key[j]) {
                    slot[j] = slot[i];
                    break;
                }
            continue;
        }
        slot[j] = (w[j] == 0 || w[j] == key[j] + 1) ? uint32_t(h[j]) : group_slot(G, key[j]);
    }
}

// Pair `pair`'s slot and rank (entry kNone32: no key).
template <typename B_>
__device__ inline void group_block_place(const GroupPlan& G, const B_& B, uint64_t pair,
                                         uint32_t entry, uint32_t lrank) {
    if (entry == kNone32) {
        G.loc[pair] = kNone32;
    } else {
        G.loc[pair] = B.slot[entry];
        G.rank[pair] = B.count[entry] + lrank;
    }
}

// plan_keys' counting by KEY within the workgroup: every lane counts its keys in an LDS table of
// the workgroup's distinct keys first; then each distinct key takes its global slot (group_slots:
// the home words read, the empty ones claimed) and its range in the slot (one add) -- one global
// probe and one add per distinct key of the workgroup instead of a probe (and, for a key first
// seen, a CAS) per pair: a hot account's thousands of pairs in a call all found its home word
// empty at once and all tried to claim it (config 3: TA_ADDR_STALLED_BY_TC 8.3M cycles a launch,
// profiles/r05_commit/pmc_config3.json).
template <uint32_t THREADS, uint32_t SLOTS>
struct GroupKeyBlockT {
    static constexpr uint32_t kThreads = THREADS, kSlots = SLOTS;
    unsigned long long key[SLOTS];  // key + 1 (0: empty)
    uint32_t count[SLOTS];          // the key's pairs here, then the base of their range
    uint32_t slot[SLOTS];           // the key's global slot
};
template <typename B_>
__device__ inline void group_key_init(B_& B) {
    for (uint32_t i = threadIdx.x; i < B_::kSlots; i += B_::kThreads) {
        B.key[i] = 0;
        B.count[i] = 0;
    }
    __syncthreads();
}
// Counts `key` in the workgroup: returns its LDS entry (*lrank: its rank among the workgroup's).
template <typename B_>
__device__ inline uint32_t group_key_count(B_& B, uint64_t key, uint32_t* lrank) {
    const unsigned long long tag = key + 1;
    uint32_t h = uint32_t(group_hash(key)) & (B_::kSlots - 1);
    while (true) {
        const unsigned long long o = atomicCAS(&B.key[h], 0ull, tag);
        if (o == 0 || o == tag) break;
        h = (h + 1) & (B_::kSlots - 1);
    }
    *lrank = atomicAdd(&B.count[h], 1u);
    return h;
}
// Each distinct key: its global slot and the base of its range (the lane's kPer entries' probes
// and adds issued together).
template <typename B_>
__device__ inline void group_key_publish(const GroupPlan& G, B_& B) {
    __syncthreads();
    constexpr uint32_t kPer = B_::kSlots / B_::kThreads;
    uint64_t k[kPer];
    uint32_t gs[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const unsigned long long t = B.key[threadIdx.x + j * B_::kThreads];
        k[j] = t ? t - 1 : kFlowNoKey;
    }
    group_slots(G, k, kFlowNoKey, gs);
    uint32_t base[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t i = threadIdx.x + j * B_::kThreads;
        base[j] = k[j] != kFlowNoKey ? atomicAdd(&G.hcnt[gs[j]], B.count[i]) : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t i = threadIdx.x + j * B_::kThreads;
        B.slot[i] = gs[j];
        B.count[i] = base[j];
    }
    __syncthreads();
}

// ---- Doomed debits ------------------------------------------------------------------------------
//
// An account L with debits_must_not_exceed_credits fails a debit of `amount` (exceeds_credits,
// create_transfer :3907-3909) whenever dpe + dpo + amount > cpo. Within one call, dpe and dpo of L
// only grow unless a post / void resolves a pending transfer of L, and cpo grows at most by the
// posted credits the call's replayed events carry to L (every event touching L replays: L's limit
// marks it hot, so no FAST event touches it). So a replayed debit of L with
//     dpe0 + dpo0 + amount > cpo0 + (the call's replayed posted credits to L)
// (balances at the plan, after the FAST deltas) fails at whatever point of the call it runs, and
// its unit needs no ordering with the other units of L: plan_keys gives it no key on L. (The
// account lanes decide such events themselves. Duplicate ids add every claimant's credits; a
// post/void whose pending transfer is uncertain -- plan_keys' rule -- turns it off for the call.)
constexpr uint32_t kPotUnbounded = 0xFFFFFFFFu;

__device__ inline bool pot_limited(const tb_account_t& a) {
    return (a.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) != 0;
}
// Adds `amount` to L's potential for this call (saturating: all-ones = unbounded).
__device__ inline void pot_add(unsigned long long* w, uint32_t epoch, uint64_t amount) {
    unsigned long long old = *w;
    while (true) {
        const uint32_t e = uint32_t(old >> 32), sum = e == epoch ? uint32_t(old) : 0u;
        const uint64_t add = sum == kPotUnbounded ? 0 : amount;
        const uint64_t next_sum = uint64_t(sum) + add >= kPotUnbounded ? kPotUnbounded : sum + add;
        const unsigned long long want = (uint64_t(epoch) << 32) | next_sum;
        if (want == old) return;
        const unsigned long long seen = atomicCAS(w, old, want);
        if (seen == old) return;
        old = seen;
    }
}
// L's potential this call (0 when no replayed event credits it).
__device__ inline uint32_t pot_of(const unsigned long long* w, uint32_t epoch) {
    const unsigned long long v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return uint32_t(v >> 32) == epoch ? uint32_t(v) : 0u;
}

__global__ void flow_credit_pot(Tables T, Call<tb_transfer_t> c, FlowPlan P,
                                unsigned int call_flags) {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= P.m) return;
    const uint32_t k = P.slow_list[s];
    const tb_transfer_t& t = c.events[k];
    if (t.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) {
        // A post / void changes its pending transfer's accounts' dpe (and dpo, cpo): both sides,
        // if limited, are unbounded; an uncertain pending transfer turns the rule off.
        // (plan_keys' certainty rule: with duplicate ids a pending id not found now, or held in
        // the call by an event with later claimants, may be another event's -- the rule is off)
        if (u128_is_zero(t.pending_id) || u128_is_max(t.pending_id)) return;
        const uint64_t ps = transfer_slot_find(T, c, t.pending_id);
        if (ps == kNone) {
            if (call_flags & kFlagDuplicate) *P.doom_off = P.epoch;
            return;
        }
        const uint64_t w = T.tr.slots[ps];
        const uint64_t r = (w & kRefMask) - 1;
        const tb_transfer_t* p = nullptr;
        if (r < c.row_base) {
            if (!(w & kOrphanBit)) p = &T.tr_rows[r];
        } else {
            const uint32_t j = uint32_t(r - c.row_base);
            if (P.dup_mark[j] == P.epoch) {
                *P.doom_off = P.epoch;
                return;
            }
            p = &c.events[j];
        }
        if (!p) return;
        const uint64_t dr = account_find(T, p->debit_account_id);
        const uint64_t cr = account_find(T, p->credit_account_id);
        if (dr != kNone && pot_limited(T.acc_rows[dr])) pot_add(&P.acc_pot[dr], P.epoch, kPotUnbounded);
        if (cr != kNone && pot_limited(T.acc_rows[cr])) pot_add(&P.acc_pot[cr], P.epoch, kPotUnbounded);
        return;
    }
    if (t.flags & TB_TRANSFER_PENDING) return;  // (a pending credit adds to cpe, not cpo)
    const uint32_t cr = c.ev_cr[k];
    if (cr == kNone32 || !pot_limited(T.acc_rows[cr])) return;
    pot_add(&P.acc_pot[cr], P.epoch, t.amount.hi ? kPotUnbounded : t.amount.lo);
}

// Is replayed event t (debit account row dr) doomed (the rule above)?
__device__ inline bool doomed_debit(const Tables& T, const FlowPlan& P, const tb_transfer_t& t,
                                   uint32_t dr) {
    if (!P.acc_pot || dr == kNone32 || *P.doom_off == P.epoch) return false;
    if (t.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING | TB_TRANSFER_BALANCING_DEBIT |
                   TB_TRANSFER_BALANCING_CREDIT | TB_TRANSFER_IMPORTED))
        return false;
    if (t.amount.hi != 0 || t.amount.lo >= (1ull << 56)) return false;
    const tb_account_t& a = T.acc_rows[dr];
    if (!pot_limited(a) || T.acc_closable[dr] == P.epoch) return false;
    constexpr uint64_t kLim = 1ull << 62;
    if (a.debits_pending.hi || a.debits_posted.hi || a.credits_posted.hi ||
        a.debits_pending.lo >= kLim || a.debits_posted.lo >= kLim || a.credits_posted.lo >= kLim)
        return false;
    const uint32_t pot = pot_of(&P.acc_pot[dr], P.epoch);
    if (pot == kPotUnbounded) return false;
    return a.debits_pending.lo + a.debits_posted.lo + t.amount.lo > a.credits_posted.lo + pot;
}

// Everything per replayed event s (flow_keys' and lanes_check's rules); its keys' grouping slots
// and ranks. Launched with kPlanThreads per workgroup.
__global__ void __launch_bounds__(kPlanKeysThreads) plan_keys(Tables T, Call<tb_transfer_t> c,
                                                              FlowPlan P, GroupPlan G,
                                                              LanePlan L, unsigned int call_flags) {
    __shared__ GroupKeyBlockT<kPlanKeysThreads, kPlanKeysSlots> B;
    group_key_init(B);
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t key[kFlowKeys] = {kFlowNoKey, kFlowNoKey, kFlowNoKey, kFlowNoKey};
    uint32_t local[kFlowKeys] = {kNone32, kNone32, kNone32, kNone32};
    uint32_t lrank[kFlowKeys] = {0, 0, 0, 0};
    bool ineligible = false;
    if (s < P.m) {
        const uint32_t k = P.slow_list[s];
        const uint32_t u = P.unit_of[s];
        const tb_transfer_t& t = c.events[k];
        // A chain longer than the lanes' undo logs is a barrier (the serial replay).
        if (P.heads[u] == s) {
            const uint32_t end = u + 1 < P.counts[0] ? P.heads[u + 1] : P.m;
            if (end - s > kFlowChainMax) P.barrier8[u] = 1;
        }
        auto keyless = [&](uint64_t row) { return acc_additive(T, row, P.add_epoch); };
        uint32_t pslot = kPvNoHint, pdr = kNone32, pcr = kNone32;  // a post/void's pending
        uint32_t add = kAddKnown;  // the replay's additive verdicts (EvRefs::add)
        // (an id key orders the events of one id, and a post/void after its pending transfer's
        // creator: a call without duplicate ids or post/void needs none -- every id slot is then
        // its own event's)
        if ((call_flags & (kFlagDuplicate | kFlagPostVoid)) && !u128_is_zero(t.id) &&
            !u128_is_max(t.id))
            key[0] = flow_id_key(t.id);
        if (t.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) {
            if (!u128_is_zero(t.pending_id) && !u128_is_max(t.pending_id)) {
                key[1] = flow_id_key(t.pending_id);
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
                } else {
                    pslot = ps == kNone ? kNone32 : uint32_t(ps);
                    if (p) {
                        const uint64_t dr = account_find(T, p->debit_account_id);
                        const uint64_t cr = account_find(T, p->credit_account_id);
                        if (dr != kNone && !keyless(dr)) key[2] = (1ull << 32) | uint32_t(dr);
                        if (cr != kNone && !keyless(cr)) key[3] = (1ull << 32) | uint32_t(cr);
                        if (dr != kNone && keyless(dr)) add |= kAddDr;
                        if (cr != kNone && keyless(cr)) add |= kAddCr;
                        pdr = dr == kNone ? kNone32 : uint32_t(dr);
                        pcr = cr == kNone ? kNone32 : uint32_t(cr);
                    }
                }
            }
        } else {
            const uint32_t dr = c.ev_dr[k], cr = c.ev_cr[k];
            // (a doomed debit reads L's balances in any order: no key on L)
            if (dr != kNone32 && !keyless(dr) && !(!G.lanes && doomed_debit(T, P, t, dr)))
                key[2] = (1ull << 32) | dr;
            if (cr != kNone32 && !keyless(cr)) key[3] = (1ull << 32) | cr;
            if (dr != kNone32 && keyless(dr)) add |= kAddDr;
            if (cr != kNone32 && keyless(cr)) add |= kAddCr;
        }
        // The expires_at entry a created pending transfer with a timeout appends (planned: one
        // slot per candidate position; a candidate that fails or whose chain is discarded leaves
        // an entry of a row that is not live, dropped at the next pulse).
        P.exp_flag[s] = (t.flags & TB_TRANSFER_PENDING) && t.timeout > 0 &&
                        !(t.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING));
        const StepInfo si = step_info(c, k, uint16_t(TB_TRANSFER_IMPORTED));
        const EvRefs x = ev_refs(c, k);
        Step st;
        st.ts_event = si.ts_event;
        st.batch = si.batch;
        st.flags = si.flags;
        st.k = k;
        st.slot = x.slot;
        const bool pv = (t.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) != 0;
        st.dr = pv ? pdr : x.dr;  // (a post/void's own accounts are read only by the lanes
        st.cr = pv ? pcr : x.cr;  // check, which a post/void never passes)
        st.pslot = pslot;
        st.add = add;
        P.steps[s] = st;
        copy_row(&P.evs[s], &c.events[k]);
        P.indeg[s] = 0;  // (units < m)
        *reinterpret_cast<uint4*>(G.succ + kFlowKeys * uint64_t(s)) =
            make_uint4(kNone32, kNone32, kNone32, kNone32);
        if (G.lanes) {
            // lanes_check: a limit event (lanes.hpp header) or an ineligible one.
            bool ok = st.dr != kNone32 && st.cr != kNone32 && st.slot != kNone32 && st.dr != st.cr;
            ok = ok && P.heads[u] == s &&
                 (u + 1 == P.counts[0] ? s + 1 == L.m : P.heads[u + 1] == s + 1);
            ok = ok && t.flags == 0 && t.timeout == 0 && u128_is_zero(t.pending_id) &&
                 t.amount.hi == 0 && t.timestamp == 0 && !(st.flags & StepInfo::kBatchImported);
            uint32_t bits = 0;
            if (ok) {
                const uint64_t w = T.tr.slots[st.slot];
                ok = w != kEmpty && w != kTomb && (w & kRefMask) == c.row_base + k + 1;
                const tb_account_t& dr = T.acc_rows[st.dr];
                const tb_account_t& cr = T.acc_rows[st.cr];
                ok = ok && !((dr.flags | cr.flags) & TB_ACCOUNT_CLOSED) && lanes_low(dr) &&
                     lanes_low(cr) && dr.ledger == cr.ledger && t.ledger == dr.ledger &&
                     t.code != 0 && t.ledger != 0 && !u128_is_zero(t.id) && !u128_is_max(t.id);
                if (lanes_owner(dr.flags)) bits |= kLaneDrOwner;
                if (lanes_owner(cr.flags)) bits |= kLaneCrOwner;
                if (dr.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) bits |= kLaneDrDecides;
                if (cr.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) bits |= kLaneCrDecides;
                ok = ok && (bits & (kLaneDrOwner | kLaneCrOwner)) != 0;
            }
            L.mailbox[s] = ok && (bits & (kLaneDrOwner | kLaneCrOwner)) ==
                                     (kLaneDrOwner | kLaneCrOwner);
            L.mb_index[s] = 0;  // the walk's verdict words (one-lane mode: rewritten)
            ineligible = !ok;
            if (ok) {
                LaneRec r;
                r.amount = t.amount.lo;
                r.dr = st.dr;
                r.bits = bits;
                L.recs[s] = r;
            }
        }
        // Grouping: this workgroup's count of each key in LDS (the global slots follow, once per
        // distinct key: group_key_publish).
#pragma unroll
        for (uint32_t j = 0; j < kFlowKeys; j++)
            if (key[j] != kFlowNoKey) local[j] = group_key_count(B, key[j], &lrank[j]);
    }
    if (G.lanes) {
        const uint64_t bad = __ballot(ineligible);
        if ((threadIdx.x & 63) == 0 && bad) atomicAdd(&L.counts[1], uint32_t(__popcll(bad)));
    }
    group_key_publish(G, B);
    if (s >= P.m) return;
#pragma unroll
    for (uint32_t j = 0; j < kFlowKeys; j++)
        group_block_place(G, B, kFlowKeys * uint64_t(s) + j, local[j], lrank[j]);
}

__global__ void group_scatter(GroupPlan G, uint64_t pairs) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= pairs) return;
    const uint32_t slot = G.loc[i];
    if (slot == kNone32) return;
    G.vals[G.hoff[slot] + G.rank[i]] = uint32_t(i);
}

// Pair v of a segment at grouped position `at` (key `key`), its unit u, and the units of its
// neighbours in the segment (kNone32 at the ends): the (key, unit) word, the successor, and the
// in-degree edge.
__device__ inline void group_emit(const GroupPlan& G, uint64_t at, uint64_t key, uint32_t v,
                                  uint32_t u, uint32_t u_prev, uint32_t u_next) {
    G.keys_sorted[at] = (key << kFlowUnitBits) | u;
    G.succ[v] = (u_next != kNone32 && u_next != u) ? u_next : kNone32;
    if (u_prev != kNone32 && u_prev != u) atomicAdd(&G.indeg[u], 1u);
}

// The free-owner verdict of an owner segment from the sum of the amounts its limit checks
// (lanes.hpp, free owners).
__device__ inline void group_owner_verdict(Tables T, const GroupPlan& G, uint32_t row, u128 sum) {
    const tb_account_t& a = T.acc_rows[row];
    const u128 dpe = U(a.debits_pending), dpo = U(a.debits_posted);
    const u128 cpe = U(a.credits_pending), cpo = U(a.credits_posted);
    // (every balance < 2^126 and the sum < 2^96 for an eligible call: no wrap below)
    if (!G.free_owners) return;
    bool free = true;
    if (a.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) free = free && dpe + dpo + sum <= cpo;
    if (a.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) free = free && cpe + cpo + sum <= dpo;
    if (free) G.acc_free[row] = G.epoch;
}

// The amount owner `row` checks on pair v's event (0: none).
__device__ inline uint64_t group_owner_contrib(const GroupPlan& G, uint32_t row, uint32_t v) {
    const LaneRec r = G.recs[v / kFlowKeys];
    const bool debit = r.dr == row;
    return (debit ? (r.bits & kLaneDrDecides) : (r.bits & kLaneCrDecides)) ? r.amount : 0;
}

// Is this segment an account lanes owner of a call the lanes run (every replayed event eligible)?
__device__ inline bool group_owner_probe(Tables T, const GroupPlan& G, uint64_t key) {
    return G.lanes && (key >> 32) == 1 && G.lane_counts[1] == 0 &&
           lanes_owner(T.acc_rows[uint32_t(key)].flags);
}
// Registers an owner segment (owner_starts; any order: one walk per owner).
__device__ inline void group_owner_add(const GroupPlan& G, uint32_t off) {
    G.owner_starts[atomicAdd(&G.lane_counts[0], 1u)] = off;
}

template <int N>
__device__ inline void sort_network(uint32_t (&v)[N]) {
#pragma unroll
    for (int k = 2; k <= N; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1)
#pragma unroll
            for (int i = 0; i < N; i++) {
                const int l = i ^ j;
                if (l > i) {
                    const bool up = (i & k) == 0;
                    const uint32_t a = v[i], b = v[l];
                    if ((a > b) == up) {
                        v[i] = b;
                        v[l] = a;
                    }
                }
            }
}

// Workgroup sums (kGroupBigThreads lanes).
__device__ inline uint32_t group_block_exclusive(uint32_t x, uint32_t* total, uint32_t* scratch) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t incl = wave_inclusive_u32(x, lane);
    if (lane == 63) scratch[wave] = incl;
    __syncthreads();
    uint32_t before = 0, all = 0;
    for (uint32_t w = 0; w < kGroupBigThreads / 64; w++) {
        if (w < wave) before += scratch[w];
        all += scratch[w];
    }
    __syncthreads();
    *total = all;
    return before + incl - x;
}

// LDS of a segment-sorting workgroup.
struct SegmentLds {
    uint32_t buf[kGroupLdsWords];
    uint32_t scratch[kGroupBigThreads / 64];
    uint32_t red_min[kGroupBigThreads / 64], red_max[kGroupBigThreads / 64];
};

// Sorts the c distinct values in[off, off + c) ascending into out[off, off + c) (one workgroup of
// kGroupBigThreads; visible to the whole workgroup on return -- a workgroup barrier: the callers'
// other readers are later kernels. An agent-scope fence here wrote back the XCD's L2 once per
// segment.): bitmap windows of up to
// kGroupWindowBits values in LDS over the values' range -- set bits, prefix popcounts, enumerate --
// or, for a sparse segment, an LDS bitonic sort of the values themselves.
// Wave scans on DPP for the bitmap windows (every lane active): lanes_walk's sequence (a
// __shfl_up scan is six dependent LDS permutes).
__device__ inline uint32_t seg_wave_inclusive(uint32_t v) {
    v += walk_dpp<0x111, 0xF>(v);  // row_shr:1
    v += walk_dpp<0x112, 0xF>(v);  // row_shr:2
    v += walk_dpp<0x114, 0xF>(v);  // row_shr:4
    v += walk_dpp<0x118, 0xF>(v);  // row_shr:8
    v += walk_dpp<0x142, 0xA>(v);  // row_bcast:15
    v += walk_dpp<0x143, 0xC>(v);  // row_bcast:31
    return v;
}
__device__ inline uint32_t seg_wave_last(uint32_t v) {
    return uint32_t(__builtin_amdgcn_readlane(int(v), 63));
}

// `compress` (the grouping's pair indices, group_sort): a segment's pair indices 4 s + j all have
// the same j >> 1 (id keys j 0 / 1, account keys 2 / 3), so 2 s + (j & 1) is one-to-one and keeps
// their order: the bitmap covers half the range, and `jhi` (j & 2) restores the indices.
__device__ inline void segment_sort(const uint32_t* in, uint32_t* out, uint32_t off, uint32_t c,
                                    SegmentLds& L, bool values = false, uint32_t bound = 0,
                                    bool compress = false, uint32_t jhi = 0) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t* buf = L.buf;
    // The segment's values, 16 loads a lane in flight at a time (a loop of one load per iteration
    // waits out every load in turn: ~50 round trips for a hot account's segment).
    constexpr uint32_t kB = 16;
    auto for_values = [&](auto&& fn) {
        for (uint32_t i0 = tid; i0 < c; i0 += kB * kGroupBigThreads) {
            uint32_t v[kB];
#pragma unroll
            for (uint32_t j = 0; j < kB; j++) {
                const uint32_t i = i0 + j * kGroupBigThreads;
                v[j] = i < c ? in[off + i] : 0u;
            }
#pragma unroll
            for (uint32_t j = 0; j < kB; j++)
                if (i0 + j * kGroupBigThreads < c) fn(i0 + j * kGroupBigThreads, v[j]);
        }
    };
    // Bitmap windows of kGroupWindowBits over [lo, hi]: set bits, prefix popcounts, enumerate.
    auto bitmap_window = [&](uint32_t lo, uint32_t hi) {
        uint32_t placed = 0;
        for (uint64_t wb = lo; wb <= hi; wb += kGroupWindowBits) {
            // the window's words, rounded up to whole lanes' shares
            const uint64_t span = hi - wb + 1 < kGroupWindowBits ? hi - wb + 1 : kGroupWindowBits;
            const uint32_t per = uint32_t((span + 32 * kGroupBigThreads - 1) / (32 * kGroupBigThreads));
            const uint32_t words = per * kGroupBigThreads;
            for (uint32_t i = tid; i < words; i += kGroupBigThreads) buf[i] = 0;
            __syncthreads();
            for_values([&](uint32_t, uint32_t v) {
                const uint32_t cv = compress ? ((v >> 2) << 1) | (v & 1) : v;
                if (cv >= wb && cv - wb < kGroupWindowBits) {
                    const uint32_t d = uint32_t(cv - wb);
                    atomicOr(&buf[d >> 5], 1u << (d & 31));
                }
            });
            __syncthreads();
            // Each wave enumerates a contiguous range of the window's words, 64 consecutive
            // words (one a lane, conflict-free LDS reads) at a time; the wave totals' prefix
            // places the waves. (A lane owning `per` consecutive words read them 32-way
            // bank-conflicted: ~13 us a window.)
            constexpr uint32_t kWaves = kGroupBigThreads / 64;
            const uint32_t ww = words / kWaves, wbase = wave * ww;
            uint32_t cnt = 0;
            for (uint32_t r = 0; r < ww; r += 64) cnt += __popc(buf[wbase + r + lane]);
            cnt = seg_wave_last(seg_wave_inclusive(cnt));
            if (lane == 0) L.scratch[wave] = cnt;
            __syncthreads();
            uint32_t run = placed, total = 0;
            for (uint32_t v = 0; v < kWaves; v++) {
                const uint32_t cv = L.scratch[v];
                run += v < wave ? cv : 0u;
                total += cv;
            }
            for (uint32_t r = 0; r < ww; r += 64) {
                uint32_t bits = buf[wbase + r + lane];
                const uint32_t pc = __popc(bits);
                const uint32_t incl = seg_wave_inclusive(pc);
                uint32_t pos = run + incl - pc;
                const uint64_t word_bit = wb + uint64_t(wbase + r + lane) * 32;
                while (bits) {
                    const uint32_t bit = __builtin_ctz(bits);
                    bits &= bits - 1;
                    const uint32_t idx = uint32_t(word_bit + bit);
                    out[off + pos++] = compress ? ((idx >> 1) << 2) | jhi | (idx & 1) : idx;
                }
                run += seg_wave_last(incl);
            }
            placed += total;
            __syncthreads();
        }
    };
    uint32_t lo = kNone32, hi = 0;
    if (bound && bound <= kGroupWindowBits && !values) {
        // every value is below `bound` (a call's pair indices): one bitmap window over
        // [0, bound), no pass over the values for their range
        bitmap_window(0, bound - 1);
        return;
    }
    for_values([&](uint32_t, uint32_t v) {
        const uint32_t cv = compress ? ((v >> 2) << 1) | (v & 1) : v;  // (the bitmap's index)
        lo = min(lo, cv);
        hi = max(hi, cv);
    });
    for (int d = 32; d >= 1; d >>= 1) {
        lo = min(lo, uint32_t(__shfl_xor(lo, d, 64)));
        hi = max(hi, uint32_t(__shfl_xor(hi, d, 64)));
    }
    if (lane == 0) {
        L.red_min[wave] = lo;
        L.red_max[wave] = hi;
    }
    __syncthreads();
    lo = L.red_min[0];
    hi = L.red_max[0];
    for (uint32_t w = 1; w < kGroupBigThreads / 64; w++) {
        lo = min(lo, L.red_min[w]);
        hi = max(hi, L.red_max[w]);
    }
    // A sparse segment (its range many times its count: a call's touches of one account spread
    // over the whole call) sorts faster as values than as a bitmap of its range: LDS bitonic
    // sort of the next power of two >= c (kNone32 padding), when it fits the buffer.
    uint32_t pw = 1;
    while (pw < c) pw <<= 1;
    // (A range within one bitmap window takes the bitmap whatever its density: clearing, setting,
    // counting and enumerating 2^20 bits costs a few microseconds, an LDS bitonic sort of 32k
    // values ~40 -- config 3's hot accounts.)
    const uint64_t range = uint64_t(hi - lo) + 1;
    if (pw <= kGroupLdsWords && (values || (range > kGroupWindowBits && range > 64ull * pw))) {
        for (uint32_t i = c + tid; i < pw; i += kGroupBigThreads) buf[i] = kNone32;
        for_values([&](uint32_t i, uint32_t v) { buf[i] = v; });
        __syncthreads();
        for (uint32_t size = 2; size <= pw; size <<= 1) {
            for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
                for (uint32_t t = tid; t < pw / 2; t += kGroupBigThreads) {
                    const uint32_t a = 2 * t - (t & (stride - 1)), b = a + stride;
                    const uint32_t x = buf[a], y = buf[b];
                    if ((x > y) == ((a & size) == 0)) {
                        buf[a] = y;
                        buf[b] = x;
                    }
                }
                __syncthreads();
            }
        }
        for (uint32_t i = tid; i < c; i += kGroupBigThreads) out[off + i] = buf[i];
        __syncthreads();
        return;
    }
    bitmap_window(lo, hi);
}

// A segment of kGroupSmall < c <= kGroupMid values sorted by one wave: lane l holds values
// l + 64 j; each value's rank is the count of smaller values (every value broadcast once); the
// values land in buf[rank]. All lanes of the wave call it with the same arguments.
__device__ inline void wave_rank_sort(const uint32_t* in, uint32_t off, uint32_t c, uint32_t* buf) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t x[4], r[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) x[j] = lane + 64 * j < c ? in[off + lane + 64 * j] : kNone32;
    for (uint32_t s = 0; s < c; s++) {
        const uint32_t src = s < 64 ? x[0] : s < 128 ? x[1] : s < 192 ? x[2] : x[3];
        const uint32_t y = __shfl(src, s & 63, 64);
#pragma unroll
        for (uint32_t j = 0; j < 4; j++) r[j] += y < x[j];
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; j++)
        if (lane + 64 * j < c) buf[r[j]] = x[j];
    wave_lds_sync();
}

// The flow plan's per-segment work for a wave-sorted segment (group_small's mid tier).
__device__ inline void group_mid_segment(Tables T, const GroupPlan& G, uint32_t off, uint32_t c,
                                         uint64_t key, uint32_t* buf) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t* units = buf + kGroupMid;
    wave_rank_sort(G.vals, off, c, buf);
    const bool owner = group_owner_probe(T, G, key);
    const uint32_t row = uint32_t(key);
    uint64_t sum_lo = 0, sum_hi = 0;
    uint32_t uu[4];
    uint64_t aa[4];
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        const uint32_t p = lane + 64 * j;
        uu[j] = p < c ? G.unit_of[buf[p] / kFlowKeys] : 0u;
        aa[j] = owner && p < c ? group_owner_contrib(G, row, buf[p]) : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        if (lane + 64 * j < c) units[lane + 64 * j] = uu[j];
        sum_lo += aa[j];
        sum_hi += sum_lo < aa[j];
    }
    wave_lds_sync();
    for (uint32_t p = lane; p < c; p += 64)
        group_emit(G, off + p, key, buf[p], units[p], p > 0 ? units[p - 1] : kNone32,
                   p + 1 < c ? units[p + 1] : kNone32);
    if (owner) {
        for (int d = 32; d >= 1; d >>= 1) {
            const uint64_t olo = __shfl_xor(sum_lo, d, 64);
            const uint64_t ohi = __shfl_xor(sum_hi, d, 64);
            const uint64_t nlo = sum_lo + olo;
            sum_hi = sum_hi + ohi + (nlo < sum_lo ? 1u : 0u);
            sum_lo = nlo;
        }
        if (lane == 0) {
            group_owner_add(G, off);
            group_owner_verdict(T, G, row, (u128(sum_hi) << 64) | sum_lo);
        }
    }
    wave_lds_sync();  // (buf is reused by the wave's next segment)
}

__global__ void __launch_bounds__(kBlock) group_small(Tables T, GroupPlan G, uint64_t slots) {
    __shared__ uint32_t wave_buf[kBlock / 64][2 * kGroupMid];
    const uint64_t h = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    uint32_t c = 0, off = 0;
    uint64_t key = 0;
    if (h < slots) {
        c = G.hcnt[h];
        if (c) {
            key = G.hkeys[h] - 1;
            off = G.hoff[h];
            G.hkeys[h] = 0;
            G.hcnt[h] = 0;
        }
    }
    if (G.stats) {  // the longest id-key / account-key segment (flow debug): one atomic per wave
        uint32_t id_max = (c > 1 && (key >> 32) == 0) ? c : 0u;
        uint32_t acc_max = (c > 1 && (key >> 32) == 1) ? c : 0u;
        for (int d = 32; d >= 1; d >>= 1) {
            id_max = max(id_max, uint32_t(__shfl_xor(id_max, d, 64)));
            acc_max = max(acc_max, uint32_t(__shfl_xor(acc_max, d, 64)));
        }
        if ((threadIdx.x & 63) == 0) {
            if (id_max) atomicMax(&G.counts[2], id_max);
            if (acc_max) atomicMax(&G.counts[3], acc_max);
        }
    }
    if (c > kGroupMid) {
        // Listed: ordered by group_sort, emitted by group_chunk in chunks of kGroupChunk pairs.
        const uint32_t b = atomicAdd(&G.counts[1], 1u);
        const uint32_t chunks = (c + kGroupChunk - 1) / kGroupChunk;
        const uint32_t cb = atomicAdd(&G.counts[4], chunks);
        G.big[b] = make_uint4(off, c, uint32_t(key), (uint32_t(key >> 32) << 31) | cb);
        G.seg_done[b] = 0;
        for (uint32_t q = 0; q < chunks; q++) G.chunk_seg[cb + q] = b;
    } else if (c == 1) {
        const uint32_t v = G.vals[off];
        group_emit(G, off, key, v, G.unit_of[v / kFlowKeys], kNone32, kNone32);
        if (group_owner_probe(T, G, key)) {
            group_owner_add(G, off);
            group_owner_verdict(T, G, uint32_t(key), group_owner_contrib(G, uint32_t(key), v));
        }
    } else if (c > 1 && c <= 4) {
        uint32_t v[4], u[4];
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) v[i] = i < c ? G.vals[off + i] : kNone32;
        sort_network(v);
#pragma unroll
        for (uint32_t i = 0; i < 4; i++) u[i] = i < c ? G.unit_of[v[i] / kFlowKeys] : kNone32;
#pragma unroll
        for (uint32_t i = 0; i < 4; i++)
            if (i < c)
                group_emit(G, off + i, key, v[i], u[i], i > 0 ? u[i - 1] : kNone32,
                           i + 1 < 4 ? u[i + 1] : kNone32);
        if (group_owner_probe(T, G, key)) {
            group_owner_add(G, off);
            u128 sum = 0;
#pragma unroll
            for (uint32_t i = 0; i < 4; i++)
                if (i < c) sum += group_owner_contrib(G, uint32_t(key), v[i]);
            group_owner_verdict(T, G, uint32_t(key), sum);
        }
    } else if (c > 4 && c <= kGroupSmall) {
        uint32_t v[kGroupSmall], u[kGroupSmall];
#pragma unroll
        for (uint32_t i = 0; i < kGroupSmall; i++) v[i] = i < c ? G.vals[off + i] : kNone32;
        sort_network(v);
#pragma unroll
        for (uint32_t i = 0; i < kGroupSmall; i++) u[i] = i < c ? G.unit_of[v[i] / kFlowKeys] : kNone32;
#pragma unroll
        for (uint32_t i = 0; i < kGroupSmall; i++)
            if (i < c)
                group_emit(G, off + i, key, v[i], u[i], i > 0 ? u[i - 1] : kNone32,
                           i + 1 < kGroupSmall ? u[i + 1] : kNone32);
        if (group_owner_probe(T, G, key)) {
            group_owner_add(G, off);
            u128 sum = 0;
#pragma unroll
            for (uint32_t i = 0; i < kGroupSmall; i++)
                if (i < c) sum += group_owner_contrib(G, uint32_t(key), v[i]);
            group_owner_verdict(T, G, uint32_t(key), sum);
        }
    }
    // The wave's mid-size segments, one at a time by the whole wave.
    uint64_t mids = __ballot(c > kGroupSmall && c <= kGroupMid);
    while (mids) {
        const int l = __ffsll((unsigned long long)mids) - 1;
        mids &= mids - 1;
        const uint32_t moff = __shfl(off, l, 64), mc = __shfl(c, l, 64);
        const uint64_t mkey = (uint64_t(uint32_t(__shfl(uint32_t(key >> 32), l, 64))) << 32) |
                              uint32_t(__shfl(uint32_t(key), l, 64));
        group_mid_segment(T, G, moff, mc, mkey, wave_buf[threadIdx.x >> 6]);
    }
}

// Listed segments, one workgroup each: the pairs in call order into vals_sorted.
__global__ void __launch_bounds__(kGroupBigThreads) group_sort(GroupPlan G) {
    __shared__ SegmentLds L;
    const uint32_t nbig = G.counts[1];
    for (uint32_t b = blockIdx.x; b < nbig; b += gridDim.x) {
        const uint4 e = G.big[b];
        // (the key's type, e.w's top bit: account keys' pairs have j >> 1 == 1)
        segment_sort(G.vals, G.vals_sorted, e.x, e.y, L, false, G.pairs / 2, true,
                     (e.w >> 31) ? 2u : 0u);
    }
}

// Chunks of the listed segments, one workgroup each (grid-stride): kGroupBatch consecutive pairs
// per lane with both neighbours, every load of a batch issued before any is used; an owner
// segment's chunks sum their contributions, and the segment's last chunk to finish (a counter,
// release / acquire at agent scope) adds them up for the free verdict and registers the owner.
__global__ void __launch_bounds__(kGroupBigThreads) group_chunk(Tables T, GroupPlan G) {
    __shared__ unsigned long long red_lo[kGroupBigThreads / 64], red_hi[kGroupBigThreads / 64];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t nchunks = G.counts[4];
    for (uint32_t g = blockIdx.x; g < nchunks; g += gridDim.x) {
        const uint32_t b = G.chunk_seg[g];
        const uint4 e = G.big[b];
        const uint32_t off = e.x, c = e.y, cb = e.w & 0x7FFFFFFFu;
        const uint64_t key = (uint64_t(e.w >> 31) << 32) | e.z;
        const uint32_t row = e.z;
        const bool owner = group_owner_probe(T, G, key);
        const uint32_t q = g - cb, chunks = (c + kGroupChunk - 1) / kGroupChunk;
        uint64_t sum_lo = 0, sum_hi = 0;
        const uint32_t i0 = q * kGroupChunk + tid * kGroupBatch;
        if (i0 < c) {
            uint32_t v[kGroupBatch + 2], u[kGroupBatch + 2];
#pragma unroll
            for (uint32_t j = 0; j < kGroupBatch + 2; j++) {
                const int64_t at = int64_t(i0) + j - 1;
                v[j] = at >= 0 && at < int64_t(c) ? G.vals_sorted[off + at] : kNone32;
            }
            uint64_t aa[kGroupBatch + 2];
#pragma unroll
            for (uint32_t j = 0; j < kGroupBatch + 2; j++) {
                u[j] = v[j] != kNone32 ? G.unit_of[v[j] / kFlowKeys] : kNone32;
                aa[j] = owner && j >= 1 && j <= kGroupBatch && v[j] != kNone32
                            ? group_owner_contrib(G, row, v[j]) : 0u;
            }
#pragma unroll
            for (uint32_t j = 1; j <= kGroupBatch; j++) {
                if (i0 + j - 1 >= c) break;
                group_emit(G, off + i0 + j - 1, key, v[j], u[j], u[j - 1], u[j + 1]);
                sum_lo += aa[j];
                sum_hi += sum_lo < aa[j];
            }
        }
        if (owner) {
            for (int d = 32; d >= 1; d >>= 1) {
                const uint64_t olo = __shfl_xor(sum_lo, d, 64);
                const uint64_t ohi = __shfl_xor(sum_hi, d, 64);
                const uint64_t nlo = sum_lo + olo;
                sum_hi = sum_hi + ohi + (nlo < sum_lo ? 1u : 0u);
                sum_lo = nlo;
            }
            if (lane == 0) {
                red_lo[wave] = sum_lo;
                red_hi[wave] = sum_hi;
            }
            __syncthreads();
            if (tid == 0) {
                u128 sum = 0;
                for (uint32_t w = 0; w < kGroupBigThreads / 64; w++)
                    sum += (u128(red_hi[w]) << 64) | red_lo[w];
                G.chunk_sum[2 * uint64_t(g)] = uint64_t(sum);
                G.chunk_sum[2 * uint64_t(g) + 1] = uint64_t(sum >> 64);
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
                if (atomicAdd(&G.seg_done[b], 1u) == chunks - 1) {
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    u128 all = 0;
                    for (uint32_t j = 0; j < chunks; j++) {
                        const uint64_t lo = __hip_atomic_load(&G.chunk_sum[2 * uint64_t(cb + j)],
                                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        const uint64_t hi = __hip_atomic_load(&G.chunk_sum[2 * uint64_t(cb + j) + 1],
                                                              __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        all += (u128(hi) << 64) | lo;
                    }
                    group_owner_add(G, off);
                    group_owner_verdict(T, G, row, all);
                }
            }
            __syncthreads();  // (red_* are rewritten by the next chunk)
        }
    }
}

// Scan ops of the plan.

// Initially ready units (no predecessor) -> the engine's queue (unit + 1), q_tail, counts[2].
struct SelectReady {
    static constexpr bool kEmitAll = false;
    const uint32_t* indeg;
    const unsigned int* counts;  // [0] units
    uint32_t* queue;
    unsigned int* engine;
    unsigned int* ready_count;
    uint32_t* indeg0;            // the in-degrees' copy (FlowPlan::indeg0)
    __device__ void load(uint64_t base, uint64_t n, uint32_t* c) const {
        const uint32_t units = counts[0];
#pragma unroll
        for (uint32_t i = 0; i < kScanItems; i++) {
            const bool unit = base + i < n && base + i < units;
            const uint32_t d = unit ? indeg[base + i] : 1u;
            if (unit) indeg0[base + i] = d;
            c[i] = d == 0;
        }
    }
    __device__ void emit(uint64_t u, uint32_t p) const { queue[p] = uint32_t(u) + 1; }
    __device__ void total(uint32_t t) const {
        engine[32] = t;
        *ready_count = t;
    }
};

// The planned expires_at entries: candidate s takes slot base + its exclusive rank.
struct PlanExpiry {
    static constexpr bool kEmitAll = false;
    const uint32_t* exp_flag;
    const uint32_t* slow_list;
    uint64_t* expiry;
    uint64_t expiry_capacity;
    uint64_t row_base;
    const unsigned long long* base;  // expiry_count at the plan's start (flow_heads)
    unsigned long long* expiry_count;
    unsigned int* scalar_flags;
    __device__ void load(uint64_t b, uint64_t n, uint32_t* c) const {
#pragma unroll
        for (uint32_t i = 0; i < kScanItems; i++) c[i] = b + i < n ? exp_flag[b + i] : 0u;
    }
    __device__ void emit(uint64_t s, uint32_t p) const {
        const uint64_t i = *base + p;
        if (i < expiry_capacity) expiry[i] = row_base + slow_list[s];
        else atomicOr(scalar_flags, kFlagTableFull);
    }
    __device__ void total(uint32_t t) const {
        const uint64_t n = *base + t;
        *expiry_count = n < expiry_capacity ? n : expiry_capacity;
    }
};

}  // namespace tbg
