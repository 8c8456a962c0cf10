// AccountEvent emission (state_machine.zig:104-220 layout, account_event :4384-4465) and the
// get_change_events read side (:2396-2434, :3395-3527), over the HBM tables.
//
// The reference writes one AccountEvent per created transfer, post / void (:3964-3973,
// :4285-4294) and expiry (:4614-4623), carrying both accounts as they stand after the event:
// balances, `closed`, timestamps. Here the events are derived after a call has executed (by any
// path: parallel, lanes, flow or serial replay) from the call's created events in call order and
// the accounts' final rows: the balances of account A after event e are
//     final(A) - (sum of the deltas of A's later events in the call)
// (u128 modular arithmetic: exact, since every true balance is in [0, 2^128)), and A's `closed`
// after e is final(A).closed XOR (the parity of A's later closed flips: closing creations set it,
// voids of closing transfers and expiries of closing transfers clear it). Each event touches two
// accounts; the (account, event) touches are grouped by account (group.hpp: an HBM hash table,
// LDS-aggregated counts, a chained scan, a scatter), each account's touches put in event order
// (registers for <= 16, else one workgroup: LDS bitonic sort or bitmap windows), and a suffix sum
// over them gives every touch the sum of its account's later deltas.
// Chains that were rolled back left no created event, so their events never appear (the groove's
// scope discard). AccountEvents are in timestamp order within a call; the log is kept sorted.
//
// The collection pass writes each touch's half as the account's final row (id, balances, account
// timestamp, flags); the emit passes subtract the later touches' sums from it in place. Nothing
// after the collection reads the accounts, which lets a small call's appends run on a side stream
// behind the next call (ae_snapshot below).
#pragma once

#include "group.hpp"

namespace tbg {

// Reference of an AccountEvent for get_change_events: the transfer row (the pending transfer's
// for an expiry) and both account rows.
struct AeRef {
    uint32_t transfer_row, dr_row, cr_row, pad;
};

// One side of an event: the deltas it applies to its account's pending and posted field (debit
// side: debits_*, credit side: credits_*) and whether it flips `closed`.
struct AeDelta {
    u128 pending, posted;
    uint32_t flip, side;  // side 0: debit, 1: credit
    uint64_t pad;
};

// The running sums of an account's later touches (the four balances and the closed flips).
struct Bal5 {
    u128 dp, dpo, cp, cpo;
    uint32_t flips;
};
// (value selects, not a branch between fields: the compiler would pick a field pointer and keep
// the sums in scratch)
__device__ inline void bal5_add(Bal5& a, const AeDelta& d) {
    const bool dr = d.side == 0;
    const u128 pending = d.pending, posted = d.posted;
    a.dp += dr ? pending : u128(0);
    a.dpo += dr ? posted : u128(0);
    a.cp += dr ? u128(0) : pending;
    a.cpo += dr ? u128(0) : posted;
    a.flips += d.flip;
}

struct AeScratch {
    AeDelta* deltas;        // per touch (2 * event + side)
    // The kernels do nothing when *skip == skip_if (a small call's appends that ae_small_emit
    // took over; null: never).
    const unsigned int* skip = nullptr;
    uint32_t skip_if = 0;
    GroupPlan G;            // the touches grouped by account row (table, segments); G.counts:
                            // [0] grouped touches, [1] listed accounts, [2] their chunks
    uint32_t* chunk_seg;    // per chunk of a listed account: the account's entry in G.big
    Bal5* chunk_tot;        // per chunk: the sums of its touches
    unsigned long long* state;  // the log on device: [0] events, [1] last timestamp, [2] unsorted,
                                // [3] overflowed (sticky: an append found no room, wrote nothing)
    uint64_t cap = ~0ull;       // the log's capacity (records)
    // Touch v's event is v >> 1: its log position is pos[v >> 1] (the side stream's appends,
    // whose touches are numbered by call event), or v >> 1 itself when pos is null.
    const uint32_t* pos;
};

// Room in the log for m more records? Every append checks before it writes (the host's bound is
// an upper bound; this makes an error of it a reported overflow, never a write past the log).
__device__ inline bool ae_room(const unsigned long long* state, uint64_t cap, uint64_t m) {
    return state[3] == 0 && state[0] + m <= cap;
}

__device__ inline void ae_side(const AeScratch& S, uint32_t i, uint32_t side, u128 pending,
                               u128 posted, uint32_t flip) {
    const uint32_t v = 2 * i + side;
    AeDelta d;
    d.pending = pending;
    d.posted = posted;
    d.flip = flip;
    d.side = side;
    d.pad = 0;
    S.deltas[v] = d;
}

// The event-level fields of AccountEvent `e` (the account halves are written by ae_emit).
__device__ inline void ae_event_fields(tb_account_event_t* e, uint64_t timestamp,
                                       uint16_t transfer_flags, uint8_t status,
                                       const tb_transfer_t* p, const tb_uint128_t& requested,
                                       const tb_uint128_t& amount, uint32_t ledger) {
    e->timestamp = timestamp;
    e->transfer_flags = transfer_flags;
    e->transfer_pending_flags = p ? p->flags : 0;
    e->transfer_pending_id = p ? p->id : tb_uint128_t{0, 0};
    e->amount_requested = requested;
    e->amount = amount;
    e->ledger = ledger;
    e->transfer_pending_status = status;
    for (int j = 0; j < 11; j++) e->reserved[j] = 0;
}

// A touch's half of its AccountEvent. The dr and cr halves share one layout (id and four
// balances: five 16-byte words, then the account timestamp and flags): one side's pointers,
// 16-byte stores (no struct copies, which the compiler stages through scratch).
__device__ inline uint4 ae_q(u128 x) {
    return make_uint4(uint32_t(uint64_t(x)), uint32_t(uint64_t(x) >> 32), uint32_t(uint64_t(x >> 64)),
                      uint32_t(uint64_t(x >> 64) >> 32));
}
__device__ inline u128 ae_u(uint4 v) {
    return (u128((uint64_t(v.w) << 32) | v.z) << 64) | ((uint64_t(v.y) << 32) | v.x);
}
__device__ inline uint4* ae_half_words(tb_account_event_t* log, uint32_t i, uint32_t side) {
    uint8_t* e = reinterpret_cast<uint8_t*>(&log[i]);
    return reinterpret_cast<uint4*>(e + (side ? offsetof(tb_account_event_t, cr_account_id)
                                              : offsetof(tb_account_event_t, dr_account_id)));
}
__device__ inline uint16_t* ae_half_flags(tb_account_event_t* log, uint32_t i, uint32_t side) {
    uint8_t* e = reinterpret_cast<uint8_t*>(&log[i]);
    return reinterpret_cast<uint16_t*>(e + (side ? offsetof(tb_account_event_t, cr_account_flags)
                                                 : offsetof(tb_account_event_t, dr_account_flags)));
}
__device__ inline uint64_t* ae_half_timestamp(tb_account_event_t* log, uint32_t i, uint32_t side) {
    uint8_t* e = reinterpret_cast<uint8_t*>(&log[i]);
    return reinterpret_cast<uint64_t*>(e + (side ? offsetof(tb_account_event_t, cr_account_timestamp)
                                                 : offsetof(tb_account_event_t, dr_account_timestamp)));
}

// An account's final state as a touch's half starts out (collection) -- also the snapshot's form.
struct AeFinal {
    uint4 id, dp, dpo, cp, cpo;
    uint64_t timestamp;
    uint32_t flags, pad;
};
static_assert(sizeof(AeFinal) == 96, "AeFinal layout");
__device__ inline AeFinal ae_final_of(const tb_account_t& a) {
    AeFinal f;
    const uint4* w = reinterpret_cast<const uint4*>(&a);  // id, debits_pending .. credits_posted
    f.id = w[0];
    f.dp = w[1];
    f.dpo = w[2];
    f.cp = w[3];
    f.cpo = w[4];
    f.timestamp = a.timestamp;
    f.flags = a.flags;
    f.pad = 0;
    return f;
}
__device__ inline void ae_write_final(tb_account_event_t* log, uint32_t i, uint32_t side,
                                      const AeFinal& f) {
    uint4* w = ae_half_words(log, i, side);
    w[0] = f.id;
    w[1] = f.dp;
    w[2] = f.dpo;
    w[3] = f.cp;
    w[4] = f.cpo;
    *ae_half_timestamp(log, i, side) = f.timestamp;
    *ae_half_flags(log, i, side) = uint16_t(f.flags);
}

// A whole AccountEvent as 16 16-byte stores (its fields one by one were ~35 narrow scattered
// stores per record): both halves (an account's final state), the event's fields.
static_assert(offsetof(tb_account_event_t, timestamp) == 160 &&
                  offsetof(tb_account_event_t, cr_account_timestamp) == 176 &&
                  offsetof(tb_account_event_t, dr_account_flags) == 184 &&
                  offsetof(tb_account_event_t, transfer_pending_id) == 192 &&
                  offsetof(tb_account_event_t, amount_requested) == 208 &&
                  offsetof(tb_account_event_t, amount) == 224 &&
                  offsetof(tb_account_event_t, ledger) == 240 &&
                  offsetof(tb_account_event_t, transfer_pending_status) == 244,
              "AccountEvent layout");
__device__ inline uint4 ae_q128(const tb_uint128_t& x) {
    return make_uint4(uint32_t(x.lo), uint32_t(x.lo >> 32), uint32_t(x.hi), uint32_t(x.hi >> 32));
}
__device__ inline void ae_write_record(tb_account_event_t* e, const AeFinal& d, const AeFinal& r,
                                       uint64_t timestamp, uint16_t transfer_flags, uint8_t status,
                                       const tb_transfer_t* p, const tb_uint128_t& requested,
                                       const tb_uint128_t& amount, uint32_t ledger) {
    uint4* w = reinterpret_cast<uint4*>(e);
    w[0] = d.id;
    w[1] = d.dp;
    w[2] = d.dpo;
    w[3] = d.cp;
    w[4] = d.cpo;
    w[5] = r.id;
    w[6] = r.dp;
    w[7] = r.dpo;
    w[8] = r.cp;
    w[9] = r.cpo;
    w[10] = make_uint4(uint32_t(timestamp), uint32_t(timestamp >> 32), uint32_t(d.timestamp),
                       uint32_t(d.timestamp >> 32));
    const uint32_t pf = p ? p->flags : 0u;
    w[11] = make_uint4(uint32_t(r.timestamp), uint32_t(r.timestamp >> 32),
                       (d.flags & 0xFFFFu) | ((r.flags & 0xFFFFu) << 16),
                       uint32_t(transfer_flags) | (pf << 16));
    w[12] = p ? ae_q128(p->id) : make_uint4(0, 0, 0, 0);
    w[13] = ae_q128(requested);
    w[14] = ae_q128(amount);
    w[15] = make_uint4(ledger, uint32_t(status), 0, 0);
}

// One touch's half: the account after the event = its final state (written by the collection) -
// the sums of the account's later touches in the call.
__device__ inline void ae_emit_touch(uint32_t v, const Bal5& later, tb_account_event_t* log,
                                     const uint32_t* pos) {
    const uint32_t i = pos ? pos[v >> 1] : v >> 1, side = v & 1;
    uint4* w = ae_half_words(log, i, side);
    const uint4 dp = w[1], dpo = w[2], cp = w[3], cpo = w[4];
    uint16_t* fl = ae_half_flags(log, i, side);
    const uint16_t flags = *fl;
    w[1] = ae_q(ae_u(dp) - later.dp);
    w[2] = ae_q(ae_u(dpo) - later.dpo);
    w[3] = ae_q(ae_u(cp) - later.cp);
    w[4] = ae_q(ae_u(cpo) - later.cpo);
    if (later.flips & 1) *fl = uint16_t(flags ^ TB_ACCOUNT_CLOSED);
}

__device__ inline uint64_t ae_transfer_row(const Tables& T, const tb_uint128_t& id) {
    const tb_transfer_t* rows = T.tr_rows;
    const uint64_t s = probe_find(T.tr, id, [=](uint64_t r) { return rows[r].id; });
    if (s == kNone) return kNone;
    const uint64_t w = T.tr.slots[s];
    return (w & kOrphanBit) ? kNone : (w & kRefMask) - 1;
}

// Created events of a create_transfers call: list[i] = event index k (call order).
// The created events of a create_transfers call, in call order (one chained-scan launch).
struct SelectCreated {
    static constexpr bool kEmitAll = false;
    const tb_create_result_t* results;
    uint32_t* out;
    unsigned int* count;
    __device__ void load(uint64_t base, uint64_t n, uint32_t* c) const {
#pragma unroll
        for (uint32_t i = 0; i < kScanItems; i++)
            c[i] = base + i < n && results[base + i].status == TB_STATUS_CREATED;
    }
    __device__ void emit(uint64_t i, uint32_t p) const { out[p] = uint32_t(i); }
    __device__ void total(uint32_t t) const { *count = t; }
};

// (Both collectors run kPlanThreads lanes per workgroup and group the event's two touches by
// account row; lanes past the events write "no key" for their touches.)
// (counted by account in LDS first, one global probe and add per distinct account of the
// workgroup: group_key_publish)
using AeGroupBlock = GroupKeyBlockT<kPlanThreads, kPlanLdsSlots>;
__device__ inline void ae_group_touches(const AeScratch& S, AeGroupBlock& B, uint32_t i,
                                        bool active, uint32_t dr, uint32_t cr, uint32_t bound) {
    uint32_t e0 = kNone32, e1 = kNone32, r0 = 0, r1 = 0;
    if (active) {
        e0 = group_key_count(B, dr, &r0);
        e1 = group_key_count(B, cr, &r1);
    }
    group_key_publish(S.G, B);
    if (i >= bound) return;
    group_block_place(S.G, B, 2 * uint64_t(i), e0, r0);
    group_block_place(S.G, B, 2 * uint64_t(i) + 1, e1, r1);
}

// A created transfer's account rows as ingest left them, for an event that is not a post/void: its
// record (ev_dr / ev_cr) or, for a lean FAST event, its packed balance item (pair or key items;
// ~0 once tr_commit cleared it). kNone32: look the ids up (account_find: two hash probes an event
// -- config 2's AccountEvents under wide amounts spent ~3 ms a 10M-event call there).
__device__ inline void ae_known_rows(const Call<tb_transfer_t>& c, uint32_t k, uint8_t info,
                                     uint32_t* dr, uint32_t* cr) {
    *dr = *cr = kNone32;
    if (!(info & kInfoLean)) {
        if (c.ev_dr && c.ev_cr) {
            *dr = c.ev_dr[k];
            *cr = c.ev_cr[k];
        }
        return;
    }
    if (!c.bal_items) return;
    if (c.pair_shift) {
        const uint64_t x = c.bal_items[k];
        if (x == ~0ull) return;
        const uint64_t m = (1ull << c.pair_shift) - 1;
        *dr = uint32_t(x & m);
        *cr = uint32_t((x >> c.pair_shift) & m);
    } else {
        const uint64_t i0 = c.bal_items[2 * uint64_t(k)], i1 = c.bal_items[2 * uint64_t(k) + 1];
        if (i0 == ~0ull || i1 == ~0ull) return;
        const uint64_t km = (1ull << c.key_bits) - 1;
        *dr = uint32_t((i0 & km) >> 2);
        *cr = uint32_t((i1 & km) >> 2);
    }
}

// Both sides' deltas of created transfer t (p: its pending transfer, for a post/void); returns the
// event's TransferPendingStatus.
__device__ inline uint8_t ae_transfer_sides(const AeScratch& S, uint32_t i, const tb_transfer_t& t,
                                            const tb_transfer_t* p) {
    const uint16_t f = t.flags;
    const u128 amount = U(t.amount);
    uint8_t status = TB_PENDING_NONE;
    u128 d_pending = 0, d_posted = 0;
    uint32_t flip_dr = 0, flip_cr = 0;
    if (p) {
        d_pending = u128(0) - U(p->amount);
        if (f & TB_TRANSFER_POST_PENDING) {
            status = TB_PENDING_POSTED;
            d_posted = amount;
        } else {
            status = TB_PENDING_VOIDED;
            flip_dr = (p->flags & TB_TRANSFER_CLOSING_DEBIT) != 0;
            flip_cr = (p->flags & TB_TRANSFER_CLOSING_CREDIT) != 0;
        }
    } else if (f & TB_TRANSFER_PENDING) {
        status = TB_PENDING_PENDING;
        d_pending = amount;
        flip_dr = (f & TB_TRANSFER_CLOSING_DEBIT) != 0;
        flip_cr = (f & TB_TRANSFER_CLOSING_CREDIT) != 0;
    } else {
        d_posted = amount;
    }
    ae_side(S, i, 0, d_pending, d_posted, flip_dr);
    ae_side(S, i, 1, d_pending, d_posted, flip_cr);
    return status;
}

__device__ inline void ae_collect_transfer(Tables T, const Call<tb_transfer_t>& c, uint32_t k,
                                           uint32_t i, const AeScratch& S, tb_account_event_t* log,
                                           AeRef* refs, uint32_t* dr_out, uint32_t* cr_out) {
    const uint64_t row = c.row_base + k;
    const tb_transfer_t& t = T.tr_rows[row];  // the created transfer (amount actual, accounts)
    const uint16_t f = t.flags;
    // A created transfer that is not a post/void has the event's own accounts, whose rows the
    // ingest found (c.ev_dr / ev_cr, unless it packed them into balance items: kInfoLean); a
    // post/void's are the pending transfer's.
    const bool pv = (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) != 0;
    uint32_t edr = kNone32, ecr = kNone32;
    if (!pv) ae_known_rows(c, k, c.ev_info[k], &edr, &ecr);
    const uint64_t dr = edr != kNone32 ? uint64_t(edr) : account_find(T, t.debit_account_id);
    const uint64_t cr = ecr != kNone32 ? uint64_t(ecr) : account_find(T, t.credit_account_id);
    const tb_transfer_t* p =
        pv ? &T.tr_rows[ae_transfer_row(T, t.pending_id)] : nullptr;
    const uint8_t status = ae_transfer_sides(S, i, t, p);
    ae_write_record(&log[i], ae_final_of(T.acc_rows[dr]), ae_final_of(T.acc_rows[cr]), t.timestamp,
                    f, status, p, c.events[k].amount, t.amount, t.ledger);
    refs[i] = AeRef{uint32_t(row), uint32_t(dr), uint32_t(cr), 0};
    *dr_out = uint32_t(dr);
    *cr_out = uint32_t(cr);
}

__global__ void __launch_bounds__(kPlanThreads)
ae_collect_transfers(Tables T, Call<tb_transfer_t> c, const uint32_t* list,
                     const unsigned int* count, AeScratch S, tb_account_event_t* log, AeRef* refs) {
    __shared__ AeGroupBlock B;
    group_key_init(B);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) S.G.counts[1] = S.G.counts[2] = 0;  // listed accounts / chunks (ae_group_small)
    const bool room = ae_room(S.state, S.cap, *count);
    log += S.state[0];
    refs += S.state[0];
    if (!room && i == 0) S.state[3] = 1;
    const bool active = room && i < *count;
    uint32_t dr_row = 0, cr_row = 0;
    if (active) ae_collect_transfer(T, c, list[i], i, S, log, refs, &dr_row, &cr_row);
    ae_group_touches(S, B, i, active, dr_row, cr_row, c.n);
}

// ---- Small calls: the appends behind the next call --------------------------------------------
//
// A create_transfers call of at most kAeAsyncMax events hands its appends to a side stream
// (executor: ae_transfers_async). The staging pass runs on the call's stream (fused into its
// stage_out), before the next call can change anything: per created event k it writes the finished
// AccountEvent but for the later touches' sums -- event fields and both accounts' final state --
// its reference, both sides' deltas (touches 2k, 2k + 1) and a created flag. The side stream then
// numbers the created events (a chained scan), copies each record to its log position and groups
// the touches by account, and the emit passes subtract the later sums in place. It reads only
// the staging (and writes only the log), so the next call runs beside it.
constexpr uint32_t kAeAsyncMax = 8192;

struct AeStage {
    tb_account_event_t* rec;  // per event
    AeRef* ref;               // per event
    AeDelta* delta;           // per touch (2k + side)
    uint8_t* created;         // per event
    // [0] the epoch of the last call whose staging holds an event ae_small_emit cannot take;
    // [1] the epoch of the last call whose appends ae_small_emit made (the graph then skips)
    unsigned int* words;
};
// An event ae_small_emit takes: created single-phase (its deltas are posted balances only, no
// `closed` flip) with an amount below 2^19 (u32 sums over <= 8192 events cannot wrap).
constexpr uint64_t kAeSmallAmountMax = 1ull << 19;

struct AeSnapJob {
    Tables T;
    Call<tb_transfer_t> c;
    AeStage st;
    // Taken right after the call (before the host knows whether a replay follows): with a replay
    // pending (stats[0], set by tr_commit) nothing is final yet -- a replayed event's slot may still
    // read `created` from the speculation -- so the staging holds no created event (the side
    // stream's appends, already queued, find none) and the executor stages again after the replay.
    bool speculative;
    // Mapped pinned word: the call's epoch when an event needs the general appends (the host reads
    // it once the snapshot has completed and queues only the appends the staging needs), or null.
    unsigned long long* host_general;
};
__device__ inline void ae_snapshot_one(const AeSnapJob& J, uint32_t k) {
    const Tables& T = J.T;
    const Call<tb_transfer_t>& c = J.c;
    if (k >= c.n) {
        J.st.created[k] = 0;
        return;
    }
    // (the result, the row's flags and the event's account refs loaded together, before the
    // created test: one round trip before the account rows instead of three)
    const uint64_t row = c.row_base + k;
    const tb_transfer_t& t = T.tr_rows[row];
    const bool have_refs = c.ev_dr && c.ev_cr;
    const uint32_t status_k = c.results[k].status;
    const uint16_t f = t.flags;
    const uint32_t info = have_refs ? c.ev_info[k] : 0u;
    const uint32_t edr0 = have_refs ? c.ev_dr[k] : kNone32;
    const uint32_t ecr0 = have_refs ? c.ev_cr[k] : kNone32;
    const bool made = status_k == TB_STATUS_CREATED;
    J.st.created[k] = made;
    if (!made) return;
    const bool pv = (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) != 0;
    const bool refs_ok = !pv && have_refs && !(info & kInfoLean);
    const uint32_t edr = refs_ok ? edr0 : kNone32;
    const uint32_t ecr = refs_ok ? ecr0 : kNone32;
    const uint64_t dr = edr != kNone32 ? uint64_t(edr) : account_find(T, t.debit_account_id);
    const uint64_t cr = ecr != kNone32 ? uint64_t(ecr) : account_find(T, t.credit_account_id);
    const uint64_t pr = pv ? ae_transfer_row(T, t.pending_id) : kNone;
    if (dr == kNone || cr == kNone || (pv && pr == kNone)) {  // (never for a final result)
        J.st.created[k] = 0;
        return;
    }
    const tb_transfer_t* p = pv ? &T.tr_rows[pr] : nullptr;
    AeScratch D{};
    D.deltas = J.st.delta;
    const uint8_t status = ae_transfer_sides(D, k, t, p);
    if (status != TB_PENDING_NONE || t.amount.hi != 0 || t.amount.lo >= kAeSmallAmountMax) {
        J.st.words[0] = c.epoch;  // (ae_small_emit leaves this call to the general appends)
        if (J.host_general)
            __hip_atomic_store(J.host_general, (unsigned long long)c.epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
    tb_account_event_t* rec = J.st.rec;
    ae_write_record(&rec[k], ae_final_of(T.acc_rows[dr]), ae_final_of(T.acc_rows[cr]), t.timestamp,
                    f, status, p, c.events[k].amount, t.amount, t.ledger);
    J.st.ref[k] = AeRef{uint32_t(row), uint32_t(dr), uint32_t(cr), 0};
}

__global__ void ae_snapshot(AeSnapJob J) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= kAeAsyncMax) return;
    if (J.speculative && J.T.scalars->stats[0] != 0) J.st.created[k] = 0;
    else ae_snapshot_one(J, k);
}

// A pulse's expiries staged like a small call (ae_expiry_one's records, ae_collect_expiry's
// order and stamps): the first m of `rows` (m on device), expiry i stamped timestamp - m + i + 1.
// ae_small_emit takes a pulse whose expiries release pending amounts below 2^19 and close no
// account (else the general appends, words[0]).
struct AeExpirySnap {
    Tables T;
    const uint64_t* rows;
    const unsigned int* m_dev;
    uint64_t timestamp;
    AeStage st;
    uint32_t epoch;
    // Mapped pinned word: the epoch when an expiry needs the general appends (the host reads it
    // after the pulse's synchronisation and queues only the appends the pulse needs), or null.
    unsigned long long* host_general;
};
__global__ void ae_expiry_snapshot(AeExpirySnap J) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= kAeAsyncMax) return;
    const uint32_t m = *J.m_dev;
    J.st.created[i] = i < m;
    if (i >= m) return;
    const Tables& T = J.T;
    const uint64_t row = J.rows[i];
    const tb_transfer_t& p = T.tr_rows[row];
    const uint64_t dr = account_find(T, p.debit_account_id);
    const uint64_t cr = account_find(T, p.credit_account_id);
    const u128 d_pending = u128(0) - U(p.amount);
    const uint32_t fd = (p.flags & TB_TRANSFER_CLOSING_DEBIT) != 0;
    const uint32_t fc = (p.flags & TB_TRANSFER_CLOSING_CREDIT) != 0;
    AeScratch D{};
    D.deltas = J.st.delta;
    ae_side(D, i, 0, d_pending, 0, fd);
    ae_side(D, i, 1, d_pending, 0, fc);
    ae_write_record(&J.st.rec[i], ae_final_of(T.acc_rows[dr]), ae_final_of(T.acc_rows[cr]),
                    J.timestamp - m + i + 1, 0, TB_PENDING_EXPIRED, &p, tb_uint128_t{0, 0},
                    p.amount, p.ledger);
    J.st.ref[i] = AeRef{uint32_t(row), uint32_t(dr), uint32_t(cr), 0};
    if (fd || fc || p.amount.hi != 0 || p.amount.lo >= kAeSmallAmountMax) {
        J.st.words[0] = J.epoch;
        if (J.host_general)
            __hip_atomic_store(J.host_general, (unsigned long long)J.epoch, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// u8 flags -> pos[i] = the number of flagged items before i (flagged items only); the count.
struct PositionsOf8 {
    static constexpr bool kEmitAll = false;
    const uint8_t* flags;
    uint32_t* pos;
    unsigned int* count;
    __device__ void load(uint64_t base, uint64_t n, uint32_t* c) const {
        const uint4 v = *reinterpret_cast<const uint4*>(flags + base);  // (n: a multiple of 16)
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (uint32_t i = 0; i < kScanItems; i++) c[i] = ((w[i >> 2] >> (8 * (i & 3))) & 0xFF) != 0;
        (void)n;
    }
    __device__ void emit(uint64_t i, uint32_t p) const { pos[i] = p; }
    __device__ void total(uint32_t t) const { *count = t; }
};

// One lane per call event: a created event's record and reference to its log position, its
// touches (2k, 2k + 1) into the grouping.
__global__ void __launch_bounds__(kPlanThreads)
ae_copy_group(AeStage st, const uint32_t* pos, const unsigned int* m_dev, AeScratch S,
              tb_account_event_t* log, AeRef* refs) {
    __shared__ AeGroupBlock B;
    if (S.skip && *S.skip == S.skip_if) return;
    group_key_init(B);
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k == 0) S.G.counts[1] = S.G.counts[2] = 0;  // listed accounts / chunks (ae_group_small)
    const bool room = ae_room(S.state, S.cap, *m_dev);
    if (!room && k == 0) S.state[3] = 1;
    const uint64_t used = S.state[0];
    const bool active = room && k < kAeAsyncMax && st.created[k];
    uint32_t dr_row = 0, cr_row = 0;
    if (active) {
        const uint64_t i = used + pos[k];
        const uint4* src = reinterpret_cast<const uint4*>(&st.rec[k]);
        uint4* dst = reinterpret_cast<uint4*>(&log[i]);
#pragma unroll
        for (int w = 0; w < 16; w++) dst[w] = src[w];
        const AeRef r = st.ref[k];
        refs[i] = r;
        dr_row = r.dr_row;
        cr_row = r.cr_row;
    }
    ae_group_touches(S, B, k, active, dr_row, cr_row, kAeAsyncMax);
}

// Expiries of a pulse (execute_expire_pending_transfers :4540-4626): rows[i] in expiry order,
// event i stamped timestamp - m + i + 1 -- or stamps[i], a shard's expiries stamped by their
// positions in the pulse's expiry order across all shards.
__device__ inline void ae_expiry_one(Tables T, uint64_t row, uint32_t m, uint32_t i,
                                     uint64_t timestamp, const uint64_t* stamps, const AeScratch& S,
                                     tb_account_event_t* log, AeRef* refs, uint32_t* dr_out,
                                     uint32_t* cr_out) {
    const tb_transfer_t& p = T.tr_rows[row];
    const uint64_t dr = account_find(T, p.debit_account_id);
    const uint64_t cr = account_find(T, p.credit_account_id);
    const u128 d_pending = u128(0) - U(p.amount);
    ae_side(S, i, 0, d_pending, 0, (p.flags & TB_TRANSFER_CLOSING_DEBIT) != 0);
    ae_side(S, i, 1, d_pending, 0, (p.flags & TB_TRANSFER_CLOSING_CREDIT) != 0);
    ae_write_record(&log[i], ae_final_of(T.acc_rows[dr]), ae_final_of(T.acc_rows[cr]),
                    stamps ? stamps[i] : timestamp - m + i + 1, 0, TB_PENDING_EXPIRED, &p,
                    tb_uint128_t{0, 0}, p.amount, p.ledger);
    refs[i] = AeRef{uint32_t(row), uint32_t(dr), uint32_t(cr), 0};
    *dr_out = uint32_t(dr);
    *cr_out = uint32_t(cr);
}

__global__ void __launch_bounds__(kPlanThreads)
ae_collect_expiry(Tables T, const uint64_t* rows, uint32_t m_upper, const unsigned int* m_dev,
                  uint64_t timestamp, const uint64_t* stamps, AeScratch S, tb_account_event_t* log,
                  AeRef* refs) {
    const uint32_t m = m_dev ? *m_dev : m_upper;  // (the pulse's count, on device)
    __shared__ AeGroupBlock B;
    group_key_init(B);
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) S.G.counts[1] = S.G.counts[2] = 0;  // listed accounts / chunks (ae_group_small)
    const bool room = ae_room(S.state, S.cap, m);
    if (!room && i == 0) S.state[3] = 1;
    log += S.state[0];
    refs += S.state[0];
    const bool active = room && i < m;
    uint32_t dr_row = 0, cr_row = 0;
    if (active) ae_expiry_one(T, rows[i], m, i, timestamp, stamps, S, log, refs, &dr_row, &cr_row);
    ae_group_touches(S, B, i, active, dr_row, cr_row, m_upper);
}

// Closes an appended block: the log's length and last timestamp advance on device (the host reads
// them only when it needs them, ae_settle), and a block that starts at or before the previous
// last timestamp marks the log unsorted (get_change_events sorts it first).
__global__ void ae_tail(const tb_account_event_t* log, const unsigned int* d_count, uint32_t n,
                        unsigned long long* state) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint32_t m = d_count ? *d_count : n;
    if (m == 0 || state[3]) return;  // (an overflowed append wrote nothing)
    const uint64_t used = state[0];
    const uint64_t first = log[used].timestamp, last = log[used + m - 1].timestamp;
    if (used && first <= state[1]) state[2] = 1;
    state[1] = last > state[1] ? last : state[1];
    state[0] = used + m;
}


// Listed accounts are processed in chunks of kAeChunk touches (kAeRun per lane of a workgroup).
constexpr uint32_t kAeRun = 4;
constexpr uint32_t kAeChunk = kGroupBigThreads * kAeRun;
constexpr uint32_t kAeChunkBlocks = 512;  // ae_chunk_totals / ae_chunk_emit grid (grid-stride)

// Per grouped account: <= kGroupSmall touches in registers (sorted, then emitted last to first with
// the running sums); larger groups are listed for ae_group_sort / ae_chunk_*. Clears the slot.
// A wave-sorted account (kGroupSmall < c <= kGroupMid touches in buf, event order): lane l takes
// positions 4l .. 4l + 3; the later sums of its run = a suffix scan over the lanes after it.
__device__ inline u128 wave_suffix_exclusive_u128(u128 x) {
    const uint32_t lane = threadIdx.x & 63;
    u128 f = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t lo = __shfl_down(uint64_t(f), d, 64), hi = __shfl_down(uint64_t(f >> 64), d, 64);
        if (lane + d < 64) f += (u128(hi) << 64) | lo;
    }
    return f - x;
}
__device__ inline void ae_mid_account(Tables T, const AeScratch& S, uint32_t off, uint32_t c,
                                      uint32_t row, uint32_t* buf, tb_account_event_t* log) {
    const uint32_t lane = threadIdx.x & 63;
    wave_rank_sort(S.G.vals, off, c, buf);
    uint32_t v[4];
    Bal5 run{};
#pragma unroll
    for (uint32_t j = 0; j < 4; j++) {
        v[j] = 4 * lane + j < c ? buf[4 * lane + j] : kNone32;
        if (v[j] != kNone32) bal5_add(run, S.deltas[v[j]]);
    }
    Bal5 later;
    later.dp = wave_suffix_exclusive_u128(run.dp);
    later.dpo = wave_suffix_exclusive_u128(run.dpo);
    later.cp = wave_suffix_exclusive_u128(run.cp);
    later.cpo = wave_suffix_exclusive_u128(run.cpo);
    later.flips = uint32_t(wave_suffix_exclusive_u128(run.flips));
    (void)T;
    (void)row;
#pragma unroll
    for (int j = 3; j >= 0; j--) {
        if (v[j] == kNone32) continue;
        ae_emit_touch(v[j], later, log, S.pos);
        bal5_add(later, S.deltas[v[j]]);
    }
    wave_lds_sync();  // (buf is reused by the wave's next account)
}

// Per grouped account: <= kGroupSmall touches in registers (sorted, then emitted last to first with
// the running sums), <= kGroupMid by the slot's wave (ae_mid_account); larger ones are listed for
// ae_group_sort / ae_chunk_*. Clears the slot.
__global__ void __launch_bounds__(kBlock) ae_group_small(Tables T, AeScratch S, uint64_t slots,
                                                         tb_account_event_t* log) {
    __shared__ uint32_t wave_buf[kBlock / 64][kGroupMid];
    if (S.skip && *S.skip == S.skip_if) return;
    const GroupPlan& G = S.G;
    log += S.state[0];
    const uint64_t h = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    uint32_t c = 0, off = 0, row = 0;
    if (h < slots) {
        c = G.hcnt[h];
        if (c) {
            row = uint32_t(G.hkeys[h] - 1);
            off = G.hoff[h];
            G.hkeys[h] = 0;
            G.hcnt[h] = 0;
        }
    }
    if (c > kGroupMid) {
        const uint32_t b = atomicAdd(&G.counts[1], 1u);
        const uint32_t chunks = (c + kAeChunk - 1) / kAeChunk;
        const uint32_t cb = atomicAdd(&G.counts[2], chunks);
        G.big[b] = make_uint4(off, c, row, cb);
        for (uint32_t q = 0; q < chunks; q++) S.chunk_seg[cb + q] = b;
    } else if (c >= 1 && c <= kGroupSmall) {
        uint32_t v[kGroupSmall];
#pragma unroll
        for (uint32_t i = 0; i < kGroupSmall; i++) v[i] = i < c ? G.vals[off + i] : kNone32;
        sort_network(v);
        Bal5 later{};
#pragma unroll
        for (int i = kGroupSmall - 1; i >= 0; i--) {
            if (uint32_t(i) >= c) continue;
            ae_emit_touch(v[i], later, log, S.pos);
            bal5_add(later, S.deltas[v[i]]);
        }
    }
    uint64_t mids = __ballot(c > kGroupSmall && c <= kGroupMid);
    while (mids) {
        const int l = __ffsll((unsigned long long)mids) - 1;
        mids &= mids - 1;
        ae_mid_account(T, S, __shfl(off, l, 64), __shfl(c, l, 64), __shfl(row, l, 64),
                       wave_buf[threadIdx.x >> 6], log);
    }
}

// Sums across a workgroup of kGroupBigThreads: exclusive prefix over lanes (in lane order) and
// the total, one u128 at a time (a Bal5 is five of them: registers stay low).
struct Bal5Lds {
    unsigned long long w[kGroupBigThreads / 64][2];
};
__device__ inline u128 block_exclusive_u128(u128 x, u128* total, Bal5Lds& L) {
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u128 f = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint64_t lo = __shfl_up(uint64_t(f), d, 64), hi = __shfl_up(uint64_t(f >> 64), d, 64);
        if (lane >= uint32_t(d)) f += (u128(hi) << 64) | lo;
    }
    if (lane == 63) {
        L.w[wave][0] = uint64_t(f);
        L.w[wave][1] = uint64_t(f >> 64);
    }
    __syncthreads();
    u128 before = 0, all = 0;
    for (uint32_t w = 0; w < kGroupBigThreads / 64; w++) {
        const u128 t = (u128(L.w[w][1]) << 64) | L.w[w][0];
        if (w < wave) before += t;
        all += t;
    }
    __syncthreads();
    *total = all;
    return before + f - x;
}
__device__ inline Bal5 bal5_block_exclusive(const Bal5& x, Bal5* total, Bal5Lds& L) {
    Bal5 r;
    r.dp = block_exclusive_u128(x.dp, &total->dp, L);
    r.dpo = block_exclusive_u128(x.dpo, &total->dpo, L);
    r.cp = block_exclusive_u128(x.cp, &total->cp, L);
    r.cpo = block_exclusive_u128(x.cpo, &total->cpo, L);
    u128 tf;
    r.flips = uint32_t(block_exclusive_u128(x.flips, &tf, L));
    total->flips = uint32_t(tf);
    return r;
}

// A segment of at most kWaveSortMax values sorted by one wave: an LDS bitonic sort of the next
// power of two (kNone32 padding) with wave-level barriers only. All lanes of the wave call it.
constexpr uint32_t kWaveSortMax = 2048;
__device__ inline void wave_bitonic_sort(const uint32_t* in, uint32_t* out, uint32_t off, uint32_t c,
                                         uint32_t* buf) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t pw = 64;
    while (pw < c) pw <<= 1;
    for (uint32_t i = lane; i < pw; i += 64) buf[i] = i < c ? in[off + i] : kNone32;
    wave_lds_sync();
    // (each stage's reads all issue before any compare: one LDS round trip per stage)
    constexpr uint32_t kPer = kWaveSortMax / 128;
    const uint32_t pairs = pw / 2;
    for (uint32_t size = 2; size <= pw; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            uint32_t xs[kPer], ys[kPer];
#pragma unroll
            for (uint32_t j = 0; j < kPer; j++) {
                const uint32_t t = lane + 64 * j;
                const uint32_t a = 2 * t - (t & (stride - 1)), b = a + stride;
                if (t < pairs) {
                    xs[j] = buf[a];
                    ys[j] = buf[b];
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < kPer; j++) {
                const uint32_t t = lane + 64 * j;
                const uint32_t a = 2 * t - (t & (stride - 1)), b = a + stride;
                if (t < pairs && (xs[j] > ys[j]) == ((a & size) == 0)) {
                    buf[a] = ys[j];
                    buf[b] = xs[j];
                }
            }
            wave_lds_sync();
        }
    }
    for (uint32_t i = lane; i < c; i += 64) out[off + i] = buf[i];
    wave_lds_sync();  // (buf is reused by the wave's next segment)
}

// Listed accounts: the touches in event order into vals_sorted -- an account of at most
// kWaveSortMax touches by one wave (the workgroup's eight waves sort eight of them at once), a
// larger one by the whole workgroup (segment_sort). (One workgroup per account sorted config 2's
// 10k accounts of ~2,000 touches forty at a time per CU: 2.4 ms per 10M-event step.)
__global__ void __launch_bounds__(kGroupBigThreads) ae_group_sort(AeScratch S) {
    __shared__ SegmentLds L;
    static_assert(kGroupBigThreads / 64 * kWaveSortMax <= kGroupLdsWords, "wave sort slices");
    const GroupPlan& G = S.G;
    const uint32_t nbig = G.counts[1];
    const uint32_t wave = threadIdx.x >> 6, waves = kGroupBigThreads / 64;
    // (only when there are many more accounts than workgroups: with a few hundred, one workgroup
    // each finishes sooner -- the large ones would wait behind the waves' share)
    const bool by_waves = nbig > 4 * gridDim.x;
    uint32_t* slice = L.buf + wave * kWaveSortMax;
    for (uint32_t b = blockIdx.x * waves + wave; by_waves && b < nbig; b += gridDim.x * waves) {
        const uint4 e = G.big[b];
        if (e.y <= kWaveSortMax) wave_bitonic_sort(G.vals, G.vals_sorted, e.x, e.y, slice);
    }
    __syncthreads();
    for (uint32_t b = blockIdx.x; b < nbig; b += gridDim.x) {
        const uint4 e = G.big[b];
        if (!by_waves || e.y > kWaveSortMax) segment_sort(G.vals, G.vals_sorted, e.x, e.y, L);
    }
}

// Chunk q of a listed account holds the touches at positions (from the account's last touch
// backwards) [q * kAeChunk, (q + 1) * kAeChunk); lane t the kAeRun of them from q * kAeChunk +
// t * kAeRun. Loads the lane's run and returns its sums.
__device__ inline Bal5 ae_chunk_run(const AeScratch& S, const uint4& e, uint32_t q,
                                    uint32_t (&v)[kAeRun]) {
    const uint32_t off = e.x, c = e.y;
    const uint32_t r0 = q * kAeChunk + threadIdx.x * kAeRun;
    Bal5 run{};
#pragma unroll
    for (uint32_t j = 0; j < kAeRun; j++)
        v[j] = r0 + j < c ? S.G.vals_sorted[off + c - 1 - (r0 + j)] : kNone32;
#pragma unroll
    for (uint32_t j = 0; j < kAeRun; j++)
        if (v[j] != kNone32) bal5_add(run, S.deltas[v[j]]);
    return run;
}

// Every chunk's sums (one workgroup per chunk, grid-stride).
__global__ void __launch_bounds__(kGroupBigThreads) ae_chunk_totals(AeScratch S) {
    __shared__ Bal5Lds B;
    const GroupPlan& G = S.G;
    const uint32_t nchunks = G.counts[2];
    for (uint32_t g = blockIdx.x; g < nchunks; g += gridDim.x) {
        const uint32_t b = S.chunk_seg[g];
        const uint4 e = G.big[b];
        uint32_t v[kAeRun];
        const Bal5 run = ae_chunk_run(S, e, g - e.w, v);
        Bal5 total;
        (void)bal5_block_exclusive(run, &total, B);
        if (threadIdx.x == 0) S.chunk_tot[g] = total;
    }
}

// Every chunk's touches emitted: later sums = the totals of the account's chunks before this one
// (chunk 0 holds its last touches; summed by the first wave) + the lanes before in the chunk + the
// run's touches after.
__global__ void __launch_bounds__(kGroupBigThreads) ae_chunk_emit(Tables T, AeScratch S,
                                                                 tb_account_event_t* log) {
    __shared__ Bal5Lds B;
    __shared__ Bal5 carry_lds;
    const GroupPlan& G = S.G;
    log += S.state[0];
    const uint32_t nchunks = G.counts[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    for (uint32_t g = blockIdx.x; g < nchunks; g += gridDim.x) {
        const uint32_t b = S.chunk_seg[g];
        const uint4 e = G.big[b];
        const uint32_t q = g - e.w;
        if (tid < 64) {  // chunks 0 .. q - 1 (the later touches): lanes sum, the wave reduces
            u128 f[4] = {0, 0, 0, 0};
            uint32_t fl = 0;
            for (uint32_t j = lane; j < q; j += 64) {
                const Bal5 t = S.chunk_tot[e.w + j];
                f[0] += t.dp;
                f[1] += t.dpo;
                f[2] += t.cp;
                f[3] += t.cpo;
                fl += t.flips;
            }
#pragma unroll
            for (int d = 32; d >= 1; d >>= 1) {
#pragma unroll
                for (int x = 0; x < 4; x++) {
                    const uint64_t lo = __shfl_xor(uint64_t(f[x]), d, 64);
                    const uint64_t hi = __shfl_xor(uint64_t(f[x] >> 64), d, 64);
                    f[x] += (u128(hi) << 64) | lo;
                }
                fl += __shfl_xor(fl, d, 64);
            }
            if (lane == 0) {
                carry_lds.dp = f[0];
                carry_lds.dpo = f[1];
                carry_lds.cp = f[2];
                carry_lds.cpo = f[3];
                carry_lds.flips = fl;
            }
        }
        uint32_t v[kAeRun];
        const Bal5 run = ae_chunk_run(S, e, q, v);
        Bal5 chunk;
        Bal5 later = bal5_block_exclusive(run, &chunk, B);  // (its barriers publish carry_lds)
        later.dp += carry_lds.dp;
        later.dpo += carry_lds.dpo;
        later.cp += carry_lds.cp;
        later.cpo += carry_lds.cpo;
        later.flips += carry_lds.flips;
        (void)T;
        for (uint32_t j = 0; j < kAeRun; j++) {
            if (v[j] == kNone32) break;
            ae_emit_touch(v[j], later, log, S.pos);
            bal5_add(later, S.deltas[v[j]]);
        }
        __syncthreads();  // (carry_lds is rewritten by the next chunk)
    }
}

// ---- The side stream's graph (small calls) ---------------------------------------------------

// group_scatter + the log's tail (ae_tail) + the graph's scan words cleared for its next replay.
// The block's base position in the log is kept at base[0] for the emit kernels that follow (the
// tail advances the log's length first).
__global__ void ae_scatter_tail(GroupPlan G, uint64_t pairs, const tb_account_event_t* log,
                                const unsigned int* d_count, unsigned long long* state,
                                unsigned long long* base, unsigned long long* scan_words,
                                uint32_t n_scan_words, const unsigned int* skip, uint32_t skip_if) {
    if (skip && *skip == skip_if) return;
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (blockIdx.x == 0) {
        for (uint32_t w = threadIdx.x; w < n_scan_words; w += blockDim.x) scan_words[w] = 0;
        if (threadIdx.x == 0) {
            const uint32_t m = *d_count;
            const uint64_t used = state[0];
            base[0] = used;
            if (m && !state[3]) {
                const uint64_t first = log[used].timestamp, last = log[used + m - 1].timestamp;
                if (used && first <= state[1]) state[2] = 1;
                state[1] = last > state[1] ? last : state[1];
                state[0] = used + m;
            }
        }
    }
    if (i >= pairs) return;
    const uint32_t slot = G.loc[i];
    if (slot == kNone32) return;
    G.vals[G.hoff[slot] + G.rank[i]] = uint32_t(i);
}

// Listed accounts of a small call, one workgroup each from sort to emission: the touches in event
// order (segment_sort), then the chunks from the last touch backwards with the later chunks' sums
// carried in registers (ae_group_sort + ae_chunk_totals + ae_chunk_emit in one launch; a small
// call's listed accounts hold at most 2 * kAeAsyncMax touches between them).
__global__ void __launch_bounds__(kGroupBigThreads) ae_group_big_serial(AeScratch S,
                                                                      tb_account_event_t* log) {
    __shared__ SegmentLds L;
    __shared__ Bal5Lds B;
    if (S.skip && *S.skip == S.skip_if) return;
    const GroupPlan& G = S.G;
    log += S.state[0];
    const uint32_t nbig = G.counts[1];
    for (uint32_t b = blockIdx.x; b < nbig; b += gridDim.x) {
        const uint4 e = G.big[b];
        segment_sort(G.vals, G.vals_sorted, e.x, e.y, L);
        const uint32_t chunks = (e.y + kAeChunk - 1) / kAeChunk;
        Bal5 carry{};
        for (uint32_t q = 0; q < chunks; q++) {
            uint32_t v[kAeRun];
            const Bal5 run = ae_chunk_run(S, e, q, v);
            Bal5 chunk;
            Bal5 later = bal5_block_exclusive(run, &chunk, B);
            later.dp += carry.dp;
            later.dpo += carry.dpo;
            later.cp += carry.cp;
            later.cpo += carry.cpo;
            later.flips += carry.flips;
            for (uint32_t j = 0; j < kAeRun; j++) {
                if (v[j] == kNone32) break;
                ae_emit_touch(v[j], later, log, S.pos);
                bal5_add(later, S.deltas[v[j]]);
            }
            carry.dp += chunk.dp;
            carry.dpo += chunk.dpo;
            carry.cp += chunk.cp;
            carry.cpo += chunk.cpo;
            carry.flips += chunk.flips;
        }
        __syncthreads();  // (L is reused by the next listed account)
    }
}

// ---- AccountEvents of balance-window calls in one pass ------------------------------------------
//
// A create_transfers call on the balance window path (kernels.hpp: pair items, <= 2^14 accounts)
// whose created events are all plain single-phase FAST events -- no replay, no linked chain,
// post/void or imported event, no pending transfer, every amount packed in its item (no
// kFlagChain / kFlagPostVoid / kFlagImported / kFlagAeSlow) and every window sum below 2^32 (no
// kFlagWideSums) -- changes nothing of an account but its posted balances, each created event by
// its item's amount. The AccountEvent of created event e (account_event :4384-4465) then carries,
// for each of its accounts A,
//     A's posted balances after e = A's final posted balances - A's deltas of the events after e
// and A's final row for everything else (pending balances, `closed`, timestamp, id). The later
// deltas come from the window's per-workgroup partial sums: ae_window_suffix turns them into
// suffix sums over the slices (partials[w][key] = the key's deltas in slices w, w + 1, ...), and
// ae_window_emit walks slice w (bal_window_accumulate's) in rounds of 1024 events with the slice's
// suffix sums in LDS, one u32 per account and side (R). Within a round the later deltas of event
// e on account A are R[A] minus A's deltas of the round's events up to and including e: every
// touch pushes itself on its account's LDS list (an exchange of the list head; a node is an event
// and a side) and e walks both of its accounts' lists, summing the nodes of events <= e (config 2
// puts ~0.2 touches on an account per round: the lists are short). After the round R drops by the
// round's deltas. Each record is written once, as 16 non-temporal 16-byte stores; no grouping,
// sorting or returning global atomics. The records' positions: the slices' created counts (from
// bal_window_accumulate) and a ballot scan per round. The final account rows are L2-resident at
// these key spaces; an event's timestamp is its result's.
constexpr uint32_t kAeWinThreads = 1024;
constexpr uint32_t kAeWinRowsMax = 12288;  // 12 B of LDS per account (R debit, R credit, list head)
constexpr uint32_t kAeWinNil = 0xFFFFFFFFu;

struct AeWindow {
    const uint64_t* items;               // the call's pair items (~0: none)
    const tb_create_result_t* results;
    const tb_account_t* acc_rows;
    uint32_t n, ps, rows, nwg, wkeys;
    uint64_t row_base;
    uint32_t* suffix;                    // the window partials, [workgroup][key]: suffix sums
    const unsigned int* slice_count;     // per workgroup: its slice's created events
    unsigned long long* slice_ts;        // per workgroup: its first and last created timestamp
    unsigned int* done;                  // finished workgroups (the last one closes the block)
    tb_account_event_t* log;
    AeRef* refs;
    unsigned long long* state;           // the log on device (AeScratch::state)
    uint64_t cap;
};

// One lane per (account, side) key in use: partials[w][key] = sum over w' >= w (in place).
__global__ void ae_window_suffix(AeWindow W) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 2 * W.rows) return;
    const uint32_t key = t < W.rows ? t : ((1u << W.ps) | (t - W.rows));
    uint32_t* p = W.suffix + key;
    const uint64_t stride = W.wkeys;
    uint32_t s = 0;
    int64_t w = int64_t(W.nwg) - 1;
    for (; w >= 7; w -= 8) {  // (eight loads in flight)
        uint32_t v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = p[uint64_t(w - j) * stride];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            s += v[j];
            p[uint64_t(w - j) * stride] = s;
        }
    }
    for (; w >= 0; w--) {
        s += p[uint64_t(w) * stride];
        p[uint64_t(w) * stride] = s;
    }
}

__device__ inline void ae_nt_store(uint4* p, uint4 v) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u x = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(x, reinterpret_cast<v4u*>(p));
}
__device__ inline uint4 ae_sub_u32(uint4 balance, uint32_t d) {
    return ae_q(ae_u(balance) - u128(d));
}

// Record groups whose loads issue together in the emits: every row / staged word load of a batch
// goes out before its stores (the compiler cannot tell the log from the rows it reads, so one group
// at a time paid a full load latency per four records). (ae_window_emit / ae_wide_emit, 1024 lanes
// at most 128 registers each, keep their loop over the batches rolled: ae_window_emit 722 -> 683 us
// per 10M events.)
#ifndef TBG_AE_REC_BATCH
#define TBG_AE_REC_BATCH 4
#endif
constexpr uint32_t kAeRecBatch = TBG_AE_REC_BATCH;

// The end of a one-pass emit's workgroup (slice w; every thread calls it): the slice's first and
// last created timestamps (ts_lds: LDS words set to ~0 / 0 before a barrier); the last workgroup to
// finish closes the block -- the log's length, its last timestamp and whether the block broke the
// log's timestamp order.
__device__ inline void ae_slices_close(uint64_t ts_min, uint64_t ts_max, unsigned long long* ts_lds,
                                       unsigned long long* slice_ts, const unsigned int* slice_count,
                                       unsigned int* done, unsigned long long* state, uint64_t used,
                                       uint32_t w) {
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t a = __shfl_xor(ts_min, off), b = __shfl_xor(ts_max, off);
        ts_min = a < ts_min ? a : ts_min;
        ts_max = b > ts_max ? b : ts_max;
    }
    if ((threadIdx.x & 63) == 0) {
        atomicMin(&ts_lds[0], ts_min);
        atomicMax(&ts_lds[1], ts_max);
    }
    __syncthreads();
    if (threadIdx.x != 0) return;
    slice_ts[2 * w] = ts_lds[0];
    slice_ts[2 * w + 1] = ts_lds[1];
    __threadfence();
    if (atomicAdd(done, 1u) != gridDim.x - 1) return;
    __threadfence();
    uint64_t total = 0, first = 0, last = 0;
    bool any = false;
    const volatile unsigned int* counts = slice_count;  // (other workgroups' words: no cached copy)
    const volatile unsigned long long* sts = slice_ts;
    for (uint32_t j = 0; j < gridDim.x; j++) {
        const uint32_t cj = counts[j];
        if (!cj) continue;
        const uint64_t f = sts[2 * j], l = sts[2 * j + 1];
        if (!any) first = f;
        any = true;
        last = l;
        total += cj;
    }
    if (total) {
        if (used && first <= state[1]) state[2] = 1;
        if (last > state[1]) state[1] = last;
        state[0] = used + total;
    }
    *done = 0;
}

__global__ void __launch_bounds__(kAeWinThreads) ae_window_emit(AeWindow W) {
    __shared__ uint32_t Rd[kAeWinRowsMax];    // debits_posted deltas of the events from the round on
    __shared__ uint32_t Rc[kAeWinRowsMax];    // credits_posted
    __shared__ uint32_t head[kAeWinRowsMax];  // the round's touch lists (node 2e + side)
    __shared__ uint16_t next[2 * kAeWinThreads];
    __shared__ uint32_t amt[kAeWinThreads];
    __shared__ uint32_t wave_cnt[kAeWinThreads / 64];
    __shared__ unsigned long long ts_lds[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, w = blockIdx.x;
    const uint32_t per = window_slice_per(W.n, W.nwg);
    const uint32_t b0 = w * per;
    const uint32_t b1 = b0 + per < W.n ? b0 + per : W.n;
    // created events of the earlier slices; of all (the room in the log: else nothing is written)
    uint32_t before = 0, all = 0;
    for (uint32_t j = tid; j < W.nwg; j += kAeWinThreads) {
        before += j < w ? W.slice_count[j] : 0;
        all += W.slice_count[j];
    }
    for (int off = 32; off > 0; off >>= 1) {
        before += __shfl_xor(before, off);
        all += __shfl_xor(all, off);
    }
    if (!__syncthreads_and(ae_room(W.state, W.cap, all))) {
        if (tid == 0) W.state[3] = 1;
        return;
    }
    if (lane == 0) wave_cnt[wv] = before;
    const uint32_t* suf = W.suffix + uint64_t(w) * W.wkeys;
    for (uint32_t a = tid; a < W.rows; a += kAeWinThreads) {
        Rd[a] = suf[a];
        Rc[a] = suf[(1u << W.ps) + a];
        head[a] = kAeWinNil;
    }
    if (tid == 0) {
        ts_lds[0] = ~0ull;
        ts_lds[1] = 0;
    }
    const uint64_t used = W.state[0];
    __syncthreads();
    uint64_t pos = used;
    for (uint32_t j = 0; j < kAeWinThreads / 64; j++) pos += wave_cnt[j];
    __syncthreads();
    const uint32_t ps = W.ps;
    const uint64_t rmask = (1ull << ps) - 1;
    uint64_t ts_min = ~0ull, ts_max = 0;
    for (uint32_t r0 = b0; r0 < b1; r0 += kAeWinThreads) {
        const uint32_t e = r0 + tid;
        const uint64_t x = e < b1 ? W.items[e] : ~0ull;
        const bool valid = x != ~0ull;
        uint32_t dr = 0, cr = 0, a = 0;
        uint64_t ts = 0;
        if (valid) {
            dr = uint32_t(x & rmask);
            cr = uint32_t((x >> ps) & rmask);
            a = uint32_t(x >> (2 * ps + 1));  // (< 2^32: no kFlagWideSums)
            ts = W.results[e].timestamp;
            next[2 * tid] = uint16_t(atomicExch(&head[dr], 2 * tid));
            next[2 * tid + 1] = uint16_t(atomicExch(&head[cr], 2 * tid + 1));
            amt[tid] = a;
        }
        const uint64_t bal = __ballot(valid);
        if (lane == 0) wave_cnt[wv] = uint32_t(__popcll(bal));
        __syncthreads();
        uint64_t wave_pos = pos;  // the wave's first record
        uint32_t round_total = 0;
        for (uint32_t j = 0; j < kAeWinThreads / 64; j++) {
            const uint32_t cj = wave_cnt[j];
            wave_pos += j < wv ? cj : 0;
            round_total += cj;
        }
        // later deltas: [0] the debit account's debits_posted, [1] its credits_posted, [2] / [3]
        // the credit account's
        uint32_t later[4] = {0, 0, 0, 0};
        if (valid) {
#pragma unroll
            for (int side = 0; side < 2; side++) {
                const uint32_t acc = side ? cr : dr;
                uint32_t sd = 0, sc = 0;
                for (uint32_t nd = head[acc]; nd != kAeWinNil;) {
                    if ((nd >> 1) <= tid) {
                        const uint32_t v = amt[nd >> 1];
                        if (nd & 1) sc += v;
                        else sd += v;
                    }
                    const uint32_t nx = next[nd];
                    nd = nx == 0xFFFFu ? kAeWinNil : nx;
                }
                later[2 * side] = Rd[acc] - sd;
                later[2 * side + 1] = Rc[acc] - sc;
            }
        }
        __syncthreads();  // (every list walked and R read before the round's updates)
        if (valid) {
            head[dr] = kAeWinNil;
            head[cr] = kAeWinNil;
            atomicSub(&Rd[dr], a);
            atomicSub(&Rc[cr], a);
            ts_min = ts < ts_min ? ts : ts_min;
            ts_max = ts > ts_max ? ts : ts_max;
            const uint32_t rank = lane ? __popcll(bal & (~0ull >> (64 - lane))) : 0;
            ae_nt_store(reinterpret_cast<uint4*>(&W.refs[wave_pos + rank]),
                        make_uint4(uint32_t(W.row_base + e), dr, cr, 0));
        }
        // The wave's records, four at a time (one 1 KB store per instruction when the four are
        // consecutive): lane L writes word L % 16 of the record of event lane 4 j + L / 16,
        // loading the one row word it needs (L2) and the event lane's values by lane shuffles.
        //   words 0-4 / 5-9: the debit / credit account's id and balances (posted ones less the
        //   later deltas); 10: timestamps; 11: the credit account's timestamp and both flags;
        //   12: pending id (0); 13, 14: amount requested and amount; 15: ledger, status (none).
        const uint32_t wd = lane & 15, sub = lane >> 4;
        const bool credit_half = (wd >= 5 && wd < 10) || wd == 11;
        const uint32_t k = wd < 5 ? wd : wd < 10 ? wd - 5 : 7;
        // (kAeRecBatch groups' row loads issued together; the loop over the batches not
        // unrolled -- unrolled, the loads of all 16 groups are hoisted and spill)
#pragma unroll 1
        for (uint32_t j0 = 0; j0 < 16; j0 += kAeRecBatch) {
            if (((bal >> (4 * j0)) & 0xFFFFull) == 0) continue;
            uint4 qb[kAeRecBatch];
#pragma unroll
            for (uint32_t b = 0; b < kAeRecBatch; b++) {
                const uint32_t src = 4 * (j0 + b) + sub;
                const uint32_t s_dr = __shfl(dr, src), s_cr = __shfl(cr, src);
                qb[b] = make_uint4(0, 0, 0, 0);
                if ((bal >> src) & 1) qb[b] = reinterpret_cast<const uint4*>(&W.acc_rows[credit_half ? s_cr : s_dr])[k];
            }
#pragma unroll
            for (uint32_t b = 0; b < kAeRecBatch; b++) {
                const uint32_t j = j0 + b;
                const uint32_t src = 4 * j + sub;
                const uint32_t s_a = __shfl(a, src);
                const uint32_t l0 = __shfl(later[0], src), l1 = __shfl(later[1], src);
                const uint32_t l2 = __shfl(later[2], src), l3 = __shfl(later[3], src);
                const uint32_t l_dpo = credit_half ? l2 : l0, l_cpo = credit_half ? l3 : l1;
                const uint32_t ts_lo = __shfl(uint32_t(ts), src), ts_hi = __shfl(uint32_t(ts >> 32), src);
                const bool v = (bal >> src) & 1;
                const uint4 q = qb[b];
                const uint32_t dflags = __shfl(q.y, lane > 0 ? lane - 1 : 0);
                if (!v) continue;
                uint4 o = q;
                if (k == 2) o = ae_sub_u32(q, l_dpo);
                else if (k == 4) o = ae_sub_u32(q, l_cpo);
                else if (wd == 10) o = make_uint4(ts_lo, ts_hi, q.z, q.w);
                else if (wd == 11) o = make_uint4(q.z, q.w, (dflags >> 16) | (q.y & 0xFFFF0000u), 0u);
                else if (wd == 12) o = make_uint4(0, 0, 0, 0);
                else if (wd == 13 || wd == 14) o = make_uint4(s_a, 0, 0, 0);
                else if (wd == 15) o = make_uint4(q.x, uint32_t(TB_PENDING_NONE), 0, 0);
                const uint64_t at = wave_pos + uint64_t(__popcll(bal & ((1ull << src) - 1)));
                ae_nt_store(reinterpret_cast<uint4*>(&W.log[at]) + wd, o);
            }
        }
        pos += round_total;
        __syncthreads();  // (the lists are empty and R is current for the next round)
    }
    ae_slices_close(ts_min, ts_max, ts_lds, W.slice_ts, W.slice_count, W.done, W.state, used, w);
}

// ---- AccountEvents of window calls with wide amounts -----------------------------------------
//
// A balance-window call whose created events are all plain single-phase FAST events (as for
// ae_window_emit) but whose amounts do not fit its u32 later-sums: a wide item (an amount too wide
// to pack, kFlagWideItems) or a window key's sum of 2^32 or more (kFlagWideSums). A call's later
// deltas of one account reach 2^70 and more, so the per-account state is u128 and lives in HBM, not
// LDS:
//   ae_wide_partials  per slice (ae_wide_per events) and posted field (a workgroup each), the
//                     field's sum per account in three u32 LDS limbs (2^96: 2^14 events of < 2^64)
//   ae_wide_suffix    per account and field, the exclusive suffix over the slices: sums[w] = the
//                     deltas of slices w + 1, w + 2, ... (u128)
//   ae_wide_emit      per slice, its rounds of 1024 events from the LAST one back: R = sums[w] (the
//                     slice's own region, updated in place) holds the deltas after the round; the
//                     round's touch lists (LDS, as in ae_window_emit) give the deltas of the round's
//                     events after e, and the list's head owner adds the round's deltas to R before
//                     the round before it. A record's posted balances are the final ones less
//                     R + those (u128); records are written once, in call order (positions from a
//                     count of the slice's created events per round and wave).
// account_event :4384-4465 (the balances after the event), as ae_window_emit.
constexpr uint32_t kAeWideThreads = 1024;
constexpr uint32_t kAeWideWaves = kAeWideThreads / 64;
// A slice is `per` events, a multiple of 1024: at least 16 rounds, and as many as it takes for the
// emit's workgroups (one per CU: 128 KB of LDS) to run in one generation, up to 64 rounds.
constexpr uint32_t kAeWideRoundsMin = 16, kAeWideRoundsMax = 64;
constexpr uint32_t kAeWideGrid = 256;
__host__ __device__ inline uint32_t ae_wide_per(uint32_t n) {
    uint32_t rounds = (n + kAeWideGrid * kAeWideThreads - 1) / (kAeWideGrid * kAeWideThreads);
    rounds = rounds < kAeWideRoundsMin ? kAeWideRoundsMin : rounds > kAeWideRoundsMax ? kAeWideRoundsMax : rounds;
    return rounds * kAeWideThreads;
}

struct AeWide {
    const uint64_t* items;               // the call's pair items (~0: none)
    const uint64_t* amounts;             // ev_amount: a wide item's amount
    const tb_create_result_t* results;
    const tb_account_t* acc_rows;
    uint32_t n, ps, rows, slices, per;
    uint64_t row_base;
    u128* sums;                          // [slice][field][row]: partials, suffix sums, then R
    unsigned int* slice_count;           // per slice: its created events
    unsigned long long* slice_ts;        // per slice: its first and last created timestamp
    unsigned int* done;                  // finished emit workgroups (the last one closes the block)
    tb_account_event_t* log;
    AeRef* refs;
    unsigned long long* state;           // the log on device (AeScratch::state)
    uint64_t cap;
};

__device__ inline void ae_wide_item(const AeWide& A, uint64_t x, uint64_t wide_amount,
                                    uint32_t* dr, uint32_t* cr, uint64_t* amount) {
    const uint64_t rmask = (1ull << A.ps) - 1;
    *dr = uint32_t(x & rmask);
    *cr = uint32_t((x >> A.ps) & rmask);
    const uint64_t a = x >> (2 * A.ps + 1);
    *amount = a == pair_amount_mask(A.ps) ? wide_amount : a;
}

// Workgroup 2 w + f: slice w's sums of field f (0 debits_posted, 1 credits_posted) per account.
__global__ void __launch_bounds__(kAeWideThreads) ae_wide_partials(AeWide A) {
    __shared__ uint32_t lo[kAeWinRowsMax], hi[kAeWinRowsMax], top[kAeWinRowsMax];
    __shared__ uint32_t wave_cnt[kAeWideWaves];
    const uint32_t tid = threadIdx.x, w = blockIdx.x >> 1, f = blockIdx.x & 1;
    for (uint32_t r = tid; r < A.rows; r += kAeWideThreads) {
        lo[r] = 0;
        hi[r] = 0;
        top[r] = 0;
    }
    const uint32_t b0 = w * A.per;
    const uint32_t b1 = b0 + A.per < A.n ? b0 + A.per : A.n;
    __syncthreads();
    uint32_t cnt = 0;
    constexpr uint32_t kLoads = 16;  // (items in flight per lane)
    for (uint32_t e0 = b0 + tid; e0 < b1; e0 += kLoads * kAeWideThreads) {
        uint64_t x[kLoads];
#pragma unroll
        for (uint32_t j = 0; j < kLoads; j++) {
            const uint32_t e = e0 + j * kAeWideThreads;
            x[j] = e < b1 ? A.items[e] : ~0ull;
        }
#pragma unroll
        for (uint32_t j = 0; j < kLoads; j++) {
            if (x[j] == ~0ull) continue;
            cnt++;
            const uint32_t e = e0 + j * kAeWideThreads;
            const uint64_t mask = pair_amount_mask(A.ps);
            uint32_t dr, cr;
            uint64_t a;
            ae_wide_item(A, x[j], (x[j] >> (2 * A.ps + 1)) == mask ? A.amounts[e] : 0, &dr, &cr, &a);
            const uint32_t row = f ? cr : dr;
            const uint32_t alo = uint32_t(a);
            const uint32_t old = atomicAdd(&lo[row], alo);
            const uint64_t h = (a >> 32) + (uint32_t(old + alo) < old ? 1u : 0u);
            if (h) {
                const uint32_t oh = atomicAdd(&hi[row], uint32_t(h));
                const uint32_t t = uint32_t(h >> 32) + (uint32_t(oh + uint32_t(h)) < oh ? 1u : 0u);
                if (t) atomicAdd(&top[row], t);
            }
        }
    }
    for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
    if ((tid & 63) == 0) wave_cnt[tid >> 6] = cnt;
    __syncthreads();
    if (f == 0 && tid == 0) {
        uint32_t t = 0;
        for (uint32_t j = 0; j < kAeWideWaves; j++) t += wave_cnt[j];
        A.slice_count[w] = t;
    }
    // (an account's two fields side by side: the emit reads both with one 32-byte access)
    u128* out = A.sums + uint64_t(w) * 2 * A.rows + f;
    for (uint32_t r = tid; r < A.rows; r += kAeWideThreads)
        out[2 * r] = (u128(top[r]) << 64) | (uint64_t(hi[r]) << 32) | lo[r];
}

// One lane per (field, account) key: sums[w][key] = the key's sums over the slices after w.
__global__ void ae_wide_suffix(AeWide A) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= 2 * A.rows) return;
    const uint64_t stride = 2 * uint64_t(A.rows);
    u128* p = A.sums + k;
    u128 s = 0;
    int64_t w = int64_t(A.slices) - 1;
    for (; w >= 7; w -= 8) {  // (eight loads in flight)
        u128 v[8];
#pragma unroll
        for (int j = 0; j < 8; j++) v[j] = p[uint64_t(w - j) * stride];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            p[uint64_t(w - j) * stride] = s;
            s += v[j];
        }
    }
    for (; w >= 0; w--) {
        const u128 v = p[uint64_t(w) * stride];
        p[uint64_t(w) * stride] = s;
        s += v;
    }
}

__global__ void __launch_bounds__(kAeWideThreads) ae_wide_emit(AeWide A) {
    __shared__ uint32_t head[kAeWinRowsMax];          // the round's touch lists (node 2e + side)
    __shared__ uint16_t next[2 * kAeWideThreads];
    __shared__ uint64_t amt[kAeWideThreads];
    __shared__ uint4 later[4][kAeWideThreads];        // dr debits / credits, cr debits / credits
    __shared__ uint32_t offs[kAeWideRoundsMax * kAeWideWaves];  // a round's wave's first record
    __shared__ uint32_t red[2][kAeWideWaves];
    __shared__ unsigned long long ts_lds[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, w = blockIdx.x;
    const uint32_t b0 = w * A.per;
    const uint32_t b1 = b0 + A.per < A.n ? b0 + A.per : A.n;
    const uint32_t rounds = (b1 - b0 + kAeWideThreads - 1) / kAeWideThreads;
    // created events of the earlier slices; of all (the room in the log: else nothing is written)
    uint32_t before = 0, all = 0;
    for (uint32_t j = tid; j < A.slices; j += kAeWideThreads) {
        before += j < w ? A.slice_count[j] : 0;
        all += A.slice_count[j];
    }
    for (int off = 32; off > 0; off >>= 1) {
        before += __shfl_xor(before, off);
        all += __shfl_xor(all, off);
    }
    if (lane == 0) {
        red[0][wv] = before;
        red[1][wv] = all;
    }
    // the slice's created events per round and wave
#pragma unroll 8
    for (uint32_t r = 0; r < kAeWideRoundsMax; r++) {
        const uint32_t e = b0 + r * kAeWideThreads + tid;
        const bool valid = r < rounds && e < b1 && A.items[e] != ~0ull;
        const uint64_t bal = __ballot(valid);
        if (lane == 0) offs[r * kAeWideWaves + wv] = uint32_t(__popcll(bal));
    }
    for (uint32_t a = tid; a < A.rows; a += kAeWideThreads) head[a] = kAeWinNil;
    if (tid == 0) {
        ts_lds[0] = ~0ull;
        ts_lds[1] = 0;
    }
    const uint64_t used = A.state[0];
    __syncthreads();
    uint64_t total = 0, pos = used;
    for (uint32_t j = 0; j < kAeWideWaves; j++) {
        pos += red[0][j];
        total += red[1][j];
    }
    if (!ae_room(A.state, A.cap, total)) {
        if (tid == 0) A.state[3] = 1;
        return;
    }
    // exclusive scan of the (round, wave) counts, one entry per thread
    static_assert(kAeWideRoundsMax * kAeWideWaves == kAeWideThreads, "one scan entry per thread");
    const uint32_t v = offs[tid];
    uint32_t inc = v;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t t = __shfl_up(inc, off, 64);
        if (lane >= uint32_t(off)) inc += t;
    }
    __syncthreads();  // (every count read; red reused)
    if (lane == 63) red[0][wv] = inc;
    __syncthreads();
    {
        uint32_t base = 0;
        for (uint32_t j = 0; j < wv; j++) base += red[0][j];
        offs[tid] = base + inc - v;
    }
    __syncthreads();
    u128* R = A.sums + uint64_t(w) * 2 * A.rows;  // [2 row] debits_posted, [2 row + 1] credits
    uint64_t ts_min = ~0ull, ts_max = 0;
    // (the next round's item, timestamp and amount are loaded during the current round)
    uint64_t x_n = ~0ull, ts_n = 0, am_n = 0;
    auto prefetch = [&](int32_t r) {
        const uint32_t e = b0 + uint32_t(r) * kAeWideThreads + tid;
        x_n = ~0ull;
        if (r >= 0 && e < b1) {
            x_n = A.items[e];
            ts_n = A.results[e].timestamp;
            am_n = A.amounts[e];
        }
    };
    // (and the round's R words: loaded during the round after it, once its owners stored theirs)
    u128 Rd[2] = {0, 0}, Rc[2] = {0, 0};
    auto load_r = [&]() {
        if (x_n == ~0ull) return;
        uint32_t ndr, ncr;
        uint64_t na;
        ae_wide_item(A, x_n, am_n, &ndr, &ncr, &na);
#pragma unroll
        for (int side = 0; side < 2; side++) {
            const uint32_t acc = side ? ncr : ndr;
            Rd[side] = R[2 * acc];
            Rc[side] = R[2 * acc + 1];
        }
    };
    prefetch(int32_t(rounds) - 1);
    load_r();
    for (int32_t r = int32_t(rounds) - 1; r >= 0; r--) {
        const uint32_t e = b0 + uint32_t(r) * kAeWideThreads + tid;
        const uint64_t x = x_n, ts = ts_n, wide_amount = am_n;
        const bool valid = x != ~0ull;
        uint32_t dr = 0, cr = 0;
        uint64_t a = 0;
        if (valid) {
            ae_wide_item(A, x, wide_amount, &dr, &cr, &a);
            next[2 * tid] = uint16_t(atomicExch(&head[dr], 2 * tid));
            next[2 * tid + 1] = uint16_t(atomicExch(&head[cr], 2 * tid + 1));
            amt[tid] = a;
        }
        const uint64_t bal = __ballot(valid);
        __syncthreads();
        // Per side: the account's R (deltas after the round), the round's deltas after e, and --
        // for the list's head owner -- the round's total, which it adds to R after every read.
        // (the owner keeps R plus the round's total for after the barrier: nd_ / nc_)
        u128 nd_[2] = {0, 0}, nc_[2] = {0, 0};
        bool own[2] = {false, false};
        prefetch(r - 1);
        if (valid) {
#pragma unroll
            for (int side = 0; side < 2; side++) {
                const uint32_t acc = side ? cr : dr;
                const uint32_t h = head[acc];
                own[side] = h == 2 * tid + side;
                u128 ad = 0, ac = 0, td = 0, tc = 0;
                for (uint32_t nd = h; nd != kAeWinNil;) {
                    const u128 val = amt[nd >> 1];
                    const bool after = (nd >> 1) > tid;
                    if (nd & 1) {
                        tc += val;
                        ac += after ? val : u128(0);
                    } else {
                        td += val;
                        ad += after ? val : u128(0);
                    }
                    const uint32_t nx = next[nd];
                    nd = nx == 0xFFFFu ? kAeWinNil : nx;
                }
                later[2 * side][tid] = ae_q(Rd[side] + ad);
                later[2 * side + 1][tid] = ae_q(Rc[side] + ac);
                nd_[side] = own[side] ? Rd[side] + td : u128(0);
                nc_[side] = own[side] ? Rc[side] + tc : u128(0);
            }
        }
        __syncthreads();  // (every R read and list walked before the round's updates)
        if (valid) {
#pragma unroll
            for (int side = 0; side < 2; side++) {
                if (!own[side]) continue;
                const uint32_t acc = side ? cr : dr;
                R[2 * acc] = nd_[side];
                R[2 * acc + 1] = nc_[side];
                head[acc] = kAeWinNil;
            }
            ts_min = ts < ts_min ? ts : ts_min;
            ts_max = ts > ts_max ? ts : ts_max;
        }
        __syncthreads();  // (the round's R stores before the next round's loads)
        load_r();
        const uint64_t wave_pos = pos + offs[uint32_t(r) * kAeWideWaves + wv];
        if (valid) {
            const uint32_t rank = lane ? __popcll(bal & (~0ull >> (64 - lane))) : 0;
            ae_nt_store(reinterpret_cast<uint4*>(&A.refs[wave_pos + rank]),
                        make_uint4(uint32_t(A.row_base + e), dr, cr, 0));
        }
        // The wave's records, four at a time, as in ae_window_emit (lane L writes word L % 16 of
        // the record of event lane 4 j + L / 16; the later sums from LDS), kWideRecBatch groups'
        // row loads issued together.
        constexpr uint32_t kWideRecBatch = 4;
        const uint32_t wd = lane & 15, sub = lane >> 4;
        const bool credit_half = (wd >= 5 && wd < 10) || wd == 11;
        const uint32_t k = wd < 5 ? wd : wd < 10 ? wd - 5 : 7;
#pragma unroll 1
        for (uint32_t j0 = 0; j0 < 16; j0 += kWideRecBatch) {
            if (((bal >> (4 * j0)) & ((1ull << (4 * kWideRecBatch)) - 1)) == 0) continue;
            uint4 q[kWideRecBatch];
#pragma unroll
            for (uint32_t b = 0; b < kWideRecBatch; b++) {
                const uint32_t src = 4 * (j0 + b) + sub;
                const uint32_t s_dr = __shfl(dr, src), s_cr = __shfl(cr, src);
                q[b] = make_uint4(0, 0, 0, 0);
                if ((bal >> src) & 1)
                    q[b] = reinterpret_cast<const uint4*>(&A.acc_rows[credit_half ? s_cr : s_dr])[k];
            }
#pragma unroll
            for (uint32_t b = 0; b < kWideRecBatch; b++) {
                const uint32_t src = 4 * (j0 + b) + sub;
                const uint32_t a_lo = __shfl(uint32_t(a), src), a_hi = __shfl(uint32_t(a >> 32), src);
                const uint32_t ts_lo = __shfl(uint32_t(ts), src), ts_hi = __shfl(uint32_t(ts >> 32), src);
                const uint32_t dflags = __shfl(q[b].y, lane > 0 ? lane - 1 : 0);
                if (!((bal >> src) & 1)) continue;
                uint4 o = q[b];
                if (k == 2 || k == 4) {
                    const uint4 l = later[(credit_half ? 2 : 0) + (k == 4 ? 1 : 0)][wv * 64 + src];
                    o = ae_q(ae_u(q[b]) - ae_u(l));
                } else if (wd == 10) {
                    o = make_uint4(ts_lo, ts_hi, q[b].z, q[b].w);
                } else if (wd == 11) {
                    o = make_uint4(q[b].z, q[b].w, (dflags >> 16) | (q[b].y & 0xFFFF0000u), 0u);
                } else if (wd == 12) {
                    o = make_uint4(0, 0, 0, 0);
                } else if (wd == 13 || wd == 14) {
                    o = make_uint4(a_lo, a_hi, 0, 0);
                } else if (wd == 15) {
                    o = make_uint4(q[b].x, uint32_t(TB_PENDING_NONE), 0, 0);
                }
                const uint64_t at = wave_pos + uint64_t(__popcll(bal & ((1ull << src) - 1)));
                ae_nt_store(reinterpret_cast<uint4*>(&A.log[at]) + wd, o);
            }
        }
        __syncthreads();  // (R current and the lists empty for the round before)
    }
    ae_slices_close(ts_min, ts_max, ts_lds, A.slice_ts, A.slice_count, A.done, A.state, used, w);
}

// ---- AccountEvents of small calls in one pass ----------------------------------------------------
//
// A small create_transfers call's appends (the side stream, behind the next call) when every
// created event is single-phase with an amount below 2^19 and the key space is dense enough for
// the LDS (<= kAeWinRowsMax accounts): the staged records (stage_out's snapshot: the finished
// AccountEvent with both accounts' final state) need only their posted balances lowered by the
// later events' deltas. One launch of kAeSmallWgs workgroups, one per 256 staged events; each
// sums the posted deltas of the events from its own first one on into LDS (R, the accounts' later
// deltas at its start), then resolves its 1024 events as one round of ae_window_emit (touch lists
// in LDS) and copies the records into the log with the balances patched, four records per 1 KB
// store. The last workgroup closes the block (length, last timestamp, order). Calls it cannot take
// go to the general appends queued behind it (their kernels skip the calls it took).
constexpr uint32_t kAeSmallThreads = 256;
constexpr uint32_t kAeSmallWgs = 32;  // (32 CUs of waves in flight; 8 of 1024 lanes: 35 us a call)
static_assert(kAeSmallWgs * kAeSmallThreads == kAeAsyncMax, "one round per workgroup over the staging");

struct AeSmall {
    AeStage st;
    uint32_t epoch;
    uint32_t rows;
    // 0: created transfers (posted deltas, words 2 / 4 lowered); 1: a pulse's expiries (pending
    // deltas -amount, words 1 / 3 raised by the later expiries' amounts)
    uint32_t pending;
    tb_account_event_t* log;
    AeRef* refs;
    unsigned long long* state;     // the log on device (AeScratch::state)
    unsigned int* counts;          // [kAeSmallWgs] created per workgroup, [kAeSmallWgs] done
    unsigned long long* slice_ts;  // [2 * kAeSmallWgs]
    uint64_t cap;
};

// A staged event's amount on both of its accounts (every staged event moves the same amount on
// its two sides): posted for created transfers, the pending amount released by an expiry.
__device__ inline uint32_t ae_small_amount(const AeSmall& A, uint32_t e) {
    return A.pending ? uint32_t(0u - uint32_t(A.st.delta[2 * e].pending))
                     : uint32_t(A.st.delta[2 * e].posted);
}
__device__ inline uint4 ae_add_u32(uint4 balance, uint32_t d) {
    return ae_q(ae_u(balance) + u128(d));
}

__global__ void __launch_bounds__(kAeSmallThreads) ae_small_emit(AeSmall A) {
    __shared__ uint32_t Rd[kAeWinRowsMax];
    __shared__ uint32_t Rc[kAeWinRowsMax];
    __shared__ uint32_t head[kAeWinRowsMax];
    __shared__ uint16_t next[2 * kAeSmallThreads];
    __shared__ uint32_t amt[kAeSmallThreads];
    __shared__ uint32_t wave_cnt[kAeSmallThreads / 64];
    __shared__ uint32_t before_lds, all_lds;
    __shared__ unsigned long long ts_lds[2];
    if (A.st.words[0] == A.epoch) return;  // (an event the general appends take)
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, w = blockIdx.x;
    if (w == 0 && tid == 0) A.st.words[1] = A.epoch;  // (the general appends skip)
    for (uint32_t a = tid; a < A.rows; a += kAeSmallThreads) {
        Rd[a] = 0;
        Rc[a] = 0;
        head[a] = kAeWinNil;
    }
    if (tid == 0) {
        before_lds = 0;
        all_lds = 0;
        ts_lds[0] = ~0ull;
        ts_lds[1] = 0;
    }
    __syncthreads();
    // R: the posted deltas of the staged events from this workgroup's first one on; the created
    // events before it (the block's positions).
    const uint32_t e0 = w * kAeSmallThreads;
    uint32_t before = 0, all = 0;
    // (8 events a lane at a time, their staged words loaded unconditionally and all at once: the
    // staging is always readable, and a load per event in sequence waited a latency each)
    constexpr uint32_t kU = 8;
    static_assert(kAeAsyncMax % (kAeSmallThreads * kU) == 0, "whole passes");
    for (uint32_t eb = tid; eb < kAeAsyncMax; eb += kAeSmallThreads * kU) {
        uint8_t made[kU];
        uint32_t rdr[kU], rcr[kU], am[kU];
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            const uint32_t e = eb + u * kAeSmallThreads;
            made[u] = A.st.created[e];
            const AeRef r = A.st.ref[e];
            rdr[u] = r.dr_row;
            rcr[u] = r.cr_row;
            am[u] = ae_small_amount(A, e);
        }
#pragma unroll
        for (uint32_t u = 0; u < kU; u++) {
            const uint32_t e = eb + u * kAeSmallThreads;
            if (!made[u]) continue;
            all++;
            if (e < e0) {
                before++;
                continue;
            }
            atomicAdd(&Rd[rdr[u]], am[u]);
            atomicAdd(&Rc[rcr[u]], am[u]);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        before += __shfl_xor(before, off);
        all += __shfl_xor(all, off);
    }
    if (lane == 0 && before) atomicAdd(&before_lds, before);
    if (lane == 0 && all) atomicAdd(&all_lds, all);
    __syncthreads();
    if (!ae_room(A.state, A.cap, all_lds)) {  // (uniform: the same counts in every workgroup)
        if (tid == 0) A.state[3] = 1;
        return;
    }
    // this workgroup's round: its events' touches on the accounts' lists
    const uint32_t e = e0 + tid;
    const bool valid = A.st.created[e] != 0;
    uint32_t dr = 0, cr = 0, a = 0;
    uint64_t ts = 0;
    if (valid) {
        const AeRef r = A.st.ref[e];
        dr = r.dr_row;
        cr = r.cr_row;
        a = ae_small_amount(A, e);
        ts = A.st.rec[e].timestamp;
        next[2 * tid] = uint16_t(atomicExch(&head[dr], 2 * tid));
        next[2 * tid + 1] = uint16_t(atomicExch(&head[cr], 2 * tid + 1));
        amt[tid] = a;
    }
    const uint64_t bal = __ballot(valid);
    if (lane == 0) wave_cnt[wv] = uint32_t(__popcll(bal));
    __syncthreads();
    uint64_t wave_pos = A.state[0] + before_lds;
    uint32_t total = 0;
    for (uint32_t j = 0; j < kAeSmallThreads / 64; j++) {
        const uint32_t cj = wave_cnt[j];
        wave_pos += j < wv ? cj : 0;
        total += cj;
    }
    uint32_t later[4] = {0, 0, 0, 0};
    if (valid) {
#pragma unroll
        for (int side = 0; side < 2; side++) {
            const uint32_t acc = side ? cr : dr;
            uint32_t sd = 0, sc = 0;
            for (uint32_t nd = head[acc]; nd != kAeWinNil;) {
                if ((nd >> 1) <= tid) {
                    const uint32_t v = amt[nd >> 1];
                    if (nd & 1) sc += v;
                    else sd += v;
                }
                const uint32_t nx = next[nd];
                nd = nx == 0xFFFFu ? kAeWinNil : nx;
            }
            later[2 * side] = Rd[acc] - sd;
            later[2 * side + 1] = Rc[acc] - sc;
        }
        atomicMin(&ts_lds[0], ts);
        atomicMax(&ts_lds[1], ts);
        const uint32_t rank = lane ? __popcll(bal & (~0ull >> (64 - lane))) : 0;
        ae_nt_store(reinterpret_cast<uint4*>(&A.refs[wave_pos + rank]),
                    *reinterpret_cast<const uint4*>(&A.st.ref[e]));
    }
    // The records, four per 1 KB store: lane L copies word L % 16 of event lane 4 j + L / 16's
    // staged record, the posted balances (words 2, 4 / 7, 9) lowered by the later deltas.
    const uint32_t wd = lane & 15, sub = lane >> 4;
    const bool credit_half = wd >= 5 && wd < 10;
    const uint32_t k = credit_half ? wd - 5 : wd;
    const uint4* recs = reinterpret_cast<const uint4*>(A.st.rec);
    const uint32_t kd = A.pending ? 1 : 2, kc = A.pending ? 3 : 4;  // the patched words
    for (uint32_t j0 = 0; j0 < 16; j0 += kAeRecBatch) {
        if (((bal >> (4 * j0)) & ((1ull << (4 * kAeRecBatch)) - 1)) == 0) continue;  // (uniform)
        uint4 qs[kAeRecBatch];
#pragma unroll
        for (uint32_t u = 0; u < kAeRecBatch; u++) {
            const uint32_t src = 4 * (j0 + u) + sub;
            const uint32_t es = e0 + (tid & ~63u) + src;
            qs[u] = ((bal >> src) & 1) ? recs[uint64_t(es) * 16 + wd] : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (uint32_t u = 0; u < kAeRecBatch; u++) {
            const uint32_t src = 4 * (j0 + u) + sub;
            const uint32_t l0 = __shfl(later[0], src), l1 = __shfl(later[1], src);
            const uint32_t l2 = __shfl(later[2], src), l3 = __shfl(later[3], src);
            if (!((bal >> src) & 1)) continue;
            uint4 q = qs[u];
            const uint32_t l = wd >= 10 ? 0u : k == kd ? (credit_half ? l2 : l0)
                                          : k == kc ? (credit_half ? l3 : l1) : 0u;
            if (l) q = A.pending ? ae_add_u32(q, l) : ae_sub_u32(q, l);
            const uint64_t at = wave_pos + uint64_t(__popcll(bal & ((1ull << src) - 1)));
            ae_nt_store(reinterpret_cast<uint4*>(&A.log[at]) + wd, q);
        }
    }
    __syncthreads();
    if (tid != 0) return;
    A.counts[w] = total;
    A.slice_ts[2 * w] = ts_lds[0];
    A.slice_ts[2 * w + 1] = ts_lds[1];
    __threadfence();
    if (atomicAdd(&A.counts[kAeSmallWgs], 1u) != gridDim.x - 1) return;
    __threadfence();
    const volatile unsigned int* counts = A.counts;
    const volatile unsigned long long* sts = A.slice_ts;
    uint64_t appended = 0, first = 0, last = 0;
    bool any = false;
    for (uint32_t j = 0; j < gridDim.x; j++) {
        const uint32_t cj = counts[j];
        if (!cj) continue;
        if (!any) first = sts[2 * j];
        any = true;
        last = sts[2 * j + 1];
        appended += cj;
    }
    const uint64_t used = A.state[0];
    if (appended) {
        if (used && first <= A.state[1]) A.state[2] = 1;
        if (last > A.state[1]) A.state[1] = last;
        A.state[0] = used + appended;
    }
    A.counts[kAeSmallWgs] = 0;
}

// ---- AccountEvents of general calls in one pass (dense key spaces) ------------------------------
//
// A create_transfers call of any shape -- replayed events, pending transfers, posts and voids --
// over <= kAeWinRowsMax accounts, when no created event flips `closed` and every amount moved is
// below 2^19: every created event moves the same pending delta (a pending transfer's amount, or
// minus the amount a post / void releases) and posted delta (the amount posted) on both of its
// accounts. The record of created event e carries, for each account A of e,
//     A's balance after e = A's final balance - A's deltas of the created events after e
// for all four balances, and A's final row otherwise. The call is cut into slices of
// kAeDenseSlice events:
//   ae_dense_stage     per event: its touch (rows, deltas; absent unless created) and the record's
//                      event words, from the transfer row (and the pending transfer's);
//                      kFlagAeWide-style refusal in *fail (a flip, an amount >= 2^19)
//   ae_dense_partials  per slice and balance pair (pending / posted): the slice's deltas per
//                      account (LDS sums), and its created count
//   ae_dense_suffix    per pair and account key: the partials summed over the later slices (i64;
//                      refusal when a sum reaches 2^30: a later delta is then a suffix less at
//                      most kAeDenseSlice * 2^19 = 2^30, inside the i32 range)
//   ae_dense_later     per slice: its touches (account, event, side) sorted in registers
//                      (block_bitonic_sort), one segmented scan of the four deltas (pending /
//                      posted on the debit / credit side) along the sorted order gives every touch
//                      its account's sums up to its event, the slice's suffix less those is its
//                      later deltas; with each event's position in the block.
//                      (Touch lists walked per event cost O(L^2) in a round's L touches of one
//                      hot account; the sort costs the same for any key distribution.)
//   ae_dense_records   per 256 events: the records from the final rows, four per 1 KB store
//                      (a kernel of its own: small workgroups keep enough waves in flight for the
//                      row loads, which the sort's 64 large workgroups did not).
// The host checks the refusal word between the suffix and the emit; a refused call takes the
// general appends.
constexpr uint32_t kAeDenseSlice = 2048;
constexpr uint32_t kAeDenseEmitThreads = 1024;
constexpr uint32_t kAeDenseEv = kAeDenseSlice / kAeDenseEmitThreads;  // events per lane
constexpr uint32_t kAeDenseKeys = 2 * kAeDenseEv;                      // touches per lane
constexpr uint32_t kAeDenseTixBits = 12;                               // log2(2 * kAeDenseSlice)
static_assert(2 * kAeDenseSlice == (1u << kAeDenseTixBits), "touch index bits");
static_assert(kAeWinRowsMax < (1u << (32 - kAeDenseTixBits)), "account row bits");

struct AeTouch {
    uint32_t dr, cr;  // account rows (kNone32: the event created nothing)
    uint32_t dpe, dpo;  // pending / posted delta on both accounts (i32 as u32)
};

struct AeDense {
    Tables T;
    Call<tb_transfer_t> c;
    uint32_t rows, slices;
    AeTouch* touch;           // per event
    uint4* ev;                // per event, 5 words: pending id, amount requested, amount,
                              // (ts lo, ts hi, transfer flags | pending flags << 16, ledger),
                              // (status, 0, 0, 0)
    uint32_t* partials;       // [pair][slice][2 * rows]: debit-side then credit-side sums
    unsigned int* slice_count;  // [slices] created events
    unsigned int* done;         // finished record workgroups (a word of its own: zero between calls)
    unsigned long long* slice_ts;  // [0] / [1]: the first / last created timestamp (~0 / 0 between calls)
    uint4* later;               // per event, two words (ae_dense_later)
    uint32_t* pos;              // per event: its position among the call's created events
    unsigned int* fail;       // == epoch: the call takes the general appends (the low half of a
                              // mapped pinned word the host reads after its synchronisation)
    unsigned int* claim;      // device words: [0] == epoch: ae_dense_stage refused the call (the
                              // later kernels return at once; ae_dense_suffix's block 0 forwards it
                              // to `fail`); [1] == epoch: a suffix wave has written `fail`;
                              // [2] == epoch: a created event moves a pending balance (else the
                              // pending pair's partials are neither written nor read: all zero)
    uint32_t epoch;
    tb_account_event_t* log;
    AeRef* refs;
    unsigned long long* state;
    uint64_t cap;
};

// The host's refusal word, one system-scope release per call (with wide amounts nearly every wave
// of ae_dense_stage refuses: those only store claim[0]).
__device__ inline void ae_dense_refuse(const AeDense& A) {
    *A.fail = A.epoch;
    __threadfence_system();
}

__device__ inline bool ae_dense_refused(const AeDense& A) { return A.claim[0] == A.epoch; }

__global__ void ae_dense_stage(AeDense A) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const Call<tb_transfer_t>& c = A.c;
    AeTouch o{kNone32, kNone32, 0, 0};
    bool bad = false;
    if (k < c.n && c.results[k].status == TB_STATUS_CREATED) {
        const Tables& T = A.T;
        const uint64_t row = c.row_base + k;
        const tb_transfer_t& t = T.tr_rows[row];
        const uint16_t f = t.flags;
        const bool pv = (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) != 0;
        uint32_t edr = kNone32, ecr = kNone32;
        if (!pv) ae_known_rows(c, k, c.ev_info[k], &edr, &ecr);
        const uint64_t dr = edr != kNone32 ? uint64_t(edr) : account_find(T, t.debit_account_id);
        const uint64_t cr = ecr != kNone32 ? uint64_t(ecr) : account_find(T, t.credit_account_id);
        const tb_transfer_t* p = pv ? &T.tr_rows[ae_transfer_row(T, t.pending_id)] : nullptr;
        uint8_t status = TB_PENDING_NONE;
        u128 dpe = 0, dpo = 0;
        bool flip = false;
        if (p) {
            dpe = u128(0) - U(p->amount);
            if (f & TB_TRANSFER_POST_PENDING) {
                status = TB_PENDING_POSTED;
                dpo = U(t.amount);
            } else {
                status = TB_PENDING_VOIDED;
                flip = (p->flags & (TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT)) != 0;
            }
        } else if (f & TB_TRANSFER_PENDING) {
            status = TB_PENDING_PENDING;
            dpe = U(t.amount);
            flip = (f & (TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT)) != 0;
        } else {
            dpo = U(t.amount);
        }
        const u128 mag = (dpe >> 127) ? u128(0) - dpe : dpe;
        bad = flip || mag >= kAeSmallAmountMax || dpo >= kAeSmallAmountMax;
        o = AeTouch{uint32_t(dr), uint32_t(cr), uint32_t(uint64_t(dpe)), uint32_t(uint64_t(dpo))};
        const uint32_t pf = p ? p->flags : 0u;
        uint4* e = A.ev + uint64_t(k) * 5;
        e[0] = p ? ae_q128(p->id) : make_uint4(0, 0, 0, 0);
        e[1] = ae_q128(c.events[k].amount);
        e[2] = ae_q128(t.amount);
        e[3] = make_uint4(uint32_t(t.timestamp), uint32_t(t.timestamp >> 32),
                          uint32_t(f) | (pf << 16), t.ledger);
        e[4] = make_uint4(status, 0, 0, 0);
    }
    if (__any(bad) && (threadIdx.x & 63) == 0) A.claim[0] = A.epoch;
    if (__any(o.dpe != 0) && (threadIdx.x & 63) == 0) A.claim[2] = A.epoch;
    if (k < c.n) A.touch[k] = o;
}

// Workgroup 2 s + q: slice s, pair q (0 pending, 1 posted).
__global__ void __launch_bounds__(kAeWinThreads) ae_dense_partials(AeDense A) {
    __shared__ uint32_t Rd[kAeWinRowsMax];
    __shared__ uint32_t Rc[kAeWinRowsMax];
    __shared__ uint32_t wave_cnt[kAeWinThreads / 64];
    const uint32_t tid = threadIdx.x, s = blockIdx.x >> 1, q = blockIdx.x & 1;
    if (ae_dense_refused(A)) return;  // (written before this launch: uniform over the block)
    if (q == 0 && A.claim[2] != A.epoch) return;  // (no pending deltas in the call)
    for (uint32_t a = tid; a < A.rows; a += kAeWinThreads) {
        Rd[a] = 0;
        Rc[a] = 0;
    }
    __syncthreads();
    const uint32_t e0 = s * kAeDenseSlice;
    const uint32_t e1 = e0 + kAeDenseSlice < A.c.n ? e0 + kAeDenseSlice : A.c.n;
    uint32_t made = 0;
    for (uint32_t e = e0 + tid; e < e1; e += kAeWinThreads) {
        const AeTouch t = A.touch[e];
        if (t.dr == kNone32) continue;
        made++;
        const uint32_t d = q ? t.dpo : t.dpe;
        if (d) {
            atomicAdd(&Rd[t.dr], d);
            atomicAdd(&Rc[t.cr], d);
        }
    }
    for (int off = 32; off > 0; off >>= 1) made += __shfl_xor(made, off);
    if ((tid & 63) == 0) wave_cnt[tid >> 6] = made;
    __syncthreads();
    uint32_t* out = A.partials + (uint64_t(q) * A.slices + s) * 2 * A.rows;
    for (uint32_t a = tid; a < A.rows; a += kAeWinThreads) {
        out[a] = Rd[a];
        out[A.rows + a] = Rc[a];
    }
    if (q == 1 && tid == 0) {  // (the posted pair's workgroups always run)
        uint32_t total = 0;
        for (uint32_t w = 0; w < kAeWinThreads / 64; w++) total += wave_cnt[w];
        A.slice_count[s] = total;
    }
}

// partials[pair][s][key] = the sum over slices >= s (i64; a sum of magnitude 2^30 or more
// refuses the call). A workgroup takes 64 (pair, key) columns and splits each column's slices
// into kAeSufGroups ranges, one wave per range: each wave sums its range, the ranges' totals
// meet in LDS, and each wave then writes its range's suffixes from the total of the ranges
// above it. (One lane per column walking every slice was a chain of slices/8 dependent load
// batches: 20 us for a 131k-event call's 64 slices.)
constexpr int kAeSufGroups = 16;
constexpr int kAeSufThreads = 64 * kAeSufGroups;

// (Holding a range in registers between the passes, 32 loads in flight a lane, took 16 us: 78
// VGPRs left room for one 1,024-lane workgroup per CU, and capping them spilled.)
__global__ __launch_bounds__(kAeSufThreads) void ae_dense_suffix(AeDense A) {
    __shared__ long long total[kAeSufGroups][64];
    const uint32_t lane = threadIdx.x & 63, g = threadIdx.x >> 6;
    if (ae_dense_refused(A)) {
        if (blockIdx.x == 0 && threadIdx.x == 0) ae_dense_refuse(A);
        return;
    }
    const uint32_t keys = 2 * A.rows;
    const uint32_t t = blockIdx.x * 64 + lane;
    const uint32_t q = t < 2 * keys ? t / keys : 0, key = t < 2 * keys ? t % keys : 0;
    const bool live = t < 2 * keys && (q == 1 || A.claim[2] == A.epoch);  // (pending: all zero)
    uint32_t* p = A.partials + uint64_t(q) * A.slices * keys + key;
    const uint32_t per = (A.slices + kAeSufGroups - 1) / kAeSufGroups;
    const uint32_t lo = min(g * per, A.slices), hi = min(lo + per, A.slices);
    constexpr int kB = 8;  // (loads in flight before their uses)
    int64_t sum = 0;
    if (live) {
        for (uint32_t s0 = lo; s0 < hi; s0 += kB) {
            uint32_t v[kB];
#pragma unroll
            for (int j = 0; j < kB; j++) v[j] = s0 + j < hi ? p[uint64_t(s0 + j) * keys] : 0u;
#pragma unroll
            for (int j = 0; j < kB; j++) sum += int32_t(v[j]);
        }
    }
    total[g][lane] = sum;
    __syncthreads();
    int64_t acc = 0;
    for (uint32_t h = g + 1; h < kAeSufGroups; h++) acc += total[h][lane];
    bool wide = false;
    if (live) {
        for (int64_t s1 = hi; s1 > int64_t(lo); s1 -= kB) {
            uint32_t v[kB];
#pragma unroll
            for (int j = 0; j < kB; j++) {
                const int64_t s = s1 - 1 - j;
                v[j] = s >= int64_t(lo) ? p[uint64_t(s) * keys] : 0u;
            }
#pragma unroll
            for (int j = 0; j < kB; j++) {
                const int64_t s = s1 - 1 - j;
                if (s >= int64_t(lo)) {
                    acc += int32_t(v[j]);
                    wide |= acc >= (int64_t(1) << 30) || acc <= -(int64_t(1) << 30);
                    p[uint64_t(s) * keys] = uint32_t(int32_t(acc));
                }
            }
        }
    }
    if (__any(wide) && lane == 0 && atomicExch(A.claim + 1, A.epoch) != A.epoch) ae_dense_refuse(A);
}

__global__ void ae_dense_ts_init(unsigned long long* ts) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        ts[0] = ~0ull;
        ts[1] = 0;
    }
}

// A balance less a sign-extended i32 later delta.
__device__ inline uint4 ae_sub_i32(uint4 balance, uint32_t d) {
    return ae_q(ae_u(balance) - u128(int64_t(int32_t(d))));  // (sign-extended: u128 wraps)
}

// ae_dense_later's LDS: the sort's stages, the slice's deltas by event, the later deltas by touch.
struct AeDenseLds {
    uint32_t keys[2 * kAeDenseSlice];
    uint32_t pe[kAeDenseSlice], po[kAeDenseSlice];
    uint4 later[2 * kAeDenseSlice];  // (pending debit-side, credit-side; posted debit, credit)
    uint32_t scan_f[kAeDenseEmitThreads / 64];
    uint4 scan_v[kAeDenseEmitThreads / 64];
    uint32_t wave_cnt[kAeDenseEv][kAeDenseEmitThreads / 64];
    uint32_t before;
};

__device__ inline uint4 ae_add4(uint4 a, uint4 b) {
    return make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}
__device__ inline uint4 ae_shfl_up4(uint4 v, int d) {
    return make_uint4(__shfl_up(v.x, d, 64), __shfl_up(v.y, d, 64), __shfl_up(v.z, d, 64),
                      __shfl_up(v.w, d, 64));
}

// Per slice: every created event's later deltas (A.later[2 e]: pending, debit account's debits /
// credits then the credit account's; [2 e + 1]: posted) and its position among the call's created
// events (A.pos[e]).
__global__ void __launch_bounds__(kAeDenseEmitThreads) ae_dense_later(AeDense A) {
    constexpr uint32_t kWaves = kAeDenseEmitThreads / 64, N = kAeDenseKeys;
    constexpr uint32_t kTixMask = (1u << kAeDenseTixBits) - 1;
    __shared__ AeDenseLds L;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, s = blockIdx.x;
    const uint32_t e0 = s * kAeDenseSlice;
    // created events of the earlier slices
    uint32_t before = 0;
    for (uint32_t j = tid; j < s; j += kAeDenseEmitThreads) before += A.slice_count[j];
    for (int off = 32; off > 0; off >>= 1) before += __shfl_xor(before, off);
    if (tid == 0) L.before = 0;
    __syncthreads();
    if (lane == 0 && before) atomicAdd(&L.before, before);
    // The slice's touches as sort keys (account row, then touch = 2 event + side; none: ~0), the
    // deltas by event. Lane tid takes events j * kAeDenseEmitThreads + tid.
    AeTouch t[kAeDenseEv];
    uint32_t k[N];
#pragma unroll
    for (uint32_t j = 0; j < kAeDenseEv; j++) {
        const uint32_t le = j * kAeDenseEmitThreads + tid, e = e0 + le;
        t[j] = e < A.c.n ? A.touch[e] : AeTouch{kNone32, kNone32, 0, 0};
        const bool valid = t[j].dr != kNone32;
        k[2 * j] = valid ? (t[j].dr << kAeDenseTixBits) | (2 * le) : ~0u;
        k[2 * j + 1] = valid ? (t[j].cr << kAeDenseTixBits) | (2 * le + 1) : ~0u;
        L.pe[le] = t[j].dpe;
        L.po[le] = t[j].dpo;
    }
    block_bitonic_sort<N, kAeDenseEmitThreads>(k, L.keys);
#pragma unroll
    for (uint32_t m = 0; m < N; m++) L.keys[tid * N + m] = k[m];
    __syncthreads();
    // Segmented inclusive sums along the sorted order (a segment: one account), four deltas at
    // once: (start flag, sums) pairs combine as (f1 | f2, f2 ? v2 : v1 + v2).
    const uint32_t prev_key = tid ? L.keys[tid * N - 1] : ~0u;
    bool f[N];
    uint4 v[N];
#pragma unroll
    for (uint32_t m = 0; m < N; m++) {
        const uint32_t key = k[m], pk = m ? k[m - 1] : prev_key;
        f[m] = (tid == 0 && m == 0) || (key >> kAeDenseTixBits) != (pk >> kAeDenseTixBits);
        v[m] = make_uint4(0, 0, 0, 0);
        if (key != ~0u) {
            const uint32_t tix = key & kTixMask, le = tix >> 1;
            const uint32_t dpe = L.pe[le], dpo = L.po[le];
            v[m] = (tix & 1) ? make_uint4(0, dpe, 0, dpo) : make_uint4(dpe, 0, dpo, 0);
        }
    }
    bool F = false;
    uint4 V = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t m = 0; m < N; m++) {
        V = f[m] ? v[m] : ae_add4(V, v[m]);
        F |= f[m];
    }
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t fo = __shfl_up(uint32_t(F), d, 64);
        const uint4 vo = ae_shfl_up4(V, d);
        if (lane >= uint32_t(d)) {
            if (!F) V = ae_add4(V, vo);
            F |= fo != 0;
        }
    }
    if (lane == 63) {
        L.scan_f[wv] = F;
        L.scan_v[wv] = V;
    }
    uint32_t fx = __shfl_up(uint32_t(F), 1, 64);
    uint4 vx = ae_shfl_up4(V, 1);
    if (lane == 0) {
        fx = 0;
        vx = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    uint4 carry = make_uint4(0, 0, 0, 0);
    for (uint32_t w = 0; w < wv; w++) carry = L.scan_f[w] ? L.scan_v[w] : ae_add4(carry, L.scan_v[w]);
    uint4 run = fx ? vx : ae_add4(carry, vx);
    // Every touch's later deltas: the suffix from this slice less its account's sums so far.
    const uint32_t* suf_pe = A.partials + (uint64_t(0) * A.slices + s) * 2 * A.rows;
    const uint32_t* suf_po = A.partials + (uint64_t(1) * A.slices + s) * 2 * A.rows;
    const bool pend = A.claim[2] == A.epoch;  // (else the pending partials were not written)
#pragma unroll
    for (uint32_t m = 0; m < N; m++) {
        run = f[m] ? v[m] : ae_add4(run, v[m]);
        const uint32_t key = k[m];
        if (key == ~0u) continue;
        const uint32_t acc = key >> kAeDenseTixBits;
        const uint32_t pe_d = pend ? suf_pe[acc] : 0u, pe_c = pend ? suf_pe[A.rows + acc] : 0u;
        L.later[key & kTixMask] = make_uint4(pe_d - run.x, pe_c - run.y,
                                             suf_po[acc] - run.z, suf_po[A.rows + acc] - run.w);
    }
    uint64_t bals[kAeDenseEv];
#pragma unroll
    for (uint32_t j = 0; j < kAeDenseEv; j++) {
        bals[j] = __ballot(t[j].dr != kNone32);
        if (lane == 0) L.wave_cnt[j][wv] = uint32_t(__popcll(bals[j]));
    }
    __syncthreads();
    uint32_t pos = L.before;
#pragma unroll
    for (uint32_t r = 0; r < kAeDenseEv; r++) {
        const uint32_t le = r * kAeDenseEmitThreads + tid, e = e0 + le;
        uint32_t wave_pos = pos, round_total = 0;
        for (uint32_t j = 0; j < kWaves; j++) {
            const uint32_t cj = L.wave_cnt[r][j];
            wave_pos += j < wv ? cj : 0;
            round_total += cj;
        }
        if (t[r].dr != kNone32) {
            const uint4 d = L.later[2 * le], c = L.later[2 * le + 1];
            A.later[2 * uint64_t(e)] = make_uint4(d.x, d.y, c.x, c.y);
            A.later[2 * uint64_t(e) + 1] = make_uint4(d.z, d.w, c.z, c.w);
            const uint32_t rank = lane ? __popcll(bals[r] & (~0ull >> (64 - lane))) : 0;
            A.pos[e] = wave_pos + rank;
        }
        pos += round_total;
    }
}

// The records: 256 lanes a workgroup, a wave's 64 events at a time (enough waves in flight to hide
// the row loads), four records per 1 KB store; the last workgroup closes the block.
constexpr uint32_t kAeDenseRecThreads = 256;

__global__ void __launch_bounds__(kAeDenseRecThreads) ae_dense_records(AeDense A) {
    __shared__ unsigned long long ts_lds[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    // the call's created events (the room in the log: else nothing is written)
    uint32_t all = 0;
    for (uint32_t j = tid; j < A.slices; j += kAeDenseRecThreads) all += A.slice_count[j];
    for (int off = 32; off > 0; off >>= 1) all += __shfl_xor(all, off);
    if (tid == 0) {
        ts_lds[0] = ~0ull;
        ts_lds[1] = 0;
    }
    if (!__syncthreads_and(ae_room(A.state, A.cap, all))) {
        if (tid == 0) A.state[3] = 1;
        return;
    }
    const uint64_t used = A.state[0];
    const uint32_t e = blockIdx.x * kAeDenseRecThreads + tid;
    const AeTouch t = e < A.c.n ? A.touch[e] : AeTouch{kNone32, kNone32, 0, 0};
    const bool valid = t.dr != kNone32;
    const uint64_t bal = __ballot(valid);
    uint4 lpe = make_uint4(0, 0, 0, 0), lpo = make_uint4(0, 0, 0, 0);
    uint32_t my_pos = 0;
    uint64_t ts_min = ~0ull, ts_max = 0;
    if (valid) {
        lpe = A.later[2 * uint64_t(e)];
        lpo = A.later[2 * uint64_t(e) + 1];
        my_pos = A.pos[e];
        ae_nt_store(reinterpret_cast<uint4*>(&A.refs[used + my_pos]),
                    make_uint4(uint32_t(A.c.row_base + e), t.dr, t.cr, 0));
        const uint4 w3 = A.ev[uint64_t(e) * 5 + 3];
        ts_min = ts_max = (uint64_t(w3.y) << 32) | w3.x;
    }
    // The records, four per 1 KB store (lane L: word L % 16 of event lane 4 j + L / 16):
    //   0-4 / 5-9 the debit / credit account's id and balances less the later deltas,
    //   10 timestamps, 11 the credit account's timestamp and the flags, 12-14 the event's
    //   pending id and amounts, 15 ledger and status.
    const uint32_t wd = lane & 15, sub = lane >> 4;
    const bool credit_half = (wd >= 5 && wd < 10) || wd == 11;
    const uint32_t kw = wd < 5 ? wd : wd < 10 ? wd - 5 : 7;
    const uint32_t ew0 = e - lane;  // the wave's first event
    for (uint32_t j0 = 0; j0 < 16; j0 += kAeRecBatch) {
        if (((bal >> (4 * j0)) & ((1ull << (4 * kAeRecBatch)) - 1)) == 0) continue;  // (uniform)
        uint4 qw[kAeRecBatch], xw[kAeRecBatch];
#pragma unroll
        for (uint32_t u = 0; u < kAeRecBatch; u++) {
            const uint32_t src = 4 * (j0 + u) + sub;
            const bool v = (bal >> src) & 1;
            const uint32_t s_dr = __shfl(t.dr, src), s_cr = __shfl(t.cr, src);
            qw[u] = make_uint4(0, 0, 0, 0);
            xw[u] = make_uint4(0, 0, 0, 0);
            if (v && (wd < 12 || wd == 15))
                qw[u] = reinterpret_cast<const uint4*>(&A.T.acc_rows[credit_half ? s_cr : s_dr])[kw];
            if (v && wd >= 10)
                xw[u] = A.ev[uint64_t(ew0 + src) * 5 + (wd <= 11 ? 3 : wd == 15 ? 4 : wd - 12)];
        }
#pragma unroll
        for (uint32_t u = 0; u < kAeRecBatch; u++) {
            const uint32_t src = 4 * (j0 + u) + sub;
            const uint32_t a0 = __shfl(lpe.x, src), a1 = __shfl(lpe.y, src);
            const uint32_t a2 = __shfl(lpe.z, src), a3 = __shfl(lpe.w, src);
            const uint32_t b0 = __shfl(lpo.x, src), b1 = __shfl(lpo.y, src);
            const uint32_t b2 = __shfl(lpo.z, src), b3 = __shfl(lpo.w, src);
            const uint32_t at_pos = __shfl(my_pos, src);
            const uint4 q = qw[u], x = xw[u];
            const uint32_t dflags = __shfl(q.y, lane > 0 ? lane - 1 : 0);
            if (!((bal >> src) & 1)) continue;
            uint4 o = q;
            if (wd < 10) {
                // (words 1 / 3: debits / credits pending; 2 / 4: posted; the account's own deltas)
                const uint32_t le2 = kw == 1 ? (credit_half ? a2 : a0) : kw == 3 ? (credit_half ? a3 : a1) : 0u;
                const uint32_t lo = kw == 2 ? (credit_half ? b2 : b0) : kw == 4 ? (credit_half ? b3 : b1) : 0u;
                if (le2) o = ae_sub_i32(o, le2);
                if (lo) o = ae_sub_i32(o, lo);
            } else if (wd == 10) {
                o = make_uint4(x.x, x.y, q.z, q.w);
            } else if (wd == 11) {
                o = make_uint4(q.z, q.w, (dflags >> 16) | (q.y & 0xFFFF0000u), x.z);
            } else if (wd < 15) {
                o = x;
            } else {
                o = make_uint4(q.x, x.x, 0, 0);
            }
            ae_nt_store(reinterpret_cast<uint4*>(&A.log[used + at_pos]) + wd, o);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t x = __shfl_xor(ts_min, off), y = __shfl_xor(ts_max, off);
        ts_min = x < ts_min ? x : ts_min;
        ts_max = y > ts_max ? y : ts_max;
    }
    if (lane == 0 && bal) {
        atomicMin(&ts_lds[0], ts_min);
        atomicMax(&ts_lds[1], ts_max);
    }
    __syncthreads();
    if (tid != 0) return;
    if (ts_lds[1]) {
        atomicMin(&A.slice_ts[0], ts_lds[0]);
        atomicMax(&A.slice_ts[1], ts_lds[1]);
    }
    __threadfence();
    if (atomicAdd(A.done, 1u) != gridDim.x - 1) return;
    __threadfence();
    volatile unsigned long long* sts = A.slice_ts;
    const uint64_t first = sts[0], last = sts[1];
    if (all) {
        if (used && first <= A.state[1]) A.state[2] = 1;
        if (last > A.state[1]) A.state[1] = last;
        A.state[0] = used + all;
    }
    sts[0] = ~0ull;
    sts[1] = 0;
    *A.done = 0;
}

// ---- get_change_events ---------------------------------------------------------------------

// The first log position with timestamp >= lo, and the first with timestamp > hi.
__global__ void ae_bounds(const tb_account_event_t* log, uint64_t n, uint64_t lo, uint64_t hi,
                          unsigned long long* out) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t a = 0, b = n;
    while (a < b) {
        const uint64_t mid = (a + b) >> 1;
        if (log[mid].timestamp < lo) a = mid + 1;
        else b = mid;
    }
    out[0] = a;
    b = n;
    while (a < b) {
        const uint64_t mid = (a + b) >> 1;
        if (log[mid].timestamp <= hi) a = mid + 1;
        else b = mid;
    }
    out[1] = a;
}

// get_change_event (:3424-3527): the AccountEvent joined with its transfer and both accounts
// (immutable fields: user data, code, timestamps).
__global__ void ae_change_events(Tables T, const tb_account_event_t* log, const AeRef* refs,
                                 uint64_t start, uint32_t count, tb_change_event_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const tb_account_event_t& e = log[start + i];
    const AeRef r = refs[start + i];
    const tb_transfer_t& t = T.tr_rows[r.transfer_row];
    const tb_account_t& dr = T.acc_rows[r.dr_row];
    const tb_account_t& cr = T.acc_rows[r.cr_row];
    tb_change_event_t o;
    o.transfer_id = t.id;
    o.transfer_amount = e.amount;
    o.transfer_pending_id = t.pending_id;
    o.transfer_user_data_128 = t.user_data_128;
    o.transfer_user_data_64 = t.user_data_64;
    o.transfer_user_data_32 = t.user_data_32;
    o.transfer_timeout = t.timeout;
    o.transfer_code = t.code;
    o.transfer_flags = t.flags;
    o.ledger = e.ledger;
    o.type = e.transfer_pending_status == TB_PENDING_NONE      ? TB_CHANGE_SINGLE_PHASE
             : e.transfer_pending_status == TB_PENDING_PENDING ? TB_CHANGE_TWO_PHASE_PENDING
             : e.transfer_pending_status == TB_PENDING_POSTED  ? TB_CHANGE_TWO_PHASE_POSTED
             : e.transfer_pending_status == TB_PENDING_VOIDED  ? TB_CHANGE_TWO_PHASE_VOIDED
                                                               : TB_CHANGE_TWO_PHASE_EXPIRED;
    for (int j = 0; j < 39; j++) o.reserved[j] = 0;
    o.debit_account_id = dr.id;
    o.debit_account_debits_pending = e.dr_debits_pending;
    o.debit_account_debits_posted = e.dr_debits_posted;
    o.debit_account_credits_pending = e.dr_credits_pending;
    o.debit_account_credits_posted = e.dr_credits_posted;
    o.debit_account_user_data_128 = dr.user_data_128;
    o.debit_account_user_data_64 = dr.user_data_64;
    o.debit_account_user_data_32 = dr.user_data_32;
    o.debit_account_code = dr.code;
    o.debit_account_flags = e.dr_account_flags;
    o.credit_account_id = cr.id;
    o.credit_account_debits_pending = e.cr_debits_pending;
    o.credit_account_debits_posted = e.cr_debits_posted;
    o.credit_account_credits_pending = e.cr_credits_pending;
    o.credit_account_credits_posted = e.cr_credits_posted;
    o.credit_account_user_data_128 = cr.user_data_128;
    o.credit_account_user_data_64 = cr.user_data_64;
    o.credit_account_user_data_32 = cr.user_data_32;
    o.credit_account_code = cr.code;
    o.credit_account_flags = e.cr_account_flags;
    o.timestamp = e.timestamp;
    o.transfer_timestamp = t.timestamp;
    o.debit_account_timestamp = dr.timestamp;
    o.credit_account_timestamp = cr.timestamp;
    out[i] = o;
}

// ---- Log order repair -------------------------------------------------------------------------
//
// The log is a sequence of appended blocks, each in timestamp order; an imported transfer (whose
// timestamp precedes a pulse's expiries already in the log) breaks the order between blocks.
// ae_sort_log (executor) restores it by merging the log's natural runs: ae_run_flags marks each
// run's first position (a timestamp below its predecessor's), a selection lists the runs, and each
// ae_merge_pass merges runs 2j and 2j + 1 (every lane finds its first output's split by a merge-path
// binary search, then merges kMergePer outputs), ceil(log2(runs)) passes; the resulting
// permutation gathers the records and references (ae_permute). Timestamps are unique, so the
// order is total (no library sort).
__global__ void ae_sort_keys(const tb_account_event_t* log, uint64_t n, uint64_t* keys,
                             uint32_t* idx, uint8_t* run_first) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t ts = log[i].timestamp;
    keys[i] = ts;
    idx[i] = uint32_t(i);
    run_first[i] = i == 0 || ts < log[i - 1].timestamp;
}

constexpr uint32_t kMergePer = 8;
// starts[0 .. runs]: the runs' first positions, starts[runs] = n.
__global__ void ae_merge_pass(const uint64_t* key, const uint32_t* val, const uint64_t* starts,
                              uint32_t runs, uint64_t n, uint64_t* key_out, uint32_t* val_out) {
    uint64_t d = (uint64_t(blockIdx.x) * blockDim.x + threadIdx.x) * kMergePer;
    if (d >= n) return;
    const uint64_t d_end = d + kMergePer < n ? d + kMergePer : n;
    // the pair of runs holding output d: the last p with starts[2p] <= d
    const uint32_t pairs = (runs + 1) / 2;
    uint32_t lo = 0, hi = pairs;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (starts[2 * mid] <= d) lo = mid;
        else hi = mid;
    }
    for (uint32_t p = lo; d < d_end && p < pairs; p++) {
        const uint64_t a0 = starts[2 * p];
        const uint64_t a1 = starts[2 * p + 1 < runs ? 2 * p + 1 : runs];
        const uint64_t b1 = starts[2 * p + 2 < runs ? 2 * p + 2 : runs];
        const uint64_t b0 = a1, la = a1 - a0, lb = b1 - b0;
        // of the pair's first k outputs, the number taken from run a
        const uint64_t k = d - a0;
        uint64_t l = k > lb ? k - lb : 0, h = k < la ? k : la;
        while (l < h) {
            const uint64_t m = (l + h) >> 1;
            if (key[b0 + (k - 1 - m)] < key[a0 + m]) h = m;
            else l = m + 1;
        }
        uint64_t i = a0 + l, j = b0 + (k - l);
        const uint64_t stop = d_end < b1 ? d_end : b1;
        for (; d < stop; d++) {
            const bool take_a = j >= b1 || (i < a1 && key[i] < key[j]);
            const uint64_t src = take_a ? i++ : j++;
            key_out[d] = key[src];
            val_out[d] = val[src];
        }
    }
}
__global__ void ae_permute(const tb_account_event_t* log, const AeRef* refs, const uint32_t* idx,
                           uint64_t n, tb_account_event_t* log_out, AeRef* refs_out) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    log_out[i] = log[idx[i]];
    refs_out[i] = refs[idx[i]];
}

}  // namespace tbg
