// Device kernels of the executor (host orchestration in executor.hip).
//
// create_transfers, per call of N events:
//
//   tr_ingest    one lane per event, one read of the 128-byte event: the reference's checks in
//                their order (state_machine.zig:3029-3104, :3719-3873) up to the first check that
//                depends on in-call state; claim of the event's id in the transfer id table
//                (earliest duplicate wins); debit/credit account rows; `closable` marks (closing
//                transfers, voids). Outcome per event: DONE (result fixed), FAST (commits in
//                parallel: the transfer row and result are written here), SLOW (ordered replay,
//                marks its accounts `hot`).
//   tr_commit    one lane per event: re-validates what ingest could only know provisionally
//                (still the earliest holder of its id, no hot/closable account, no post/void in
//                the call for pending-with-timeout) and commits FAST events (status, liveness,
//                expires_at entry, pulse_next_timestamp, balance deltas) or demotes them to SLOW;
//                finalises the id slots of DONE events (orphan / tombstone).
//   balances     FAST balance deltas as (account field, amount) items summed per account field in
//                LDS (the balance window, the buckets, or per-workgroup hash tables: bal_hash_apply)
//                and added to the rows; sparse key spaces and small calls use u128 atomics.
//   replay       the SLOW events in serial order on one lane (replay.hpp), then their id slots.
//
// Exactness argument: DESIGN.md §4.
#pragma once

#include "device_common.hpp"
#include "replay.hpp"
#include "prims.hpp"

namespace tbg {

constexpr int kBlock = 256;
constexpr uint32_t kIngestWgPerCu = 4;  // tr_ingest's occupancy (workgroups per CU, launch bounds)

// Bucketed balance path: keys (account row * 4 + field) fall into buckets of 8192 consecutive
// keys (2048 accounts); a call uses it when 4 * accounts <= kBucketsMax * 8192.
constexpr uint32_t kBucketShift = 13;
constexpr uint32_t kBucketKeys = 1u << kBucketShift;
constexpr uint32_t kBucketsMax = 128;
// Items per accumulate block: with key_bits >= 16 every packed amount is < 2^48, so a slice's
// u64 LDS sums stay below 2^63.
constexpr uint32_t kSliceItems = 32768;

__device__ inline void count_stat(DevScalars* s, int which, bool pred) {
    unsigned long long mask = __ballot(pred);
    if ((threadIdx.x & 63) == 0 && mask)
        atomicAdd(&s->stats[which], (unsigned long long)__popcll(mask));
}

__device__ inline void set_flag_any(DevScalars* s, bool pred, unsigned int flag) {
    if (__any(pred) && (threadIdx.x & 63) == 0) atomicOr(&s->flags, flag);
}

// Block-wide reduction (kBlock threads, every thread participates); the result is returned to
// every thread. Keeps call-wide counters at one atomic per block: same-address atomics from every
// wave serialise at the memory side and cost milliseconds at 10^7 events.
struct OpAdd {
    template <typename V>
    __device__ V operator()(V a, V b) const { return a + b; }
};
struct OpMax {
    template <typename V>
    __device__ V operator()(V a, V b) const { return a > b ? a : b; }
};
struct OpOr {
    template <typename V>
    __device__ V operator()(V a, V b) const { return a | b; }
};

template <typename V, typename Op>
__device__ inline V block_reduce(V v, Op op) {
    __shared__ V lds[kBlock / 64];
    for (int off = 32; off > 0; off >>= 1) v = op(v, __shfl_xor(v, off));
    if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
    __syncthreads();
    V r = lds[0];
    for (int i = 1; i < int(blockDim.x >> 6); i++) r = op(r, lds[i]);  // (kBlock or fewer lanes)
    __syncthreads();
    return r;
}

// Grid-stride kernels run at most this many blocks (16 per CU on 256 CUs).
constexpr uint32_t kMaxGrid = 4096;

template <typename Event>
__device__ inline uint64_t ts_event_of(const Call<Event>& c, uint32_t b, uint32_t k) {
    if (c.event_ts) return c.event_ts[k];
    return c.batch_ts[b] - c.batch_ends[b] + k + 1;
}

template <typename Event>
__device__ inline uint32_t batch_start_of(const Call<Event>& c, uint32_t b) {
    return b == 0 ? 0 : c.batch_ends[b - 1];
}

__device__ inline uint32_t row32(uint64_t r) { return r == kNone ? kNone32 : uint32_t(r); }

// ================================ create_transfers ==========================================

// What the checks after the id lookup read of an account: a snapshot taken by ingest. Account
// existence, ledger and limit flags are static within a create_transfers call; `closed` and the
// balances are not, and every decision that reads them is re-validated by tr_commit.
struct AccSnap {
    uint32_t row;         // kNone32: not found
    uint32_t ledger;
    uint16_t flags;
    uint64_t hi_pending;  // .hi of the pending / posted balance the event adds to
    uint64_t hi_posted;   // (debit side: debits_*, credit side: credits_*)
};

__device__ inline AccSnap acc_snap_load(const tb_account_t* a, uint32_t row, bool debit) {
    AccSnap s;
    s.row = row;
    // ledger (112), code (116), flags (118): one 8-byte word.
    const uint64_t lcf = *reinterpret_cast<const uint64_t*>(reinterpret_cast<const uint8_t*>(a) + 112);
    s.ledger = uint32_t(lcf);
    s.flags = uint16_t(lcf >> 48);
    s.hi_pending = debit ? a->debits_pending.hi : a->credits_pending.hi;
    s.hi_posted = debit ? a->debits_posted.hi : a->credits_posted.hi;
    return s;
}

// An account as the checks see it, from its index entry (one 16-byte load per probe step). An
// entry with no hazard bit names an open account whose balances are all < 2^126 and whose ledger
// fits the entry: the snapshot is complete without the row (balance hi words read as 0, which
// classify_after_lookup only compares with 2^62). Otherwise the row is read.
__device__ inline AccSnap acc_lookup_snap(const Tables& T, const tb_uint128_t& id, bool valid,
                                          bool debit) {
    AccSnap a;
    a.row = kNone32;
    a.ledger = 0;
    a.flags = 0;
    a.hi_pending = a.hi_posted = 0;
    if (!valid) return a;
    AccEntry e;
    if (acc_index_find(T.acc_index, T.acc_rows, id, &e) == kNone) return a;
    const uint32_t row = e.ref - 1;
    if (meta_hazard(e.meta)) return acc_snap_load(&T.acc_rows[row], row, debit);
    a.row = row;
    a.ledger = meta_ledger(e.meta);
    a.flags = meta_flags(e.meta);
    return a;
}

// The same lookup split in two: issue both candidate entries' loads (unconditionally, entry 0 for
// an id that is not looked up), then match. Ingest issues the id claim's CAS and both accounts'
// four loads back to back, so the common event pays one memory round trip, not three.
struct AccProbe {
    uint4 v1, v2;
};
__device__ inline AccProbe acc_probe_issue(const AccIndex& x, const tb_uint128_t& id, bool valid) {
    const uint64_t s1 = valid ? acc_entry_h1(id) & x.mask : 0;
    const uint64_t s2 = valid ? acc_entry_h2(id) & x.mask : 0;
    AccProbe p;
    p.v1 = *reinterpret_cast<const uint4*>(&x.entries[s1]);
    p.v2 = *reinterpret_cast<const uint4*>(&x.entries[s2]);
    return p;
}
__device__ inline AccSnap acc_probe_snap(const Tables& T, const AccProbe& p, const tb_uint128_t& id,
                                         bool valid, bool debit) {
    AccSnap a;
    a.row = kNone32;
    a.ledger = 0;
    a.flags = 0;
    a.hi_pending = a.hi_posted = 0;
    if (!valid) return a;
    uint4 v;
    if (acc_entry_match(p.v1, T.acc_rows, id)) v = p.v1;
    else if (acc_entry_match(p.v2, T.acc_rows, id)) v = p.v2;
    else return a;
    const uint32_t row = v.z - 1;
    if (meta_hazard(v.w)) return acc_snap_load(&T.acc_rows[row], row, debit);
    a.row = row;
    a.ledger = meta_ledger(v.w);
    a.flags = meta_flags(v.w);
    return a;
}

// ---- post / void on the parallel path ----------------------------------------------------------
//
// A post/void (post_or_void_pending_transfer, :4053-4300) of a committed pending transfer X whose
// status is `pending` at the call's start is decided by the call's start state alone -- every check
// reads X's immutable row, its TransferPending status, the event and the accounts' `closed` flags
// -- unless an earlier event of the call changes X's status, which only a post/void of X does. So
// the earliest post/void of X in the call (a claim on X's id, smallest event index wins) may be FAST
// when it would succeed: its effects are X's status (posted / voided, written once), the accounts'
// balance deltas (pending -= X.amount, posted += amount: u128 atomics, commutative), its own row,
// and a pulse_next_timestamp reset recorded at the event (pnt_resolve). tr_commit confirms the claim
// and the usual demotions (hot / closable accounts, duplicates). Later post/voids of X replay after
// the FAST one's effects, exactly as in call order.
__device__ inline uint64_t pv_home(const Call<tb_transfer_t>& c, const tb_uint128_t& x) {
    return mix64(x.lo ^ mix64(x.hi ^ 0x5851F42D4C957F2Dull)) & c.pv_mask;
}
// Claims pending id `x` for event k (keeping the earliest claimant).
__device__ inline void pv_claim(const Call<tb_transfer_t>& c, uint32_t k, const tb_uint128_t& x) {
    const unsigned long long mine = (uint64_t(c.epoch) << 32) | (k + 1);
    uint64_t s = pv_home(c, x);
    for (uint64_t n = 0; n <= c.pv_mask; n++) {
        unsigned long long w = c.pv_slots[s];
        while ((w >> 32) != c.epoch) {  // free (another call's): take it
            const unsigned long long o = atomicCAS(&c.pv_slots[s], w, mine);
            if (o == w) return;
            w = o;
        }
        if (u128_eq(c.events[uint32_t(w) - 1].pending_id, x)) {
            if (mine < w) atomicMin(&c.pv_slots[s], mine);
            return;
        }
        s = (s + 1) & c.pv_mask;
    }
}
// Is event k the earliest post/void of pending id `x` in the call?
__device__ inline bool pv_first(const Call<tb_transfer_t>& c, uint32_t k, const tb_uint128_t& x) {
    uint64_t s = pv_home(c, x);
    for (uint64_t n = 0; n <= c.pv_mask; n++) {
        const unsigned long long w = c.pv_slots[s];
        if ((w >> 32) != c.epoch) return false;
        if (u128_eq(c.events[uint32_t(w) - 1].pending_id, x)) return uint32_t(w) == k + 1;
        s = (s + 1) & c.pv_mask;
    }
    return false;
}

// The earliest post/void of pending id `x` in the call (kNone32: no claim this call).
__device__ inline uint32_t pv_winner(const Call<tb_transfer_t>& c, const tb_uint128_t& x) {
    uint64_t s = pv_home(c, x);
    for (uint64_t n = 0; n <= c.pv_mask; n++) {
        const unsigned long long w = c.pv_slots[s];
        if ((w >> 32) != c.epoch) return kNone32;
        if (u128_eq(c.events[uint32_t(w) - 1].pending_id, x)) return uint32_t(w) - 1;
        s = (s + 1) & c.pv_mask;
    }
    return kNone32;
}

// The committed pending transfer a post/void names (kNone: not a committed, un-orphaned row).
__device__ inline uint64_t pv_pending_row(const Tables& T, const Call<tb_transfer_t>& c,
                                          const tb_uint128_t& pending_id) {
    const uint64_t ps = transfer_slot_find(T, c, pending_id);
    if (ps == kNone) return kNone;
    const uint64_t w = T.tr.slots[ps];
    const uint64_t r = (w & kRefMask) - 1;
    if (r >= c.row_base || (w & kOrphanBit)) return kNone;
    return r;
}

struct PvFast {
    uint32_t dr, cr;  // the pending transfer's account rows
    uint64_t amount;  // the amount posted (void: 0)
    uint64_t prow;    // the pending transfer's row
};

// post_or_void_pending_transfer's checks (:4053-4246) for a fresh, unique id; DONE where the
// outcome is fixed by the call's start state, FAST where it succeeds if no earlier event of the
// call posts / voids the same pending transfer (tr_commit: pv_first), else SLOW.
__device__ inline uint8_t classify_post_void(const Tables& T, const Call<tb_transfer_t>& c,
                                             uint32_t k, uint64_t ts_event, const tb_transfer_t& t,
                                             uint32_t* status, PvFast* out) {
    const uint16_t f = t.flags;
    uint32_t st = 0;
    if ((f & TB_TRANSFER_POST_PENDING) && (f & TB_TRANSFER_VOID_PENDING))
        st = TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    else if (f & (TB_TRANSFER_PENDING | TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT |
                  TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT))
        st = TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    else if (u128_is_zero(t.pending_id)) st = TB_CT_PENDING_ID_MUST_NOT_BE_ZERO;
    else if (u128_is_max(t.pending_id)) st = TB_CT_PENDING_ID_MUST_NOT_BE_INT_MAX;
    else if (u128_eq(t.pending_id, t.id)) st = TB_CT_PENDING_ID_MUST_BE_DIFFERENT;
    else if (t.timeout != 0) st = TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
    if (st) {
        *status = st;
        return kClassDone;
    }
    // (not found now: an earlier event of the call may create it -- the replay decides)
    const uint64_t ps = transfer_slot_find(T, c, t.pending_id);
    if (ps == kNone) return kClassSlow;
    const uint64_t pw = T.tr.slots[ps];
    const uint64_t pr = (pw & kRefMask) - 1;
    if (pr >= c.row_base) return kClassSlow;  // created in this call
    if (pw & kOrphanBit) st = TB_CT_PENDING_TRANSFER_NOT_FOUND;
    const tb_transfer_t& p = T.tr_rows[pr];  // committed rows are immutable
    if (!st && !(p.flags & TB_TRANSFER_PENDING)) st = TB_CT_PENDING_TRANSFER_NOT_PENDING;
    if (st) {
        *status = st;
        return kClassDone;
    }
    if (!u128_is_zero(t.debit_account_id) && !u128_eq(t.debit_account_id, p.debit_account_id))
        st = TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID;
    else if (!u128_is_zero(t.credit_account_id) && !u128_eq(t.credit_account_id, p.credit_account_id))
        st = TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID;
    else if (t.ledger > 0 && t.ledger != p.ledger) st = TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER;
    else if (t.code > 0 && t.code != p.code) st = TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CODE;
    const u128 p_amount = U(p.amount);
    const u128 amount = (f & TB_TRANSFER_VOID_PENDING)
                            ? (U(t.amount) == 0 ? p_amount : U(t.amount))
                            : (U(t.amount) == kU128Max ? p_amount : U(t.amount));
    if (!st && amount > p_amount) st = TB_CT_EXCEEDS_PENDING_TRANSFER_AMOUNT;
    else if (!st && (f & TB_TRANSFER_VOID_PENDING) && amount < p_amount)
        st = TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT;
    if (!st) {
        switch (T.tr_status[pr]) {  // no event of the call makes a resolved transfer pending
            case TB_PENDING_PENDING: break;
            case TB_PENDING_POSTED: st = TB_CT_PENDING_TRANSFER_ALREADY_POSTED; break;
            case TB_PENDING_VOIDED: st = TB_CT_PENDING_TRANSFER_ALREADY_VOIDED; break;
            default: st = TB_CT_PENDING_TRANSFER_EXPIRED; break;
        }
    }
    if (st) {
        *status = st;
        return kClassDone;
    }
    // From here the outcome depends on the status an earlier post/void of the call may set, and on
    // `closed`: only the success path is parallel.
    if (p.timeout != 0 && p.timestamp + uint64_t(p.timeout) * TB_NS_PER_S <= ts_event)
        return kClassSlow;  // pending_transfer_expired, unless an earlier event resolved it
    if (p_amount >> 64) return kClassSlow;
    if ((f & TB_TRANSFER_VOID_PENDING) &&
        (p.flags & (TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT)))
        return kClassSlow;  // un-closes accounts (closable)
    AccEntry ed, ec;
    if (acc_index_find(T.acc_index, T.acc_rows, p.debit_account_id, &ed) == kNone ||
        acc_index_find(T.acc_index, T.acc_rows, p.credit_account_id, &ec) == kNone)
        return kClassSlow;
    // (a hazard: possibly closed, balances near 2^126, or a wide entry -- the replay decides)
    if (meta_hazard(ed.meta) || meta_hazard(ec.meta)) return kClassSlow;
    out->dr = ed.ref - 1;
    out->cr = ec.ref - 1;
    out->amount = (f & TB_TRANSFER_POST_PENDING) ? uint64_t(amount) : 0;
    out->prow = pr;
    return kClassFast;
}

// The checks after the id lookup (create_transfer, :3727-3873), on the ingest snapshot. `w` is
// the word of the id's slot as this event observed it.
// The narrow fields of a staged event, taken from its LDS image with 16-byte reads (words 3, 6, 7:
// amount, timeout, ledger / code / flags / timestamp). Read one by one at the image's 144-byte
// stride, the 4- and 8-byte fields put 4 lanes of a 32-lane group on one bank
// (SQ_LDS_BANK_CONFLICT, profiles/r03_final_pmc); the 16-byte reads are conflict-free.
struct EvNarrow {
    const uint4* w;  // the event's LDS image (16-byte words)
    __device__ uint16_t flags() const { return uint16_t(w[7].y >> 16); }
    __device__ uint16_t code() const { return uint16_t(w[7].y); }
    __device__ uint32_t ledger() const { return w[7].x; }
    __device__ uint32_t timeout() const { return w[6].w; }
    __device__ uint64_t timestamp() const { const uint4 q = w[7]; return (uint64_t(q.w) << 32) | q.z; }
    __device__ uint64_t amount_lo() const { const uint4 q = w[3]; return (uint64_t(q.y) << 32) | q.x; }
    __device__ uint64_t amount_hi() const { const uint4 q = w[3]; return (uint64_t(q.w) << 32) | q.z; }
};
__device__ inline EvNarrow ev_narrow(const tb_transfer_t& t) {
    return EvNarrow{reinterpret_cast<const uint4*>(&t)};
}
static_assert(offsetof(tb_transfer_t, amount) == 48 && offsetof(tb_transfer_t, timeout) == 108 &&
                  offsetof(tb_transfer_t, ledger) == 112 && offsetof(tb_transfer_t, code) == 116 &&
                  offsetof(tb_transfer_t, flags) == 118 && offsetof(tb_transfer_t, timestamp) == 120,
              "Transfer layout");

__device__ inline uint8_t classify_after_lookup(const Tables& T, const Call<tb_transfer_t>& c,
                                                uint32_t k, uint64_t ts_event,
                                                const tb_transfer_t& t, const EvNarrow& tn,
                                                uint64_t w,
                                                const AccSnap& dr, const AccSnap& cr,
                                                uint32_t* status, uint64_t* ts_out,
                                                uint8_t* info, PvFast* pv) {
    const uint16_t f = tn.flags();
    const uint64_t r = (w & kRefMask) - 1;
    if (r < c.row_base) {  // a committed id: the result is final for every event of the call
        if (w & kOrphanBit) {
            *status = TB_CT_ID_ALREADY_FAILED;
            return kClassDone;
        }
        const tb_transfer_t& e = T.tr_rows[r];  // committed rows are immutable
        const tb_transfer_t* p = nullptr;
        if (f == e.flags && U(t.pending_id) == U(e.pending_id) && tn.timeout() == e.timeout &&
            (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING))) {
            const uint64_t ps = transfer_slot_find(T, c, t.pending_id);
            if (ps == kNone) return kClassSlow;
            const uint64_t pw = T.tr.slots[ps];
            const uint64_t pr = (pw & kRefMask) - 1;
            if (pr >= c.row_base || (pw & kOrphanBit)) return kClassSlow;
            p = &T.tr_rows[pr];
        }
        *status = create_transfer_exists(t, e, p, ts_out);
        return kClassDone;
    }
    if (r != c.row_base + k) return kClassSlow;  // a later duplicate of an in-call id
    // Provisionally the first occurrence: every DONE below is valid only if that holds.
    *info |= kInfoPostLookup;
    if (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING))
        return c.pv_slots ? classify_post_void(T, c, k, ts_event, t, status, pv) : kClassSlow;
    uint32_t st = 0;
    if (u128_is_zero(t.debit_account_id)) st = TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    else if (u128_is_max(t.debit_account_id)) st = TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    else if (u128_is_zero(t.credit_account_id)) st = TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    else if (u128_is_max(t.credit_account_id)) st = TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    else if (u128_eq(t.credit_account_id, t.debit_account_id)) st = TB_CT_ACCOUNTS_MUST_BE_DIFFERENT;
    else if (!u128_is_zero(t.pending_id)) st = TB_CT_PENDING_ID_MUST_BE_ZERO;
    else if (!(f & TB_TRANSFER_PENDING) && tn.timeout() != 0)
        st = TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
    else if (!(f & TB_TRANSFER_PENDING) &&
             (f & (TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT)))
        st = TB_CT_CLOSING_TRANSFER_MUST_BE_PENDING;
    else if (tn.ledger() == 0) st = TB_CT_LEDGER_MUST_NOT_BE_ZERO;
    else if (tn.code() == 0) st = TB_CT_CODE_MUST_NOT_BE_ZERO;
    else if (dr.row == kNone32) st = TB_CT_DEBIT_ACCOUNT_NOT_FOUND;
    else if (cr.row == kNone32) st = TB_CT_CREDIT_ACCOUNT_NOT_FOUND;
    else if (dr.ledger != cr.ledger) st = TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    else if (tn.ledger() != dr.ledger) st = TB_CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;
    if (st) {
        *status = st;
        return kClassDone;
    }
    // From here on every outcome follows the `closed` check: a DONE is confirmed by tr_commit
    // against the call's closable marks, a FAST against closable and hot marks.
    *info |= kInfoClosedDep;
    const bool balancing_or_closing =
        (f & (TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT |
              TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT)) != 0;
    // Overflow is impossible when every balance is < 2^126 and every amount < 2^64.
    constexpr uint64_t kHiLimit = 1ull << 62;
    const bool overflow_possible = tn.amount_hi() != 0 || dr.hi_pending >= kHiLimit ||
                                   dr.hi_posted >= kHiLimit || cr.hi_pending >= kHiLimit ||
                                   cr.hi_posted >= kHiLimit;
    const bool limited = (dr.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) ||
                         (cr.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS);
    if ((dr.flags | cr.flags) & TB_ACCOUNT_CLOSED) {
        // A `closed` DONE that tr_commit demotes (an event of the call may reopen the account)
        // replays without hot marks on its accounts, so it may only be one whose later checks
        // read no order-dependent balance.
        if (balancing_or_closing || overflow_possible || limited) return kClassSlow;
        *status = (dr.flags & TB_ACCOUNT_CLOSED) ? TB_CT_DEBIT_ACCOUNT_ALREADY_CLOSED
                                                 : TB_CT_CREDIT_ACCOUNT_ALREADY_CLOSED;
        return kClassDone;
    }
    if (balancing_or_closing || overflow_possible) return kClassSlow;
    if (ts_event + (uint64_t)tn.timeout() * TB_NS_PER_S > TB_TIMESTAMP_MAX) {
        *status = TB_CT_OVERFLOWS_TIMEOUT;
        return kClassDone;
    }
    if (limited) return kClassSlow;
    if (f & TB_TRANSFER_PENDING) *info |= kInfoPending;
    if (tn.timeout() > 0) *info |= kInfoTimeout;
    return kClassFast;
}

// Does a FAST event's amount fit its call's balance item(s)? (Else tr_commit adds it with u128
// atomics.)
// A pair item's amount field (63 - 2 pair_shift bits); all ones marks a *wide* item, whose
// amount the balance window reads from the event's record (ev_amount).
__device__ inline uint64_t pair_amount_mask(uint32_t ps) { return (1ull << (63 - 2 * ps)) - 1; }
__device__ inline bool item_packable(const Call<tb_transfer_t>& c, uint64_t amount) {
    return c.pair_shift ? amount < pair_amount_mask(c.pair_shift)
                        : (amount >> (64 - c.key_bits)) == 0;
}

__device__ inline void ingest_store_result(tb_create_result_t* p, const tb_create_result_t& r) {
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
    const v4u v = {uint32_t(r.timestamp), uint32_t(r.timestamp >> 32), r.status, r.reserved};
    __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
}

// Balance-delta item: key = account_row * 4 + field (0 dp, 1 dpo, 2 cp, 3 cpo).
__device__ inline tb_uint128_t* account_field(tb_account_t* rows, uint32_t key) {
    tb_account_t* a = &rows[key >> 2];
    return reinterpret_cast<tb_uint128_t*>(reinterpret_cast<uint8_t*>(a) + 16 + 16 * (key & 3));
}

// A FAST event's balance deltas as u128 atomics on its two rows (`undo`: subtracted again, for a
// demoted event of a call without balance items, whose deltas ingest applied). An add that
// takes a balance's high word to >= 2^62 raises the account's kHazardHigh bit; a subtraction
// leaves the bits (they are a conservative, set-only summary).
__device__ inline void apply_fast_deltas(const Tables& T, uint32_t dr, uint32_t cr, bool pending,
                                         uint64_t amount, bool undo) {
    if (!amount) return;
    tb_uint128_t* fd = account_field(T.acc_rows, dr * 4 + (pending ? 0 : 1));
    tb_uint128_t* fc = account_field(T.acc_rows, cr * 4 + (pending ? 2 : 3));
    if (undo) {
        atomic_sub_u128(fd, amount);
        atomic_sub_u128(fc, amount);
        return;
    }
    if (atomic_add_u128(fd, amount) >= kHazardHiLimit)
        acc_hazard_set(T.acc_index, T.acc_entry_of, dr, kHazardHigh);
    if (atomic_add_u128(fc, amount) >= kHazardHiLimit)
        acc_hazard_set(T.acc_index, T.acc_entry_of, cr, kHazardHigh);
}

// One event of tr_ingest, `t` being the event as staged in LDS; returns the call flags it raises
// (kFlag*). The row store is done by the caller (the whole wave's rows at once, coalesced).
//
// Memory-level parallelism: the id claim (one CAS at the home slot, no preceding load) and the two
// account-index loads are independent and issue together; the common event pays one round trip.
__device__ inline unsigned int ingest_event(const Tables& T, const Call<tb_transfer_t>& c,
                                            uint32_t k, const tb_transfer_t& t,
                                            bool batch_imported, uint64_t ts_event,
                                            bool prev_linked, uint64_t* fast_ts,
                                            unsigned int* bucket_hist) {
    const EvNarrow tn = ev_narrow(t);
    bool imported = false, post_void = false, dup = false, closable = false, hot = false;
    bool need_commit = false, chain_fast = false, ae_slow = false, wide_item = false;
    bool no_lanes = false;
    if (c.pnt_force) c.pnt_call[k] = 0;  // (sharded calls record every update: none yet)
    const uint16_t f = tn.flags();
    imported = (f & TB_TRANSFER_IMPORTED) != 0;
    post_void = (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) != 0;
    const tb_uint128_t id = t.id;
    const bool valid_id = !u128_is_zero(id) && !u128_is_max(id);
    // prev_linked: the previous event of the same batch is linked.
    const bool chain = (f & TB_TRANSFER_LINKED) || prev_linked;

    uint32_t status = 0;
    uint64_t ts_out = ts_event;
    uint8_t info = 0, cls = kClassSlow;
    bool pre_done = false, pre_fail = false;
    if (!c.force_replay) {
        // execute_create's per-event checks before create_transfer (:3052-3081) and the
        // checks before the id lookup (:3729-3733): independent of every table.
        if (batch_imported != imported) {
            status = imported ? TB_CT_IMPORTED_EVENT_NOT_EXPECTED : TB_CT_IMPORTED_EVENT_EXPECTED;
            pre_done = true;
        } else if (!imported && tn.timestamp() != 0) {
            status = TB_CT_TIMESTAMP_MUST_BE_ZERO;
            pre_done = true;
        } else if (!imported && (f & TB_TRANSFER_PADDING_MASK)) {
            status = TB_CT_RESERVED_FLAG;
            pre_done = true;
        } else if (!imported && !valid_id) {
            status = u128_is_zero(id) ? TB_CT_ID_MUST_NOT_BE_ZERO : TB_CT_ID_MUST_NOT_BE_INT_MAX;
            pre_done = true;
        }
        // A failing event of a linked chain fails the chain: the replay decides it.
        if (chain && pre_done) {
            pre_done = false;
            pre_fail = true;
        }
    }
    uint64_t slot = kNone;
    AccSnap dr, cr;
    dr.row = cr.row = kNone32;
    PvFast pv{kNone32, kNone32, 0, kNone};
    if (pre_done) {
        cls = kClassDone;
    } else {
        const tb_transfer_t* ev = c.events;
        const tb_transfer_t* rows = T.tr_rows;
        const uint64_t base = c.row_base;
        const uint64_t tref = (base + k + 1) | id_tag(id);
        const uint64_t s_id = hash_id(id) & T.tr.mask;
        // The claim: a CAS at the home slot; only a taken home slot continues the probe.
        uint64_t w_slot = tref;
        const tb_uint128_t dr_id = t.debit_account_id, cr_id = t.credit_account_id;
        const bool vd = !u128_is_zero(dr_id) && !u128_is_max(dr_id);
        const bool vc = !u128_is_zero(cr_id) && !u128_is_max(cr_id);
        uint64_t w_seen = kEmpty;
        if (valid_id)
            w_seen = atomicCAS(&T.tr.slots[s_id], (unsigned long long)kEmpty,
                               (unsigned long long)tref);
        {
            // Most entries sit at their first candidate (load <= 0.25): one 16-byte load per
            // account; the second candidate only for the lanes whose first one missed.
            const AccIndex& x = T.acc_index;
            const uint64_t d1 = vd ? acc_entry_h1(dr_id) & x.mask : 0;
            const uint64_t c1 = vc ? acc_entry_h1(cr_id) & x.mask : 0;
            AccProbe pd, pc;
            pd.v1 = *reinterpret_cast<const uint4*>(&x.entries[d1]);
            pc.v1 = *reinterpret_cast<const uint4*>(&x.entries[c1]);
            const bool dm = vd && !acc_entry_match(pd.v1, T.acc_rows, dr_id);
            const bool cm = vc && !acc_entry_match(pc.v1, T.acc_rows, cr_id);
            pd.v2 = dm ? *reinterpret_cast<const uint4*>(&x.entries[acc_entry_h2(dr_id) & x.mask])
                       : make_uint4(0, 0, 0, 0);
            pc.v2 = cm ? *reinterpret_cast<const uint4*>(&x.entries[acc_entry_h2(cr_id) & x.mask])
                       : make_uint4(0, 0, 0, 0);
            dr = acc_probe_snap(T, pd, dr_id, vd, true);
            cr = acc_probe_snap(T, pc, cr_id, vc, false);
        }
        if (valid_id) {
            if (w_seen == kEmpty) {
                slot = s_id;  // claimed
            } else {
                slot = probe_claim_from(T.tr, id, base + k + 1, base, [=](uint64_t r) {
                    return r >= base ? ev[r - base].id : rows[r].id;
                }, &dup, s_id, w_seen);
                if (slot != kNone) w_slot = T.tr.slots[slot];
            }
            if (slot == kNone) atomicOr(&T.scalars->flags, kFlagTableFull);
            else info |= kInfoClaimed;
        }
        // Accounts whose `closed` flag an event of this call may change.
        if ((f & TB_TRANSFER_CLOSING_DEBIT) && dr.row != kNone32) {
            T.acc_closable[dr.row] = c.epoch;
            closable = true;
        }
        if ((f & TB_TRANSFER_CLOSING_CREDIT) && cr.row != kNone32) {
            T.acc_closable[cr.row] = c.epoch;
            closable = true;
        }
        if ((f & TB_TRANSFER_VOID_PENDING) && !u128_is_zero(t.pending_id) &&
            !u128_is_max(t.pending_id)) {
            const uint64_t ps = transfer_slot_find(T, c, t.pending_id);
            if (ps != kNone) {
                const uint64_t pr = (T.tr.slots[ps] & kRefMask) - 1;
                const tb_transfer_t& p = pr >= base ? ev[pr - base] : rows[pr];
                // A void un-closes only the accounts of a closing pending transfer (:4253-4262).
                // (With duplicate ids the holder found here may not be the final one; an in-call
                // closing creator marks its own accounts above.)
                const uint16_t pf = p.flags;
                if (pf & TB_TRANSFER_CLOSING_DEBIT) {
                    const uint64_t pd_row = account_find(T, p.debit_account_id);
                    if (pd_row != kNone) T.acc_closable[pd_row] = c.epoch;
                    closable = true;
                }
                if (pf & TB_TRANSFER_CLOSING_CREDIT) {
                    const uint64_t pc_row = account_find(T, p.credit_account_id);
                    if (pc_row != kNone) T.acc_closable[pc_row] = c.epoch;
                    closable = true;
                }
            }
        }
        // Every post/void claims its pending id: the earliest claimant may be FAST.
        if (post_void && c.pv_slots && !c.force_replay && !u128_is_zero(t.pending_id) &&
            !u128_is_max(t.pending_id))
            pv_claim(c, k, t.pending_id);
        if (!c.force_replay && !pre_fail && !imported && slot != kNone) {
            cls = classify_after_lookup(T, c, k, ts_event, t, tn, w_slot, dr, cr, &status, &ts_out,
                                        &info, &pv);
            // Linked chains (execute_create :3033-3207): a chain whose every event is FAST
            // creates every event -- tr_commit confirms that for the whole chain (commit_chain)
            // or demotes all of it; a chain with any other event is replayed.
            if (chain && cls != kClassFast) cls = kClassSlow;
            chain_fast = chain && cls == kClassFast;
        }
    }
    // A FAST post/void: its record names the pending transfer's accounts and the posted amount;
    // its effects are all tr_commit's (no balance items).
    const bool pv_fast = cls == kClassFast && post_void;
    if (pv_fast) {
        dr.row = pv.dr;
        cr.row = pv.cr;
    }
    info |= cls;
    // A FAST event whose balance items are packed needs no per-event record: tr_commit decodes
    // the rows and amount from the items and re-probes the slot if it has to.
    const bool lean = cls == kClassFast && !pv_fast &&
                      (c.bal_items ? item_packable(c, tn.amount_lo()) : c.lean_lookup != 0);
    c.ev_info[k] = info | (lean ? kInfoLean : 0);
    if (!lean) {
        c.ev_slot[k] = slot == kNone ? kNone32 : uint32_t(slot);
        c.ev_dr[k] = dr.row;
        c.ev_cr[k] = cr.row;
    }
    if (cls == kClassDone) {
        tb_create_result_t res;
        res.timestamp = status == TB_CT_EXISTS ? ts_out : ts_event;
        res.status = status;
        res.reserved = 0;
        c.results[k] = res;
    } else if (cls == kClassFast) {
        // Speculative commit (the row is already written): status, liveness, result and the
        // balance items. tr_commit confirms or demotes when the call raised a commit flag.
        const uint64_t row = c.row_base + k;
        const bool pending = (f & TB_TRANSFER_PENDING) != 0;
        if (pending) T.tr_status[row] = TB_PENDING_PENDING;  // fresh rows read TB_PENDING_NONE
        T.tr_live[row] = 1;
        const uint64_t amount = pv_fast ? pv.amount : tn.amount_lo();
        if (!lean) c.ev_amount[k] = amount;
        tb_create_result_t res;
        res.timestamp = ts_event;
        res.status = TB_STATUS_CREATED;
        res.reserved = 0;
        ingest_store_result(&c.results[k], res);
        if (pending && tn.timeout() > 0) need_commit = true;  // expires_at index
        if (pv_fast) {
            need_commit = true;
            c.ev_prow[k] = pv.prow;  // (tr_commit applies it without looking the pending id up)
            if (c.bal_items && c.pair_shift) c.bal_items[k] = ~0ull;
            else if (c.bal_items)
                *reinterpret_cast<uint4*>(c.bal_items + 2 * uint64_t(k)) = make_uint4(~0u, ~0u, ~0u, ~0u);
        } else if (c.bal_items && c.pair_shift) {
            const uint32_t ps = c.pair_shift;
            ae_slow = pending;  // (the AccountEvents window tracks posted balances only)
            // (too wide to pack: a wide item, its amount in ev_amount -- the event is not lean --
            // which the AccountEvents window takes with u128 sums, ae_wide_*)
            const bool packed = item_packable(c, amount);
            wide_item = !packed;
            c.bal_items[k] = ((packed ? amount : pair_amount_mask(ps)) << (2 * ps + 1)) |
                             (uint64_t(pending) << (2 * ps)) | (uint64_t(cr.row) << ps) | dr.row;
        } else if (c.bal_items) {
            uint4* it = reinterpret_cast<uint4*>(c.bal_items + 2 * uint64_t(k));
            if ((amount >> (64 - c.key_bits)) == 0) {
                const uint32_t kd = dr.row * 4 + (pending ? 0 : 1);
                const uint32_t kc = cr.row * 4 + (pending ? 2 : 3);
                const uint64_t i0 = (amount << c.key_bits) | kd, i1 = (amount << c.key_bits) | kc;
                *it = make_uint4(uint32_t(i0), uint32_t(i0 >> 32), uint32_t(i1), uint32_t(i1 >> 32));
                if (bucket_hist) {
                    atomicAdd(&bucket_hist[kd >> kBucketShift], 1u);
                    atomicAdd(&bucket_hist[kc >> kBucketShift], 1u);
                }
            } else {
                *it = make_uint4(~0u, ~0u, ~0u, ~0u);  // too wide to pack: atomics in tr_commit
                need_commit = true;
            }
        } else {
            // Calls without balance items (below kSortThreshold events): the deltas go to the
            // rows now, with u128 atomics (they commute with every other FAST delta, and nothing
            // reads a balance before tr_commit); a FAST event tr_commit demotes subtracts them
            // again (commit_event). A clean call then needs no tr_commit pass at all.
            apply_fast_deltas(T, dr.row, cr.row, pending, amount, false);
        }
        *fast_ts = ts_event;
    } else {
        // Accounts whose balance this event may read when it replays -- the limit flag of the
        // side it checks, balancing, a possible overflow (create_transfer :3842-3905) -- may take
        // no FAST delta of this call: tr_commit demotes FAST events touching them. An account it
        // only writes needs no mark: every FAST delta is applied before the replay and the
        // replay's own deltas commute with them. (post/void read no balance, :4053-4300; `closed`
        // is ordered by the closable marks.)
        const bool ovf = tn.amount_hi() != 0 || dr.hi_pending >= kHazardHiLimit ||
                         dr.hi_posted >= kHazardHiLimit || cr.hi_pending >= kHazardHiLimit ||
                         cr.hi_posted >= kHazardHiLimit;
        const bool read_dr = dr.row != kNone32 &&
                             (ovf || (f & TB_TRANSFER_BALANCING_DEBIT) ||
                              (dr.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS));
        const bool read_cr = cr.row != kNone32 &&
                             (ovf || (f & TB_TRANSFER_BALANCING_CREDIT) ||
                              (cr.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS));
        if (read_dr) T.acc_hot[dr.row] = c.epoch;
        if (read_cr) T.acc_hot[cr.row] = c.epoch;
        hot = read_dr || read_cr;
    }
    if (cls != kClassFast) {
        need_commit = true;
        // (lanes_check's static rules, plan_keys)
        no_lanes = cls == kClassSlow && (f != 0 || tn.timeout() != 0 || tn.amount_hi() != 0 ||
                                         tn.timestamp() != 0 || batch_imported ||
                                         !u128_is_zero(t.pending_id));
        if (c.bal_items && c.pair_shift)
            c.bal_items[k] = ~0ull;
        else if (c.bal_items)
            *reinterpret_cast<uint4*>(c.bal_items + 2 * uint64_t(k)) = make_uint4(~0u, ~0u, ~0u, ~0u);
    }
    return (imported ? kFlagImported : 0u) | (post_void ? kFlagPostVoid : 0u) |
           (dup ? kFlagDuplicate : 0u) | (closable ? kFlagClosable : 0u) | (hot ? kFlagHot : 0u) |
           (need_commit ? kFlagNeedCommit : 0u) | (chain_fast ? kFlagChain : 0u) |
           (ae_slow ? kFlagAeSlow : 0u) | (wide_item ? kFlagWideItems : 0u) |
           (no_lanes ? kFlagNoLanes : 0u);
}

// Per 64-event chunk of a create_transfers call (one lane each): the batch b0 of its first event,
// that batch's end, ts_base = batch_ts[b0] - end + 1 (event k < end is stamped ts_base + k),
// whether b0 is an imported batch, and whether the chunk's first event continues a chain of its
// batch. tr_ingest reads it with one uniform load per chunk: the batch search costs ~10
// vector-memory instructions per wave when each chunk repeats it (the compiler cannot use scalar
// loads for memory the kernel may write), and tr_ingest is bound by vector-memory issue.
constexpr uint32_t kChunkBatchMask = (1u << 30) - 1;
constexpr uint32_t kChunkImported = 1u << 30;
constexpr uint32_t kChunkPrevLinked = 1u << 31;

__device__ inline uint4 chunk_info_of(const Call<tb_transfer_t>& c, uint32_t base) {
    const uint32_t b0 = batch_of_guess(c.batch_ends, c.n_batches, c.n, base);
    const uint32_t end0 = c.batch_ends[b0];
    const uint32_t bstart0 = batch_start_of(c, b0);
    const uint64_t ts_base = c.batch_ts[b0] - end0 + 1;
    uint32_t w = b0;
    if (c.events[bstart0].flags & TB_TRANSFER_IMPORTED) w |= kChunkImported;
    if (base > bstart0 && (c.events[base - 1].flags & TB_TRANSFER_LINKED)) w |= kChunkPrevLinked;
    return make_uint4(w, end0, uint32_t(ts_base), uint32_t(ts_base >> 32));
}

// The call's words of the scalars block (flags, counters), zero before tr_ingest.
__device__ inline void reset_call_scalars(DevScalars* scalars) {
    scalars->flags = 0;
    scalars->slow_count = 0;
    for (int j = 0; j < 4; j++) scalars->stats[j] = 0;
    scalars->spec_fast = 0;
    scalars->spec_ts_max = 0;
    scalars->fixed = 0;
}

// The call's scalar words zeroed at the end of a call (queued behind it, while the host returns):
// the next small call needs neither tr_chunk_info nor a memset before its tr_ingest.
__global__ void tr_reset_scalars(DevScalars* scalars) {
    if (threadIdx.x == 0 && blockIdx.x == 0) reset_call_scalars(scalars);
}

// (Also resets the call's words of the scalars block for tr_ingest: the first kernel of a
// create_transfers call, so the call needs no separate memset.)
__global__ void tr_chunk_info(Call<tb_transfer_t> c, uint4* out, DevScalars* scalars) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) reset_call_scalars(scalars);
    const uint32_t base = i * 64;
    if (base >= c.n) return;
    out[i] = chunk_info_of(c, base);
}

// The end of a small call by tr_ingest's last workgroup (Call::finish_done), when no event raised a
// commit flag: what tr_commit's clean branch, stage_out and tr_reset_scalars would do, two launches
// earlier (calls whose results stay in HBM: tbg_create_transfers_device). A workgroup is counted
// after every wave has waited for its stores and lane 0 has released them at agent scope
// (MI355X_MICROARCH.md, inter-workgroup visibility).
// The last workgroup acquires, sums the call's counters, copies the scalars block to its mapped
// copy, clears the call's scalar words for the next call, marks the call finished for the queued
// tr_commit and stage_out (finish_done[1] = epoch: they return at once), and then publishes the
// sequence word.
__device__ inline void ingest_finish(const Tables& T, const Call<tb_transfer_t>& c) {
    __shared__ unsigned int last;  // 0: not the last workgroup; else the call's flags | 1 << 31
    DevScalars* S = T.scalars;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = 0;
        if (atomicAdd(c.finish_done, 1u) == gridDim.x - 1) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            atomicExch(c.finish_done, 0u);
            last = __hip_atomic_load(&S->flags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | (1u << 31);
        }
    }
    __syncthreads();
    const unsigned int flags = last;
    // (tr_commit and stage_out end a call with a commit flag; the rest is the first wave's alone:
    // one system-scope release, the sequence word's, instead of a fence per wave -- 3.4 -> 2.5 us
    // from the last workgroup's acquire to the sequence word)
    if (!(flags >> 31) || threadIdx.x >= 64) return;
    auto load = [](const unsigned long long* p) {
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };
    constexpr uint32_t words = uint32_t(sizeof(DevScalars) / 8);
    static_assert(sizeof(DevScalars) / 8 <= 64, "one word a lane");
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(S);
    if (flags & kCommitFlags) {
        // Not ended here: with finish_always the host learns it now (the flags without
        // kFlagFinished) and launches tr_commit and stage_out; the scalar words stay.
        if (!c.finish_always || !c.finish_seq) return;
        if (threadIdx.x < words) c.finish_scalars[threadIdx.x] = load(src + threadIdx.x);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        if (threadIdx.x == 0)
            __hip_atomic_store(c.finish_seq, c.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        return;
    }
    if (threadIdx.x == 0) {
        // tr_commit's clean branch: transfers key_range and the FAST count
        const unsigned long long ts = load(&S->spec_ts_max);
        if (ts > load(&S->transfers_key_max)) atomicMax(&S->transfers_key_max, ts);
        atomicAdd(&S->stats[1], load(&S->spec_fast));
        atomicOr(&S->flags, kFlagFinished);
        c.finish_done[1] = c.epoch;
        __threadfence();
    }
    __builtin_amdgcn_wave_barrier();
    if (threadIdx.x < words) c.finish_scalars[threadIdx.x] = load(src + threadIdx.x);
    // Every lane's copy (its load and its store) happens before lane 0's reset: a wavefront-scope
    // release / acquire around the barrier orders them in the HIP memory model, not only through
    // the wave's in-order issue.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (threadIdx.x == 0) reset_call_scalars(S);
    // The sequence word's system-scope release covers the wave's copy and reset. ISA-level
    // assumption (gfx950): a release is a wave instruction sequence -- the L2 write-back and the
    // s_waitcnt on the wave's outstanding stores -- so lane 0's release publishes the stores of all
    // 64 lanes of its wave; the other lanes' stores were ordered before it by the wavefront fence
    // above. test_gpu_parity's device-call and per-commit parity tests read finish_scalars through
    // this publication on every small call. Without a sequence word, a fence.
    if (threadIdx.x == 0) {
        if (c.finish_seq)
            __hip_atomic_store(c.finish_seq, c.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        else
            __threadfence_system();
    }
}

// LDS image of a wave's 64 events: 144 bytes per event (128 + 16 of padding), so the lanes'
// 16-byte field reads (one event per lane) fall on distinct banks.
constexpr uint32_t kLdsEventStride = 144;
constexpr uint32_t kIngestWaves = kBlock / 64;
constexpr uint32_t kIngestGrid = 12288;  // tr_ingest workgroups (grid-stride beyond)

__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// tr_ingest: each wave takes 64 consecutive events at a time. The 8 KB of events arrive as 8
// fully coalesced 16-byte loads per lane, are transposed through LDS so each lane reads its own
// event's fields, and go back out as the transfer rows (timestamp patched) with 8 coalesced
// stores. The next chunk's loads are issued before the current chunk's table work, so the event
// stream overlaps the claim / index round trip.
__global__ void __launch_bounds__(kBlock, kIngestWgPerCu) tr_ingest(Tables T,
                                                                         Call<tb_transfer_t> c) {
    __shared__ __attribute__((aligned(16))) uint8_t lds_ev[kIngestWaves][64 * kLdsEventStride];
    __shared__ uint64_t lds_ts[kIngestWaves][64];
    __shared__ unsigned int bucket_hist[kBucketsMax];
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    if (c.bucket_counts) {
        for (uint32_t i = threadIdx.x; i < c.n_buckets; i += blockDim.x) bucket_hist[i] = 0;
        __syncthreads();
    }
    uint8_t* my = lds_ev[wv];
    const uint32_t waves = blockDim.x >> 6;  // (kIngestWaves, or fewer for small calls)
    const uint32_t nw = gridDim.x * waves;
    if (c.ends_out && blockIdx.x == 0)  // (the batch bounds read from the host: the later kernels' copy)
        for (uint32_t b = threadIdx.x; b < c.n_batches; b += blockDim.x) {
            c.ends_out[b] = c.batch_ends[b];
            c.ts_out[b] = c.batch_ts[b];
        }
    unsigned int flags = 0;
    uint64_t n_fast = 0, ts_max = 0;
    uint4 q[8];
    auto load_chunk = [&](uint32_t base) {
        const uint4* src = reinterpret_cast<const uint4*>(c.events + base);
        const uint32_t parts = (c.n - base < 64 ? c.n - base : 64) * 8;
#pragma unroll
        for (int i = 0; i < 8; i++) {
            // A body read from host memory: two rounds of 4 loads a lane (PCIe reads peak with
            // fewer requests in flight, tools/pciebench.hip; 77 -> 73 us a commit, r05_h A/B).
            if (i == 4 && c.events_out) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const uint32_t idx = i * 64 + lane;
            typedef unsigned int v4u __attribute__((ext_vector_type(4)));
            if (idx < parts) {
                const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(&src[idx]));
                q[i] = make_uint4(v.x, v.y, v.z, v.w);
            } else {
                q[i] = make_uint4(0, 0, 0, 0);
            }
        }
    };
    uint32_t base = (blockIdx.x * waves + wv) * 64;
    if (base < c.n) load_chunk(base);
    for (; base < c.n; base += nw * 64) {
        const uint32_t ubase = __builtin_amdgcn_readfirstlane(base);
        // (small calls: the wave finds its chunk's bounds itself -- one launch fewer)
        const uint4 ci = c.chunk_info ? c.chunk_info[ubase >> 6] : chunk_info_of(c, ubase);
        const uint32_t cnt = c.n - ubase < 64 ? c.n - ubase : 64;
        // One ds_write_b128 per part: each 8-lane group writes one event's 128 contiguous bytes,
        // which no two lanes share a bank of. (A uint4 store here was split into ds_write2_b64
        // pairs, whose 16-lane groups put two events' rows 144 B apart on the same banks: 2-way
        // conflicts, SQ_LDS_BANK_CONFLICT in profiles/r02_pmc.)
        typedef unsigned int v4u_lds __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint32_t e = i * 8 + (lane >> 3), part = lane & 7;
            const v4u_lds v = {q[i].x, q[i].y, q[i].z, q[i].w};
            *reinterpret_cast<v4u_lds*>(
                __builtin_assume_aligned(my + e * kLdsEventStride + part * 16, 16)) = v;
        }
        wave_lds_sync();
        const uint32_t k = base + lane;
        const bool active = lane < cnt;
        // The chunk's batch bounds (tr_chunk_info); lanes past the batch end (a chunk that
        // straddles one) find their own batch.
        const uint32_t w0 = __builtin_amdgcn_readfirstlane(ci.x);
        const uint32_t end0 = __builtin_amdgcn_readfirstlane(ci.y);
        // (readfirstlane returns int: widen through uint32_t, not by sign extension)
        const uint64_t ts_base =
            (uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(ci.w))) << 32) |
            uint32_t(__builtin_amdgcn_readfirstlane(ci.z));
        // (per-event timestamps take the straddling chunk's path: rows stamped from LDS)
        const bool straddle = ubase + cnt > end0 || c.event_ts != nullptr;
        uint64_t ts_event = ts_base + k;
        if (c.event_ts && active) ts_event = c.event_ts[k];
        bool batch_imported = (w0 & kChunkImported) != 0;
        bool first_of_batch = false;
        if (active && k >= end0) {
            uint32_t b = (w0 & kChunkBatchMask) + 1;
            while (c.batch_ends[b] <= k) b++;
            const uint32_t bstart = c.batch_ends[b - 1];
            ts_event = ts_event_of(c, b, k);
            batch_imported = (c.events[bstart].flags & TB_TRANSFER_IMPORTED) != 0;
            first_of_batch = k == bstart;
        }
        // ts_event (and the batch facts) may come from loads: wait for them here, before the
        // row stores and the prefetch are issued -- a wait at their first use further down would
        // have to drain the prefetch too (vmcnt counts in order). The asm redefines the registers,
        // so the compiler places no later wait for them.
        {
            uint32_t fb = first_of_batch, bi = batch_imported;
            asm volatile("s_waitcnt vmcnt(0)" : "+v"(ts_event), "+v"(fb), "+v"(bi));
            first_of_batch = fb != 0;
            batch_imported = bi != 0;
        }
        if (straddle) {
            lds_ts[wv][lane] = active ? ts_event : 0;
            wave_lds_sync();
        }
        // The rows: the events as submitted, stamped with their commit timestamps (rows of
        // events that do not create an object stay dead; an orphaned id keeps its key there).
        // Stored straight from q (timestamps patched in place): a store whose data sits in a
        // temporary that the next store reuses makes the compiler wait for the first store's
        // completion (vmcnt(0)) before the second, serialising the 8 stores.
        uint4* dst = reinterpret_cast<uint4*>(T.tr_rows + c.row_base + base);
        const bool full = cnt == 64;
        if (c.events_out) {  // (the body as submitted, for the call's later kernels)
            uint4* cp = reinterpret_cast<uint4*>(c.events_out + base);
#pragma unroll
            for (int i = 0; i < 8; i++)
                if (full || i * 64 + lane < cnt * 8) cp[i * 64 + lane] = q[i];
        }
        const uint64_t ts_lane = ts_base + ubase + (lane >> 3);  // + 8 i: event i * 8 + lane / 8
#pragma unroll
        for (int i = 0; i < 8; i++) {
            if ((lane & 7) == 7) {
                const uint64_t ts = straddle ? lds_ts[wv][i * 8 + (lane >> 3)] : ts_lane + i * 8;
                q[i].z = uint32_t(ts);
                q[i].w = uint32_t(ts >> 32);
            }
            if (full || i * 64 + lane < cnt * 8) {
                typedef unsigned int v4u __attribute__((ext_vector_type(4)));
                const v4u v = {q[i].x, q[i].y, q[i].z, q[i].w};
                __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(&dst[i * 64 + lane]));
            }
        }
        const uint32_t next = base + nw * 64;
        // (The lane's fields are read from the LDS image where they are used: 16-byte fields with
        // conflict-free ds_read_b128; the 2-8 byte ones put 2-4 lanes of a 32-lane group on a
        // bank. A register copy of the event would avoid that but spills at this kernel's
        // 128-VGPR budget.)
        // (the previous event's flags from its lane: a 2-byte LDS read of its image at the
        // 144-byte stride put 4 lanes on a bank)
        const uint32_t own_flags =
            ev_narrow(*reinterpret_cast<const tb_transfer_t*>(my + lane * kLdsEventStride)).flags();
        const uint32_t up_flags = __shfl_up(own_flags, 1, 64);
        if (active) {
            const tb_transfer_t& t = *reinterpret_cast<const tb_transfer_t*>(my + lane * kLdsEventStride);
            const bool prev_linked =
                lane > 0 ? !first_of_batch && (up_flags & TB_TRANSFER_LINKED) != 0
                         : (w0 & kChunkPrevLinked) != 0;
            uint64_t fts = 0;
            flags |= ingest_event(T, c, k, t, batch_imported, ts_event, prev_linked, &fts,
                                  c.bucket_counts ? bucket_hist : nullptr);
            n_fast += fts != 0;
            ts_max = fts > ts_max ? fts : ts_max;
        }
        if (next < c.n) load_chunk(next);
        wave_lds_sync();  // the LDS image is rewritten by the next chunk
    }
    flags = block_reduce(flags, OpOr());  // (its barriers also order the histogram adds)
    n_fast = block_reduce(n_fast, OpAdd());
    ts_max = block_reduce(ts_max, OpMax());
    if (c.bucket_counts)
        for (uint32_t i = threadIdx.x; i < c.n_buckets; i += blockDim.x)
            if (bucket_hist[i]) atomicAdd(&c.bucket_counts[i], bucket_hist[i]);
    if (threadIdx.x == 0) {
        if (flags) atomicOr(&T.scalars->flags, flags);
        if (n_fast) atomicAdd(&T.scalars->spec_fast, (unsigned long long)n_fast);
        if (ts_max) atomicMax(&T.scalars->spec_ts_max, (unsigned long long)ts_max);
    }
    if (c.finish_done) ingest_finish(T, c);
}


// A FAST event's record as tr_commit reads it: its id slot (kNone32 unless re-probed or recorded),
// account rows and amount.
struct FastRec {
    uint32_t s, dr, cr;
    uint64_t amount;
    bool post_void;
    int8_t first = -1;  // a post/void: pv_first, when its caller already knows it (-1: not known)
};
__device__ inline FastRec fast_record(const Tables& T, const Call<tb_transfer_t>& c, uint32_t k,
                                      unsigned int call_flags, uint8_t info) {
    FastRec f;
    f.s = kNone32;
    f.first = -1;
    f.post_void = (c.events[k].flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) != 0;
    const bool lean = (info & kInfoLean) != 0;
    if (lean && !c.bal_items) {
        // (Call::lean_lookup: the accounts are fixed during the call; FAST means both exist)
        const tb_transfer_t& e = c.events[k];
        f.dr = uint32_t(account_find(T, e.debit_account_id));
        f.cr = uint32_t(account_find(T, e.credit_account_id));
        f.amount = e.amount.lo;
    } else if (lean && c.pair_shift) {
        const uint32_t ps = c.pair_shift;
        const uint64_t x = c.bal_items[k];
        f.dr = uint32_t(x & ((1ull << ps) - 1));
        f.cr = uint32_t((x >> ps) & ((1ull << ps) - 1));
        f.amount = x >> (2 * ps + 1);
    } else if (lean) {
        const uint64_t kmask = (1ull << c.key_bits) - 1;
        const uint64_t* it = c.bal_items + 2 * uint64_t(k);
        const uint64_t i0 = it[0], i1 = it[1];
        f.dr = uint32_t((i0 & kmask) >> 2);
        f.cr = uint32_t((i1 & kmask) >> 2);
        f.amount = i0 >> c.key_bits;
    } else {
        f.s = c.ev_slot[k];
        f.dr = c.ev_dr[k];
        f.cr = c.ev_cr[k];
        f.amount = c.ev_amount[k];
    }
    if (lean && (call_flags & kFlagDuplicate)) {
        // The slot this event's id occupies (its own claim, or an earlier in-call holder's): the
        // duplicate check reads it. (Otherwise only a demoted or fixed event needs it: looked up
        // there.)
        const uint64_t fs = transfer_slot_find(T, c, c.events[k].id);
        f.s = fs == kNone ? kNone32 : uint32_t(fs);
    }
    return f;
}

// Does anything of the call invalidate FAST event k's speculative commit? Each re-check reads only
// when ingest raised the flag that can make it fail.
__device__ inline bool fast_demoted(const Tables& T, const Call<tb_transfer_t>& c, uint32_t k,
                                    unsigned int call_flags, const FastRec& f) {
    const uint64_t ref = c.row_base + k + 1;
    if (f.post_void && !(f.first >= 0 ? f.first != 0 : pv_first(c, k, c.events[k].pending_id)))
        return true;
    return (call_flags & kFlagImported) ||
           ((call_flags & kFlagDuplicate) &&
            (f.s == kNone32 || (T.tr.slots[f.s] & kRefMask) != ref)) ||
           ((call_flags & kFlagClosable) &&
            (T.acc_closable[f.dr] == c.epoch || T.acc_closable[f.cr] == c.epoch)) ||
           ((call_flags & kFlagHot) && (T.acc_hot[f.dr] == c.epoch || T.acc_hot[f.cr] == c.epoch));
}

// fast_demoted for another event j of the call, from what no thread of tr_commit writes: its id's
// slot and its accounts looked up again (the same slot and rows ingest found -- accounts and the
// refs of slots are fixed during tr_commit), not its balance items, which j's own thread may be
// clearing.
__device__ inline bool fast_demoted_peer(const Tables& T, const Call<tb_transfer_t>& c, uint32_t j,
                                         unsigned int call_flags) {
    if (call_flags & kFlagImported) return true;
    const tb_transfer_t& e = c.events[j];
    if (call_flags & kFlagDuplicate) {
        const uint64_t s = transfer_slot_find(T, c, e.id);
        if (s == kNone || (T.tr.slots[s] & kRefMask) != c.row_base + j + 1) return true;
    }
    const bool post_void = (e.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) != 0;
    if (post_void && !pv_first(c, j, e.pending_id)) return true;
    if (call_flags & (kFlagClosable | kFlagHot)) {
        // (a post/void's accounts are its pending transfer's)
        const tb_transfer_t* a = &e;
        if (post_void) {
            const uint64_t pr = pv_pending_row(T, c, e.pending_id);
            if (pr == kNone) return true;
            a = &T.tr_rows[pr];
        }
        const uint64_t dr = account_find(T, a->debit_account_id);
        const uint64_t cr = account_find(T, a->credit_account_id);
        if (dr == kNone || cr == kNone) return true;
        if ((call_flags & kFlagClosable) &&
            (T.acc_closable[dr] == c.epoch || T.acc_closable[cr] == c.epoch))
            return true;
        if ((call_flags & kFlagHot) && (T.acc_hot[dr] == c.epoch || T.acc_hot[cr] == c.epoch))
            return true;
    }
    return false;
}

constexpr uint32_t kFastChainMax = 32;  // (chain_demoted below)

// A later post/void k of a pending transfer X whose first post/void in the call (the winner of X's
// claim) is a single FAST event that tr_commit confirms: X is posted / voided before k runs, and
// k -- FAST at ingest, so every check before the status switch (post_or_void_pending_transfer
// :4166-4226) passed on X's immutable row -- fails with pending_transfer_already_posted /
// _voided in any order. (A winner inside a chain may roll back: then k replays.) 0: not such an
// event. Reads only what no tr_commit thread writes.
__device__ inline uint32_t later_claim_status(const Tables& T, const Call<tb_transfer_t>& c,
                                              uint32_t k, unsigned int call_flags) {
    const tb_transfer_t& e = c.events[k];
    if (!(e.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) || !c.pv_slots ||
        (call_flags & kFlagImported))
        return 0;
    const uint32_t j = pv_winner(c, e.pending_id);
    if (j == kNone32 || j >= k) return 0;
    if ((c.ev_info[j] & kInfoClassMask) != kClassFast) return 0;
    const tb_transfer_t& w = c.events[j];
    if (w.flags & TB_TRANSFER_LINKED) return 0;
    if (j > 0 && (c.events[j - 1].flags & TB_TRANSFER_LINKED) &&
        j != batch_start_of(c, batch_of_guess(c.batch_ends, c.n_batches, c.n, j)))
        return 0;
    if (fast_demoted_peer(T, c, j, call_flags)) return 0;
    // k itself must hold its id (a later duplicate's outcome follows the earlier holder's).
    if (call_flags & kFlagDuplicate) {
        const uint64_t s = transfer_slot_find(T, c, e.id);
        if (s == kNone || (T.tr.slots[s] & kRefMask) != c.row_base + k + 1) return 0;
    }
    return (w.flags & TB_TRANSFER_POST_PENDING) ? TB_CT_PENDING_TRANSFER_ALREADY_POSTED
                                                : TB_CT_PENDING_TRANSFER_ALREADY_VOIDED;
}

// A chain whose every event is FAST at ingest and whose first event that is not an undemoted FAST
// event is a later claim (above) fails there in any order: that event takes the claim's status,
// every other event of the chain linked_event_failed (execute_create :3116-3194), nothing is
// applied. Returns that status for event k (0: not such a chain). Every event of the chain
// evaluates the same rule over the same data, so they agree.
__device__ inline uint32_t chain_fail_status(const Tables& T, const Call<tb_transfer_t>& c,
                                             uint32_t k, unsigned int call_flags) {
    const uint32_t b = batch_of_guess(c.batch_ends, c.n_batches, c.n, k);
    const uint32_t bs = batch_start_of(c, b), be = c.batch_ends[b];
    uint32_t x = k, y = k;
    while (x > bs && (c.events[x - 1].flags & TB_TRANSFER_LINKED)) {
        if (k - x >= kFastChainMax) return 0;
        x--;
    }
    while (c.events[y].flags & TB_TRANSFER_LINKED) {
        if (y + 1 >= be) return 0;  // linked_event_chain_open: the replay decides
        if (y - k >= kFastChainMax) return 0;
        y++;
    }
    if (y - x >= kFastChainMax) return 0;
    for (uint32_t j = x; j <= y; j++)
        if ((c.ev_info[j] & kInfoClassMask) != kClassFast) return 0;
    for (uint32_t j = x; j <= y; j++) {
        if (!fast_demoted_peer(T, c, j, call_flags)) continue;
        const uint32_t st = later_claim_status(T, c, j, call_flags);
        if (!st) return 0;
        return j == k ? st : uint32_t(TB_CT_LINKED_EVENT_FAILED);
    }
    return 0;  // (no failure: the chain is confirmed)
}

// A FAST event of a linked chain (execute_create :3033-3207): the chain creates every event iff
// every event of it is FAST and none is demoted -- then no event fails, nothing is rolled back, and
// each event's effects are those of a FAST event. Otherwise the whole chain replays. Every event of
// the chain evaluates the same rule over the same events, so they agree. Chains longer than
// kFastChainMax (or open at their batch's end: linked_event_chain_open) replay.
__device__ inline bool chain_demoted(const Tables& T, const Call<tb_transfer_t>& c, uint32_t k,
                                     unsigned int call_flags) {
    const uint32_t b = batch_of_guess(c.batch_ends, c.n_batches, c.n, k);
    const uint32_t bs = batch_start_of(c, b), be = c.batch_ends[b];
    uint32_t x = k, y = k;
    while (x > bs && (c.events[x - 1].flags & TB_TRANSFER_LINKED)) {
        if (k - x >= kFastChainMax) return true;
        x--;
    }
    while (c.events[y].flags & TB_TRANSFER_LINKED) {
        if (y + 1 >= be) return true;  // linked_event_chain_open
        if (y - k >= kFastChainMax) return true;
        y++;
    }
    if (y - x >= kFastChainMax) return true;
    for (uint32_t j = x; j <= y; j++)
        if ((c.ev_info[j] & kInfoClassMask) != kClassFast) return true;
    for (uint32_t j = x; j <= y; j++)
        if (j != k && fast_demoted_peer(T, c, j, call_flags)) return true;
    return false;
}

// chain_demoted / chain_fail_status of a wave's events at once (tr_commit): every FAST chain event
// evaluates fast_demoted_peer (and, when demoted, later_claim_status) for itself once, and the
// lanes of a chain that lies inside the wave combine them by ballot -- instead of each event
// re-evaluating every other event of its chain. valid == false: not a chain event, or a chain that
// crosses the wave's edge (commit_event evaluates it alone). Every lane of the wave calls it.
struct ChainPre {
    bool valid;
    bool demoted;     // chain_demoted
    uint32_t fail;    // chain_fail_status (calls with post/void)
    int8_t in_chain;  // commit_event's in_chain (-1: not evaluated)
    bool has_fr;      // fr: the event's FastRec (FAST chain events)
    FastRec fr;
};
// Bit planes of a large call's linked chains (tr_chain_planes, before tr_commit): per 64-event
// group, one word each of chain heads, chain ends, open ends, FAST events, demoted FAST chain
// events (fast_demoted) and their later-claim statuses. Computed before tr_commit writes anything,
// so from the state fast_demoted_peer reads. tr_commit then resolves every chain from the words of
// three groups -- also chains that cross its wave's edges, which otherwise walked the chain event
// by event with a chain of lookups each (config 4: ~100 us tails a 131k-event call).
enum : uint32_t {
    kPlHead, kPlEnd, kPlOpen, kPlFast, kPlDemoted, kPlPosted, kPlVoided, kPlWords = 8
};

// A chain event's ChainPre from the planes: the 64-event window whose bit 32 is event k (group
// g = (k - lane) / 64 and its neighbours), chain bounds x <= 32 <= y, then chain_demoted /
// chain_fail_status's rules. Every lane of the wave calls it.
__device__ inline ChainPre chain_pre_planes(const Call<tb_transfer_t>& c, uint32_t kb, uint32_t lane,
                                            bool in_chain, unsigned int call_flags, ChainPre p) {
    const uint64_t g = kb / 64, groups = (uint64_t(c.n) + 63) / 64;
    const unsigned long long* P = c.chain_planes;
    auto win = [&](uint32_t plane) -> uint64_t {
        const uint64_t b = P[g * kPlWords + plane];
        if (lane < 32) {
            const uint64_t a = g > 0 ? P[(g - 1) * kPlWords + plane] : 0ull;
            return (a >> (32 + lane)) | (b << (32 - lane));
        }
        const uint64_t cw = g + 1 < groups ? P[(g + 1) * kPlWords + plane] : 0ull;
        const uint32_t s = lane - 32;
        return s ? (b >> s) | (cw << (64 - s)) : b;
    };
    const uint64_t H = win(kPlHead), E = win(kPlEnd), O = win(kPlOpen), F = win(kPlFast),
                   D = win(kPlDemoted), LP = win(kPlPosted), LV = win(kPlVoided);
    if (!in_chain) return p;
    p.valid = true;
    const uint64_t hb = H & ((2ull << 32) - 1);   // heads at or before this event
    const uint64_t eb = E & ~((1ull << 32) - 1);  // ends at or after it
    const uint32_t x = hb ? 63u - uint32_t(__builtin_clzll(hb)) : 0u;
    const uint32_t y = eb ? uint32_t(__builtin_ctzll(eb)) : 63u;
    // (x == 0: the head is kFastChainMax or more events back; eb == 0: the end is that far on)
    if (x == 0 || !eb || y - x >= kFastChainMax || ((O >> y) & 1)) {
        p.demoted = true;
        return p;
    }
    const uint64_t cm = (y == 63 ? ~0ull : (2ull << y) - 1) & ~((1ull << x) - 1);
    if ((F & cm) != cm) {
        p.demoted = true;
        return p;
    }
    const uint64_t pm = D & cm;
    if (pm && (call_flags & kFlagPostVoid)) {
        const uint32_t j = uint32_t(__builtin_ctzll(pm));
        const uint32_t lc = ((LP >> j) & 1) ? uint32_t(TB_CT_PENDING_TRANSFER_ALREADY_POSTED)
                            : ((LV >> j) & 1) ? uint32_t(TB_CT_PENDING_TRANSFER_ALREADY_VOIDED)
                                              : 0u;
        if (lc) p.fail = j == 32 ? lc : uint32_t(TB_CT_LINKED_EVENT_FAILED);
    }
    p.demoted = (pm & ~(1ull << 32)) != 0;
    return p;
}

__device__ inline ChainPre chain_pre_wave(const Tables& T, const Call<tb_transfer_t>& c,
                                          uint32_t k, bool active, unsigned int call_flags) {
    ChainPre p{false, false, 0, -1, false, FastRec{}};
    if (!(call_flags & kFlagChain)) {
        p.in_chain = 0;
        return p;
    }
    const uint32_t lane = threadIdx.x & 63;
    bool linked = false, prev_linked = false, open = false;
    uint8_t cls = 0, info = 0;
    if (active) {
        linked = (c.events[k].flags & TB_TRANSFER_LINKED) != 0;
        const bool pl = k > 0 && (c.events[k - 1].flags & TB_TRANSFER_LINKED);
        if (linked || pl) {  // (the batch bounds only for events next to a linked one)
            const uint32_t b = batch_of_guess(c.batch_ends, c.n_batches, c.n, k);
            const uint32_t bs = batch_start_of(c, b), be = c.batch_ends[b];
            prev_linked = pl && k > bs;
            open = linked && k + 1 >= be;  // linked_event_chain_open
        }
        info = c.ev_info[k];
        cls = info & kInfoClassMask;
    }
    const bool in_chain = active && (linked || prev_linked);
    p.in_chain = in_chain ? 1 : 0;
    if (c.chain_planes) return chain_pre_planes(c, k - lane, lane, in_chain, call_flags, p);
    const uint64_t head_m = __ballot(active && !prev_linked);
    const uint64_t end_m = __ballot(active && (!linked || open));
    const uint64_t open_m = __ballot(open);
    const uint64_t fast_m = __ballot(active && cls == kClassFast);
    bool pd = false;
    uint32_t lc = 0;
    if (in_chain && cls == kClassFast) {
        // (its own record: this thread has not touched it yet -- the same verdict the peers'
        // fast_demoted_peer reaches from lookups)
        p.fr = fast_record(T, c, k, call_flags, info);
        p.has_fr = true;
        pd = fast_demoted(T, c, k, call_flags, p.fr);
        if (pd && (call_flags & kFlagPostVoid)) lc = later_claim_status(T, c, k, call_flags);
    }
    const uint64_t pd_m = __ballot(pd);
    const uint64_t below = head_m & ((2ull << lane) - 1);       // (lane 63: all ones)
    const uint64_t above = end_m & ~((1ull << lane) - 1);
    const bool inside = in_chain && below != 0 && above != 0;
    const uint32_t x = inside ? 63u - uint32_t(__builtin_clzll(below)) : lane;
    const uint32_t y = inside ? uint32_t(__builtin_ctzll(above)) : lane;
    const uint64_t chain_m = inside ? ((y == 63 ? ~0ull : (2ull << y) - 1) & ~((1ull << x) - 1)) : 0;
    const uint64_t pm = pd_m & chain_m;
    const uint32_t j = pm ? uint32_t(__builtin_ctzll(pm)) : lane;
    const uint32_t lc_j = __shfl(lc, int(j));
    if (!inside) return p;
    p.valid = true;
    if (y - x >= kFastChainMax || ((open_m >> y) & 1) || (fast_m & chain_m) != chain_m) {
        p.demoted = true;
        return p;
    }
    if (pm && (call_flags & kFlagPostVoid) && lc_j)
        p.fail = j == lane ? lc_j : uint32_t(TB_CT_LINKED_EVENT_FAILED);
    p.demoted = (pm & ~(1ull << lane)) != 0;
    return p;
}

// The effects of a confirmed FAST post/void (post_or_void_pending_transfer :4193-4299): its row,
// the pending transfer's status, the balance deltas on the pending transfer's accounts, and the
// pulse_next_timestamp reset (recorded at the event: calls with post/void resolve them in order).
__device__ inline void commit_post_void(const Tables& T, const Call<tb_transfer_t>& c, uint32_t k,
                                        uint64_t row, uint64_t ts, uint32_t dr, uint32_t cr) {
    const tb_transfer_t t = c.events[k];
    const uint64_t pr = c.ev_prow[k];  // (ingest's lookup: committed slots and rows are fixed)
    const tb_transfer_t p = T.tr_rows[pr];
    const bool post = (t.flags & TB_TRANSFER_POST_PENDING) != 0;
    const u128 p_amount = U(p.amount);
    const u128 amount = post ? (U(t.amount) == kU128Max ? p_amount : U(t.amount)) : p_amount;
    // The row as eight 16-byte words stored straight from registers (a tb_transfer_t local copied
    // by assignment stayed in scratch: 72 bytes a lane, and each scratch load waited for every
    // memory operation issued before it). Scalar selects: a struct select keeps both rows in scratch.
    auto q = [](uint64_t lo, uint64_t hi) {
        return make_uint4(uint32_t(lo), uint32_t(lo >> 32), uint32_t(hi), uint32_t(hi >> 32));
    };
    const u128 ud128 = U(t.user_data_128) > 0 ? U(t.user_data_128) : U(p.user_data_128);
    const uint64_t ud64 = t.user_data_64 > 0 ? t.user_data_64 : p.user_data_64;
    const uint32_t ud32 = t.user_data_32 > 0 ? t.user_data_32 : p.user_data_32;
    uint4* o = reinterpret_cast<uint4*>(&T.tr_rows[row]);
    o[0] = q(t.id.lo, t.id.hi);
    o[1] = q(p.debit_account_id.lo, p.debit_account_id.hi);
    o[2] = q(p.credit_account_id.lo, p.credit_account_id.hi);
    o[3] = q(uint64_t(amount), uint64_t(amount >> 64));
    o[4] = q(t.pending_id.lo, t.pending_id.hi);
    o[5] = q(uint64_t(ud128), uint64_t(ud128 >> 64));
    o[6] = make_uint4(uint32_t(ud64), uint32_t(ud64 >> 32), ud32, 0u);  // (timeout 0)
    o[7] = make_uint4(p.ledger, uint32_t(p.code) | (uint32_t(t.flags) << 16), uint32_t(ts),
                      uint32_t(ts >> 32));
    T.tr_status[pr] = post ? TB_PENDING_POSTED : TB_PENDING_VOIDED;
    // The balance words as atomic_sub_u128 / atomic_add_u128 would update them, the four low-word
    // adds in flight together and their carries after (FAST: both amounts are < 2^64,
    // classify_post_void): one atomic round trip on the event's path instead of four in sequence.
    const uint64_t pa = uint64_t(p_amount), am = uint64_t(amount);
    const bool posts = post && am != 0;
    tb_account_t* A = T.acc_rows;
    unsigned long long* dpe = reinterpret_cast<unsigned long long*>(&A[dr].debits_pending);
    unsigned long long* cpe = reinterpret_cast<unsigned long long*>(&A[cr].credits_pending);
    unsigned long long* dpo = reinterpret_cast<unsigned long long*>(&A[dr].debits_posted);
    unsigned long long* cpo = reinterpret_cast<unsigned long long*>(&A[cr].credits_posted);
    const uint64_t o_dpe = atomicAdd(dpe, 0ull - pa);
    const uint64_t o_cpe = atomicAdd(cpe, 0ull - pa);
    uint64_t o_dpo = 0, o_cpo = 0;
    if (posts) {
        o_dpo = atomicAdd(dpo, am);
        o_cpo = atomicAdd(cpo, am);
    }
    if (o_dpe < pa) atomicAdd(dpe + 1, ~0ull);  // (borrows: the hi word less one)
    if (o_cpe < pa) atomicAdd(cpe + 1, ~0ull);
    if (posts) {
        if (o_dpo + am < o_dpo && atomicAdd(dpo + 1, 1ull) + 1 >= kHazardHiLimit)
            acc_hazard_set(T.acc_index, T.acc_entry_of, dr, kHazardHigh);
        if (o_cpo + am < o_cpo && atomicAdd(cpo + 1, 1ull) + 1 >= kHazardHiLimit)
            acc_hazard_set(T.acc_index, T.acc_entry_of, cr, kHazardHigh);
    }
    if (p.timeout != 0)
        c.pnt_call[k] = (p.timestamp + uint64_t(p.timeout) * TB_NS_PER_S) | kPntReset;
}

// One event of tr_commit: applied (committed FAST), done (final DONE), ts_applied (its timestamp).
__device__ inline void commit_event(const Tables& T, const Call<tb_transfer_t>& c, uint32_t k,
                                    unsigned int call_flags, bool& applied, bool& done,
                                    bool& slow_out, uint64_t& ts_applied,
                                    const ChainPre pre, uint64_t* expiry_row) {
    applied = false;
    done = false;
    slow_out = false;
    ts_applied = 0;
    const uint8_t info = c.ev_info[k];
    const uint8_t cls = info & kInfoClassMask;
    const uint64_t row = c.row_base + k;
    const uint64_t ref = row + 1;
    const bool pnt_rec = (call_flags & kFlagPostVoid) || c.pnt_force;
    if (pnt_rec) c.pnt_call[k] = 0;  // (the replay records its own)
    bool slow = cls == kClassSlow || (call_flags & kFlagImported);
    if (cls == kClassFast) {
        FastRec fr = pre.has_fr ? pre.fr : fast_record(T, c, k, call_flags, info);
        const uint32_t s = fr.s, dr = fr.dr, cr = fr.cr;
        const uint64_t amount = fr.amount;
        const bool lean = (info & kInfoLean) != 0;
        const bool in_chain =
            pre.in_chain >= 0
                ? pre.in_chain != 0
                : (call_flags & kFlagChain) &&
                      ((c.events[k].flags & TB_TRANSFER_LINKED) ||
                       (k > 0 && (c.events[k - 1].flags & TB_TRANSFER_LINKED) &&
                        k != batch_start_of(c, batch_of_guess(c.batch_ends, c.n_batches, c.n, k))));
        // Fixed failures of post/voids racing an earlier FAST one (later_claim_status): DONE.
        uint32_t fixed = 0;
        if (!slow && (call_flags & kFlagPostVoid)) {
            if (in_chain) {
                fixed = pre.valid ? pre.fail : chain_fail_status(T, c, k, call_flags);
            } else if (fr.post_void) {
                // (pv_first once: fast_demoted below reads it from the record)
                fr.first = pv_first(c, k, c.events[k].pending_id) ? 1 : 0;
                fixed = fr.first ? 0u : later_claim_status(T, c, k, call_flags);
            }
        }
        if (fixed) {
            // Undo the speculative liveness and balance effects (as a demotion does), release
            // the id (neither status is transient: the slot becomes a tombstone).
            done = true;
            T.tr_live[row] = 0;
            if (!c.bal_items && !fr.post_void)
                apply_fast_deltas(T, dr, cr, (info & kInfoPending) != 0, amount, true);
            if (c.bal_items && c.pair_shift) {
                c.bal_items[k] = ~0ull;
            } else if (c.bal_items) {
                uint64_t* it = c.bal_items + 2 * uint64_t(k);
                it[0] = ~0ull;
                it[1] = ~0ull;
            }
            c.results[k].status = fixed;
            // (the id's release waits for stage_out: other threads of this kernel read slots)
            const uint64_t fs = s != kNone32 ? uint64_t(s) : transfer_slot_find(T, c, c.events[k].id);
            if (fs != kNone && (T.tr.slots[fs] & kRefMask) == ref)
                c.fix_slots[atomicAdd(&T.scalars->fixed, 1ull)] = uint32_t(fs);
        } else if (slow || fast_demoted(T, c, k, call_flags, fr) ||
                   (in_chain && (pre.valid ? pre.demoted : chain_demoted(T, c, k, call_flags)))) {
            // Demoted: undo the speculative liveness and balance items (or, in a call without
            // items, the deltas ingest applied); the replay decides.
            slow = true;
            T.tr_live[row] = 0;
            if (!c.bal_items && !fr.post_void)
                apply_fast_deltas(T, dr, cr, (info & kInfoPending) != 0, amount, true);
            if (c.bal_items && c.pair_shift) {
                c.bal_items[k] = ~0ull;
            } else if (c.bal_items) {
                uint64_t* it = c.bal_items + 2 * uint64_t(k);
                it[0] = ~0ull;
                it[1] = ~0ull;
            }
            if (lean) {  // the replay reads the record
                const uint64_t fs = s != kNone32 ? uint64_t(s) : transfer_slot_find(T, c, c.events[k].id);
                c.ev_slot[k] = fs == kNone ? kNone32 : uint32_t(fs);
                c.ev_dr[k] = dr;
                c.ev_cr[k] = cr;
            }
        } else if (fr.post_void) {
            applied = true;
            ts_applied = c.results[k].timestamp;
            commit_post_void(T, c, k, row, ts_applied, dr, cr);
        } else {
            applied = true;
            ts_applied = c.results[k].timestamp;
            const bool pending = (info & kInfoPending) != 0;
            // (a call without balance items: ingest applied the deltas; a wide pair item is the
            // balance window's)
            if (c.bal_items && !c.pair_shift && !item_packable(c, amount))
                apply_fast_deltas(T, dr, cr, pending, amount, false);
            if (pending && (info & kInfoTimeout)) {
                *expiry_row = row;  // (appended by the wave: tr_commit)
                const uint64_t expires_at = ts_applied + T.tr_rows[row].timeout * TB_NS_PER_S;
                // With post/void in the call the order of updates matters (a post/void resets
                // pulse_next_timestamp when it names its expiry): recorded at the event, resolved
                // in call order after the replay (pnt_resolve).
                if (pnt_rec) c.pnt_call[k] = expires_at;
                else atomicMin(&T.scalars->pulse_next_timestamp, (unsigned long long)expires_at);
            }
        }
    } else if (!slow && cls == kClassDone) {
        done = true;
        if (info & kInfoPostLookup) {
            const uint32_t s = c.ev_slot[k];
            const uint32_t dr = c.ev_dr[k], cr = c.ev_cr[k];
            if ((call_flags & kFlagDuplicate) && (T.tr.slots[s] & kRefMask) != ref) {
                slow = true;  // a later duplicate: its outcome follows the earlier event's
            } else if ((info & kInfoClosedDep) && (call_flags & kFlagClosable) &&
                       (T.acc_closable[dr] == c.epoch || T.acc_closable[cr] == c.epoch)) {
                slow = true;
            } else {
                // transient_error (:3215-3252): the id stays taken (orphan); else released.
                if (tb_transfer_status_transient(c.results[k].status)) {
                    T.tr_rows[row].id = c.events[k].id;
                    T.tr.slots[s] |= kOrphanBit;
                } else {
                    T.tr.slots[s] = kTomb;
                }
            }
        }
        if (slow) done = false;
        else T.tr_live[row] = 0;
    }
    c.ev_slow[k] = slow;
    slow_out = slow;
}

// The planes (chain_pre_planes) of a call that raised a commit flag and has linked chains: the
// per-event facts chain_pre_wave gathers, one ballot per plane.
__global__ void tr_chain_planes(Tables T, Call<tb_transfer_t> c) {
    const unsigned int call_flags = T.scalars->flags;
    if (!(call_flags & kCommitFlags) || !(call_flags & kFlagChain)) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    for (uint64_t kb = uint64_t(blockIdx.x) * blockDim.x + (threadIdx.x & ~63u); kb < c.n;
         kb += stride) {
        const uint32_t k = uint32_t(kb) + lane;
        const bool active = k < c.n;
        bool linked = false, prev_linked = false, open = false;
        uint8_t cls = 0, info = 0;
        if (active) {
            linked = (c.events[k].flags & TB_TRANSFER_LINKED) != 0;
            const bool pl = k > 0 && (c.events[k - 1].flags & TB_TRANSFER_LINKED);
            if (linked || pl) {
                const uint32_t b = batch_of_guess(c.batch_ends, c.n_batches, c.n, k);
                const uint32_t bs = batch_start_of(c, b), be = c.batch_ends[b];
                prev_linked = pl && k > bs;
                open = linked && k + 1 >= be;  // linked_event_chain_open
            }
            info = c.ev_info[k];
            cls = info & kInfoClassMask;
        }
        const bool in_chain = active && (linked || prev_linked);
        bool pd = false;
        uint32_t lc = 0;
        if (in_chain && cls == kClassFast) {
            const FastRec fr = fast_record(T, c, k, call_flags, info);
            pd = fast_demoted(T, c, k, call_flags, fr);
            if (pd && (call_flags & kFlagPostVoid)) lc = later_claim_status(T, c, k, call_flags);
        }
        const uint64_t w0 = __ballot(active && !prev_linked);
        const uint64_t w1 = __ballot(active && (!linked || open));
        const uint64_t w2 = __ballot(open);
        const uint64_t w3 = __ballot(active && cls == kClassFast);
        const uint64_t w4 = __ballot(pd);
        const uint64_t w5 = __ballot(lc == TB_CT_PENDING_TRANSFER_ALREADY_POSTED);
        const uint64_t w6 = __ballot(lc == TB_CT_PENDING_TRANSFER_ALREADY_VOIDED);
        if (lane == 0) {
            unsigned long long* o = c.chain_planes + (kb / 64) * kPlWords;
            o[kPlHead] = w0;
            o[kPlEnd] = w1;
            o[kPlOpen] = w2;
            o[kPlFast] = w3;
            o[kPlDemoted] = w4;
            o[kPlPosted] = w5;
            o[kPlVoided] = w6;
        }
    }
}

// tr_commit's early signal (Call::commit_done). What the host reads there are scalar words that
// tr_commit changes only with agent-scope atomics, each workgroup's by its lane 0 at the end
// (tr_ingest's flags were final at the kernel boundary), so a workgroup is counted once lane 0's
// atomics have completed (its vector memory counter drained) -- no L2 write-back per workgroup,
// which an agent-scope release is (+3.5 us on config 3's tr_commit). The last one acquires, reads
// the words with agent-scope atomic loads, copies them to the mapped copy, and publishes the
// sequence word at system scope. (A table-full flag another lane may raise is read again at the call's end.)
// The call's scalar words are not cleared: the kernels queued behind tr_commit still run.
__device__ inline void commit_signal(const Tables& T, const Call<tb_transfer_t>& c) {
    __shared__ bool last;
    if (threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = atomicAdd(c.commit_done, 1u) == gridDim.x - 1;
        if (last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            atomicExch(c.commit_done, 0u);
        }
    }
    __syncthreads();
    if (!last || threadIdx.x >= 64) return;
    constexpr uint32_t words = uint32_t(sizeof(DevScalars) / 8);
    static_assert(words <= 64, "one word a lane");
    const unsigned long long* src = reinterpret_cast<const unsigned long long*>(T.scalars);
    if (threadIdx.x < words)
        c.commit_scalars[threadIdx.x] =
            __hip_atomic_load(src + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // (the wave's copies before lane 0's release, as in ingest_finish)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (threadIdx.x == 0)
        __hip_atomic_store(c.commit_seq, c.commit_seq_val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// tr_commit: when ingest raised no commit flag, every event is a confirmed FAST event whose
// effects ingest already wrote; only the call's counters remain (from ingest's speculative
// ones). Otherwise every event is re-validated.
__device__ inline void tr_commit_body(const Tables& T, const Call<tb_transfer_t>& c);
__global__ void tr_commit(Tables T, Call<tb_transfer_t> c) {
    if (c.finish_done && c.finish_done[1] == c.epoch) return;  // (tr_ingest ended the call)
    tr_commit_body(T, c);
    if (c.commit_done) commit_signal(T, c);
}

__device__ inline void tr_commit_body(const Tables& T, const Call<tb_transfer_t>& c) {
    const unsigned int call_flags = T.scalars->flags;
    if (!(call_flags & kCommitFlags)) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {  // (atomics: commit_signal reads them)
            const unsigned long long ts = T.scalars->spec_ts_max;
            if (ts > T.scalars->transfers_key_max) atomicMax(&T.scalars->transfers_key_max, ts);
            atomicAdd(&T.scalars->stats[1], T.scalars->spec_fast);
        }
        return;
    }
    uint64_t n_applied = 0, n_done = 0, n_slow = 0, ts_max = 0;
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    // A block-uniform loop: the workgroup's expires_at entries take one reservation (one returning
    // add on expiry_count a workgroup, not a wave: same-address atomics serialise at ~11 ns on
    // MI355X, and config 4's every wave appends). chain_pre_wave combines the wave's lanes; a wave
    // wholly past the call skips it (its bit planes end with the call).
    __shared__ unsigned int exp_cnt[kBlock / 64];
    __shared__ unsigned long long exp_base;
    const uint32_t wv = threadIdx.x >> 6;
    for (uint64_t kb0 = uint64_t(blockIdx.x) * blockDim.x; kb0 < c.n; kb0 += stride) {
        const uint64_t kb = kb0 + (threadIdx.x & ~63u);
        const uint32_t k = uint32_t(kb) + (threadIdx.x & 63);
        const bool active = k < c.n;
        ChainPre pre{false, false, 0, -1, false, FastRec{}};
        if (kb < c.n) pre = chain_pre_wave(T, c, k, active, call_flags);
        uint64_t exp_row = kNone;
        if (active) {
            bool applied, done, slow;
            uint64_t ts;
            commit_event(T, c, k, call_flags, applied, done, slow, ts, pre, &exp_row);
            n_applied += applied;
            n_done += done;
            n_slow += slow;
            ts_max = ts > ts_max ? ts : ts_max;
        }
        const uint32_t lane = threadIdx.x & 63;
        const uint64_t want = __ballot(exp_row != kNone);
        if (lane == 0) exp_cnt[wv] = uint32_t(__popcll(want));
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned int total = 0;
            for (uint32_t w = 0; w < kBlock / 64; w++) total += exp_cnt[w];
            exp_base = total ? atomicAdd(&T.scalars->expiry_count, (unsigned long long)total) : 0;
        }
        __syncthreads();
        if (exp_row != kNone) {
            uint64_t i = exp_base + __popcll(want & ((1ull << lane) - 1));
            for (uint32_t w = 0; w < wv; w++) i += exp_cnt[w];
            if (i < T.expiry_capacity) T.expiry[i] = exp_row;
            else atomicOr(&T.scalars->flags, kFlagTableFull);
        }
        __syncthreads();  // (exp_cnt and exp_base are the next iteration's)
    }
    // transfers objects tree key_range (groove.zig:1780): the largest committed timestamp.
    n_applied = block_reduce(n_applied, OpAdd());
    n_done = block_reduce(n_done, OpAdd());
    n_slow = block_reduce(n_slow, OpAdd());
    ts_max = block_reduce(ts_max, OpMax());
    if (threadIdx.x == 0) {
        if (ts_max) atomicMax(&T.scalars->transfers_key_max, (unsigned long long)ts_max);
        if (n_applied) atomicAdd(&T.scalars->stats[1], (unsigned long long)n_applied);
        if (n_done) atomicAdd(&T.scalars->stats[3], (unsigned long long)n_done);
        if (n_slow) atomicAdd(&T.scalars->stats[0], (unsigned long long)n_slow);
    }
}

struct BalTarget {
    tb_account_t* rows;
    AccIndex index;
    const uint32_t* entry_of;
};

__device__ inline void add_field(const BalTarget& B, uint32_t key, u128 sum, bool shared) {
    if (sum == 0) return;
    tb_uint128_t* field = account_field(B.rows, key);
    uint64_t hi;
    if (shared) {
        hi = atomic_add_u128(field, sum);
    } else {
        const tb_uint128_t v = W(U(*field) + sum);
        *field = v;
        hi = v.hi;
    }
    if (hi >= kHazardHiLimit) acc_hazard_set(B.index, B.entry_of, key >> 2, kHazardHigh);
}

// Key spaces too large for the buckets and not sparse (bal_hash_apply): each workgroup sums a slice
// of kHashSliceItems items per account field in an LDS hash table (open addressing on the key,
// u64 sums: amounts < 2^46 at these key widths, 2^11 items per slice) and adds every field's slice
// sum to its row with u128 atomics -- a hot account costs one atomic per workgroup instead of one
// per item, a cold one a u128 atomic on the row. An item whose probe window is full takes its
// atomic at once. (This replaces a library radix sort of the items and a run reduction.)
constexpr uint32_t kHashThreads = 256;
constexpr uint32_t kHashSlots = 4096;
constexpr uint32_t kHashItemsPerLane = 8;
constexpr uint32_t kHashSliceItems = kHashThreads * kHashItemsPerLane;
constexpr uint32_t kHashProbes = 32;
constexpr uint32_t kHashEmpty = 0xFFFFFFFFu;

__global__ void __launch_bounds__(kHashThreads) bal_hash_apply(BalTarget rows, const uint64_t* items,
                                                               uint64_t n, uint32_t key_bits,
                                                               uint32_t key_end) {
    __shared__ uint32_t hkey[kHashSlots];
    __shared__ unsigned long long hsum[kHashSlots];
    for (uint32_t i = threadIdx.x; i < kHashSlots; i += kHashThreads) {
        hkey[i] = kHashEmpty;
        hsum[i] = 0;
    }
    __syncthreads();
    const uint64_t kmask = (1ull << key_bits) - 1;
    const uint64_t base = uint64_t(blockIdx.x) * kHashSliceItems;
    // items base + 2 (t + j * kHashThreads), + 1: coalesced 16-byte loads (n is even)
    uint64_t it[kHashItemsPerLane];
#pragma unroll
    for (uint32_t j = 0; j < kHashItemsPerLane / 2; j++) {
        const uint64_t i = base + 2 * (uint64_t(threadIdx.x) + uint64_t(j) * kHashThreads);
        uint4 q = make_uint4(~0u, ~0u, ~0u, ~0u);
        if (i < n) q = *reinterpret_cast<const uint4*>(items + i);
        it[2 * j] = (uint64_t(q.y) << 32) | q.x;
        it[2 * j + 1] = (uint64_t(q.w) << 32) | q.z;
    }
#pragma unroll
    for (uint32_t j = 0; j < kHashItemsPerLane; j++) {
        const uint64_t k64 = it[j] & kmask;
        if (k64 >= key_end) continue;
        const uint32_t key = uint32_t(k64);
        const uint64_t amount = it[j] >> key_bits;
        uint32_t h = (key * 0x9E3779B1u) >> (32 - 12);
        bool placed = false;
        for (uint32_t p = 0; p < kHashProbes && !placed; p++, h = (h + 1) & (kHashSlots - 1)) {
            uint32_t cur = hkey[h];
            if (cur == kHashEmpty) cur = atomicCAS(&hkey[h], kHashEmpty, key);
            if (cur == kHashEmpty || cur == key) {
                atomicAdd(&hsum[h], (unsigned long long)amount);
                placed = true;
            }
        }
        if (!placed) add_field(rows, key, amount, true);
    }
    static_assert(kHashSlots == 1u << 12, "hash width");
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kHashSlots; i += kHashThreads)
        if (hkey[i] != kHashEmpty) add_field(rows, hkey[i], hsum[i], true);
}

// ---- the balance window path (key spaces of <= 2^14 accounts, e.g. config 2) -----
//
// Pair items (Call::pair_shift = s): one u64 per FAST event carries both accounts, the pending bit
// and the amount. Fields are keyed field-major, key = f << s | row with f = 0 debits_posted,
// 1 credits_posted, 2 debits_pending, 3 credits_pending: the posted fields of up to 2^14 accounts
// fall in the first kWindowKeys keys. bal_window_accumulate: one workgroup per CU sums a
// contiguous slice of the items into u32 LDS counters (the window; the u32 carries of a returning
// LDS add, and amount bits above 32, go to a per-key u64 `carry` word with a global atomic --
// never for config 2), fields outside the window with u128 atomics on the row; then writes its
// counters as u32 partials. bal_window_apply: one lane per window key sums the partials and the
// carry in u128 and adds them to the row field (plain read-modify-write: one lane per field).
// Item traffic: 8 B written by ingest and read once, plus 4 B per window key per workgroup.

constexpr uint32_t kWindowKeys = 32768;  // u32 counters: 128 KB of LDS
constexpr uint32_t kWindowThreads = 1024;
constexpr uint32_t kWindowGridMax = 256;  // one workgroup per CU
constexpr uint32_t kWindowShiftMax = 14;

// Byte offset in the Account row of window field f (see above).
__device__ inline uint32_t window_field_offset(uint32_t f) {
    return f == 0 ? 32 : f == 1 ? 64 : f == 2 ? 16 : 48;
}

__device__ inline void window_field_add(const BalTarget& B, uint32_t row, uint32_t f, u128 sum,
                                        bool shared) {
    if (sum == 0) return;
    tb_uint128_t* field = reinterpret_cast<tb_uint128_t*>(
        reinterpret_cast<uint8_t*>(&B.rows[row]) + window_field_offset(f));
    uint64_t hi;
    if (shared) {
        hi = atomic_add_u128(field, sum);
    } else {
        const tb_uint128_t v = W(U(*field) + sum);
        *field = v;
        hi = v.hi;
    }
    if (hi >= kHazardHiLimit) acc_hazard_set(B.index, B.entry_of, row, kHazardHigh);
}

// A workgroup's slice of the items: [b0, b1) with `per` even (uint4 loads). The AccountEvents
// emit of window calls (events.hpp, ae_window_emit) walks the same slices.
__host__ __device__ inline uint32_t window_slice_per(uint32_t n, uint32_t nwg) {
    return ((n + nwg - 1) / nwg + 1) & ~1u;
}

// (+ per workgroup: the count of its slice's items -- the created events of a call the
// AccountEvents window takes -- and kFlagWideSums when a u32 window counter carried)
// Calls with a wide item (kFlagWideItems: an amount too wide to pack, up to 2^64) take the wide
// layout instead: workgroup 2 w + f sums slice w of the items into field f (0 debits_posted, 1
// credits_posted) only, an amount's low and high 32 bits in two u32 LDS counters per account (the
// same 128 KB; a low counter's wrap carries into the high one, a high counter's wrap -- 2^64 --
// takes a global atomic), and writes both as partials. No AccountEvents window takes such a call.
constexpr uint32_t kWindowHalf = kWindowKeys / 2;  // accounts per field in the wide layout

// (+ per workgroup: the count of its slice's items -- the created events of a call the
// AccountEvents window takes -- and kFlagWideSums when a u32 window counter carried)
__global__ void __launch_bounds__(kWindowThreads) bal_window_accumulate(
    BalTarget B, const uint64_t* items, const uint64_t* wide_amounts, uint32_t n, uint32_t ps,
    uint32_t wkeys, uint32_t* partials, unsigned long long* carry, unsigned int* slice_count,
    unsigned int* call_flags) {
    __shared__ uint32_t acc[kWindowKeys];
    __shared__ uint32_t wave_items[kWindowThreads / 64];
    const bool wide_layout = (*call_flags & kFlagWideItems) != 0;
    for (uint32_t i = threadIdx.x; i < kWindowKeys; i += kWindowThreads) acc[i] = 0;
    __syncthreads();
    const uint32_t slices = wide_layout ? (gridDim.x + 1) / 2 : gridDim.x;
    const uint32_t w = wide_layout ? blockIdx.x >> 1 : blockIdx.x;
    const uint32_t wf = blockIdx.x & 1;  // (wide layout: this workgroup's field)
    const uint32_t per = window_slice_per(n, slices);
    const uint32_t b0 = min(w * per, n);
    const uint32_t b1 = b0 + per < n ? b0 + per : n;
    const uint64_t rmask = (1ull << ps) - 1;
    const uint64_t amask = pair_amount_mask(ps);
    uint32_t* lo_acc = acc;
    uint32_t* hi_acc = acc + kWindowHalf;
    uint32_t n_items = 0;
    bool wide = false;
    auto add = [&](uint32_t f, uint32_t row, uint64_t amount) {
        const uint32_t key = (f << ps) | row;
        if (key < wkeys) {
            const uint32_t lo = uint32_t(amount);
            const uint32_t old = atomicAdd(&acc[key], lo);
            const uint64_t hi = (amount >> 32) + (uint32_t(old + lo) < old ? 1 : 0);
            if (hi) {
                atomicAdd(&carry[key], (unsigned long long)hi);
                wide = true;
            }
        } else {
            window_field_add(B, row, f, amount, true);
        }
    };
    auto add_wide = [&](uint32_t row, uint64_t amount) {  // field wf, row < kWindowHalf
        const uint32_t lo = uint32_t(amount);
        const uint32_t old = atomicAdd(&lo_acc[row], lo);
        // (u64: an amount's high word 2^32 - 1 plus the low word's carry is 2^32)
        const uint64_t hi = (amount >> 32) + (uint32_t(old + lo) < old ? 1u : 0u);
        if (hi) {
            const uint32_t h = uint32_t(hi);
            const uint32_t old_hi = h ? atomicAdd(&hi_acc[row], h) : 0u;
            const uint32_t wraps = uint32_t(hi >> 32) + (uint32_t(old_hi + h) < old_hi ? 1u : 0u);
            if (wraps)  // (2^64 each)
                atomicAdd(&carry[(wf << ps) | row], (unsigned long long)wraps << 32);
        }
    };
    auto item = [&](uint64_t x, uint32_t e) {
        if (x == ~0ull) return;
        n_items++;
        const uint32_t dr = uint32_t(x & rmask), cr = uint32_t((x >> ps) & rmask);
        const uint32_t pend = uint32_t(x >> (2 * ps)) & 1u;
        uint64_t amount = x >> (2 * ps + 1);
        if (amount == amask) amount = wide_amounts[e];
        if (wide_layout) {
            if (pend) window_field_add(B, wf ? cr : dr, wf ? 3 : 2, amount, true);
            else add_wide(wf ? cr : dr, amount);
            return;
        }
        add(pend ? 2 : 0, dr, amount);
        add(pend ? 3 : 1, cr, amount);
    };
    // Two items per lane per load, four loads in flight.
    uint32_t i = b0 + 2 * threadIdx.x;
    constexpr uint32_t kStep = 2 * kWindowThreads;
    for (; i + 3 * kStep + 1 < b1; i += 4 * kStep) {
        uint4 q[4];
#pragma unroll
        for (int j = 0; j < 4; j++) q[j] = *reinterpret_cast<const uint4*>(items + i + j * kStep);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            item((uint64_t(q[j].y) << 32) | q[j].x, i + j * kStep);
            item((uint64_t(q[j].w) << 32) | q[j].z, i + j * kStep + 1);
        }
    }
    for (; i < b1; i += kStep) {
        item(items[i], i);
        if (i + 1 < b1) item(items[i + 1], i + 1);
    }
    if (__any(wide) && (threadIdx.x & 63) == 0) atomicOr(call_flags, kFlagWideSums);
    for (int off = 32; off > 0; off >>= 1) n_items += __shfl_xor(n_items, off);
    if ((threadIdx.x & 63) == 0) wave_items[threadIdx.x >> 6] = n_items;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t t = 0;
        for (uint32_t v = 0; v < kWindowThreads / 64; v++) t += wave_items[v];
        slice_count[blockIdx.x] = t;
    }
    if (wide_layout) {
        // partials of workgroup g: [g][0, rows) low sums, [g][kWindowHalf, + rows) high sums
        uint32_t* out = partials + uint64_t(blockIdx.x) * kWindowKeys;
        const uint32_t rows = 1u << ps;
        for (uint32_t k = threadIdx.x; k < rows; k += kWindowThreads) {
            out[k] = lo_acc[k];
            out[kWindowHalf + k] = hi_acc[k];
        }
        return;
    }
    uint32_t* out = partials + uint64_t(blockIdx.x) * wkeys;
    for (uint32_t k = threadIdx.x; k < wkeys; k += kWindowThreads) out[k] = acc[k];
}

// One workgroup per 64 window keys: its 16 waves each sum every 16th workgroup's partials for
// those keys (coalesced 256-B rows), then LDS combines them -- 5,000 waves over the chip instead
// of one lane walking all partials of a key.
constexpr uint32_t kApplyThreads = 1024;
// (kFlagWideSums when a key's total reaches 2^32: the AccountEvents window keeps u32 sums)
__global__ void __launch_bounds__(kApplyThreads) bal_window_apply(
    BalTarget B, const uint32_t* partials, uint32_t nwg, uint32_t ps, uint32_t wkeys,
    uint64_t rows_used, unsigned long long* carry, unsigned int* call_flags) {
    __shared__ uint64_t part[kApplyThreads / 64][64];
    __shared__ uint64_t part_hi[kApplyThreads / 64][64];
    const bool wide_layout = (*call_flags & kFlagWideItems) != 0;
    const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const uint32_t k = blockIdx.x * 64 + lane;
    const uint32_t row = k & ((1u << ps) - 1), f = k >> ps;
    uint64_t s = 0, sh = 0;
    if (k < wkeys && !wide_layout) {
        uint32_t w = wv;
        for (; w + 3 * (kApplyThreads / 64) < nwg; w += 4 * (kApplyThreads / 64)) {
            uint32_t x[4];
#pragma unroll
            for (int j = 0; j < 4; j++)
                x[j] = partials[uint64_t(w + j * (kApplyThreads / 64)) * wkeys + k];
#pragma unroll
            for (int j = 0; j < 4; j++) s += x[j];
        }
        for (; w < nwg; w += kApplyThreads / 64) s += partials[uint64_t(w) * wkeys + k];
    } else if (k < wkeys && f < 2) {
        // (wide layout: the workgroups 2 w + f of field f, low and high sums; the pending fields
        // took atomics)
        for (uint32_t g = 2 * wv + f; g < nwg; g += 2 * (kApplyThreads / 64)) {
            s += partials[uint64_t(g) * kWindowKeys + row];
            sh += partials[uint64_t(g) * kWindowKeys + kWindowHalf + row];
        }
    }
    part[wv][lane] = s;
    part_hi[wv][lane] = sh;
    __syncthreads();
    if (wv != 0 || k >= wkeys) return;
    for (uint32_t j = 1; j < kApplyThreads / 64; j++) {
        s += part[j][lane];
        sh += part_hi[j][lane];
    }
    if (row >= rows_used) return;
    u128 sum = u128(s) + (u128(sh) << 32);
    const unsigned long long c = carry[k];
    if (c) {
        sum += u128(c) << 32;
        carry[k] = 0;
    }
    if (c || (s >> 32) || sh) atomicOr(call_flags, kFlagWideSums);
    window_field_add(B, row, f, sum, false);
}

// ---- the bucketed balance path ------------------------------------------------
//
// ingest counts the items per bucket (block histograms); bal_bucket_plan lays the buckets out
// (offsets, cursors, slices of <= kSliceItems); bal_bucket_scatter moves the items into their
// buckets (one cursor reservation per block and bucket); bal_bucket_accumulate sums one slice per
// block in LDS (64-bit LDS atomics on 8192 keys) and writes the slice's partial sums;
// bal_bucket_apply adds, per key, its bucket's partials in u128 to the account field.
// Counts come from ingest and may exceed the items that survive tr_commit (demotions), so the
// buckets' real ends are the cursors after the scatter.

struct BucketPlan {
    unsigned int* counts;   // [kBucketsMax] from ingest
    unsigned int* cursor;   // [kBucketsMax] bucket fill positions
    unsigned int* offset;   // [kBucketsMax + 1]
    unsigned int* slice_base;  // [kBucketsMax + 1]
    uint32_t n_buckets;
};

__global__ void bal_bucket_plan(BucketPlan P) {
    if (threadIdx.x != 0) return;
    unsigned int off = 0, sl = 0;
    for (uint32_t b = 0; b < P.n_buckets; b++) {
        P.offset[b] = off;
        P.cursor[b] = off;
        P.slice_base[b] = sl;
        off += P.counts[b];
        sl += (P.counts[b] + kSliceItems - 1) / kSliceItems;
    }
    P.offset[P.n_buckets] = off;
    P.slice_base[P.n_buckets] = sl;
}

constexpr uint32_t kScatterPerLane = 16;
constexpr uint32_t kScatterTile = kBlock * kScatterPerLane;

__global__ void __launch_bounds__(kBlock) bal_bucket_scatter(BucketPlan P, const uint64_t* items,
                                                             uint64_t n, uint32_t key_bits,
                                                             uint32_t key_end, uint64_t* out) {
    __shared__ unsigned int cnt[kBucketsMax], base[kBucketsMax];
    for (uint32_t i = threadIdx.x; i < P.n_buckets; i += kBlock) cnt[i] = 0;
    __syncthreads();
    const uint64_t kmask = (1ull << key_bits) - 1;
    const uint64_t begin = uint64_t(blockIdx.x) * kScatterTile + uint64_t(threadIdx.x) * kScatterPerLane;
    uint64_t it[kScatterPerLane];
    unsigned int pos[kScatterPerLane];
    if (begin + kScatterPerLane <= n) {
        const uint4* p = reinterpret_cast<const uint4*>(items + begin);
#pragma unroll
        for (int i = 0; i < 8; i++) {
            const uint4 q = p[i];
            it[2 * i] = (uint64_t(q.y) << 32) | q.x;
            it[2 * i + 1] = (uint64_t(q.w) << 32) | q.z;
        }
    } else {
#pragma unroll
        for (int i = 0; i < (int)kScatterPerLane; i++) it[i] = begin + i < n ? items[begin + i] : ~0ull;
    }
#pragma unroll
    for (int i = 0; i < (int)kScatterPerLane; i++) {
        const uint64_t key = it[i] & kmask;
        pos[i] = key < key_end ? atomicAdd(&cnt[key >> kBucketShift], 1u) : ~0u;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < P.n_buckets; i += kBlock)
        base[i] = cnt[i] ? atomicAdd(&P.cursor[i], cnt[i]) : 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < (int)kScatterPerLane; i++)
        if (pos[i] != ~0u) out[base[(it[i] & kmask) >> kBucketShift] + pos[i]] = it[i];
}

__global__ void __launch_bounds__(kBlock) bal_bucket_accumulate(BucketPlan P, const uint64_t* bucketed,
                                                                uint32_t key_bits, uint64_t* partials) {
    __shared__ unsigned long long acc[kBucketKeys];
    const uint32_t s = blockIdx.x;
    if (s >= P.slice_base[P.n_buckets]) return;
    uint32_t b = 0;
    while (P.slice_base[b + 1] <= s) b++;
    for (uint32_t i = threadIdx.x; i < kBucketKeys; i += kBlock) acc[i] = 0;
    __syncthreads();
    const uint64_t begin = uint64_t(P.offset[b]) + uint64_t(s - P.slice_base[b]) * kSliceItems;
    const uint64_t filled = P.cursor[b];
    const uint64_t end = begin + kSliceItems < filled ? begin + kSliceItems : filled;
    const uint64_t kmask = (1ull << key_bits) - 1;
    // 8 independent loads in flight per lane, then their LDS adds.
    uint64_t j = begin + threadIdx.x;
    for (; j + 7 * kBlock < end; j += 8 * kBlock) {
        uint64_t x[8];
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = bucketed[j + i * kBlock];
#pragma unroll
        for (int i = 0; i < 8; i++)
            atomicAdd(&acc[(x[i] & kmask) & (kBucketKeys - 1)], (unsigned long long)(x[i] >> key_bits));
    }
    for (; j < end; j += kBlock) {
        const uint64_t x = bucketed[j];
        atomicAdd(&acc[(x & kmask) & (kBucketKeys - 1)], (unsigned long long)(x >> key_bits));
    }
    __syncthreads();
    uint64_t* out = partials + uint64_t(s) * kBucketKeys;
    for (uint32_t i = threadIdx.x; i < kBucketKeys; i += kBlock) out[i] = acc[i];
}

__global__ void bal_bucket_apply(BalTarget B, BucketPlan P, const uint64_t* partials,
                                 uint32_t key_end) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= key_end) return;
    const uint32_t b = k >> kBucketShift, local = k & (kBucketKeys - 1);
    u128 sum = 0;
    uint32_t s = P.slice_base[b];
    const uint32_t s_end = P.slice_base[b + 1];
    for (; s + 8 <= s_end; s += 8) {
        uint64_t x[8];
#pragma unroll
        for (int i = 0; i < 8; i++) x[i] = partials[uint64_t(s + i) * kBucketKeys + local];
#pragma unroll
        for (int i = 0; i < 8; i++) sum += x[i];
    }
    for (; s < s_end; s++) sum += partials[uint64_t(s) * kBucketKeys + local];
    add_field(B, k, sum, false);  // one thread per key: plain read-modify-write
}

// ================================ the ordered replay ========================================

template <typename Event>
__device__ inline void replay_chain_step_at(Replay& R, const Call<Event>& c, uint32_t k,
                                            const Event& ev, const StepInfo& si, const EvRefs& x,
                                            bool is_transfers, bool& chain_open,
                                            uint32_t& chain_start, bool& chain_broken) {
    const Tables& T = R.T;
    const uint32_t b = si.batch;
    const uint64_t ts_event = si.ts_event;
    const uint16_t linked_flag = is_transfers ? TB_TRANSFER_LINKED : TB_ACCOUNT_LINKED;
    const uint16_t imported_flag = is_transfers ? TB_TRANSFER_IMPORTED : TB_ACCOUNT_IMPORTED;
    const uint16_t f = ev.flags;
    uint32_t status = 0;
    uint64_t ts_actual = ts_event;
    R.pos = k;
    // (one_chain: every event links to the next, and the batch's last event closes the chain)
    const bool linked = c.one_chain || (f & linked_flag);
    const bool last = (si.flags & StepInfo::kLastOfBatch) != 0;

    do {  // execute_create's loop body (:3030-3105)
        if (linked) {
            if (!chain_open) {
                chain_open = true;
                chain_start = k;
                chain_broken = false;
                R.scope_open();
            }
            if (last && !c.one_chain) {
                status = TB_CT_LINKED_EVENT_CHAIN_OPEN;
                break;
            }
        }
        if (chain_broken) {
            status = TB_CT_LINKED_EVENT_FAILED;
            break;
        }
        const bool batch_imported = (si.flags & StepInfo::kBatchImported) != 0;
        const bool imported = (f & imported_flag) != 0;
        if (batch_imported != imported) {
            if (is_transfers)
                status = imported ? TB_CT_IMPORTED_EVENT_NOT_EXPECTED : TB_CT_IMPORTED_EVENT_EXPECTED;
            else
                status = imported ? TB_CA_IMPORTED_EVENT_NOT_EXPECTED : TB_CA_IMPORTED_EVENT_EXPECTED;
            break;
        }
        if (imported) {
            if (ev.timestamp < TB_TIMESTAMP_MIN || ev.timestamp > TB_TIMESTAMP_MAX) {
                status = is_transfers ? TB_CT_IMPORTED_EVENT_TIMESTAMP_OUT_OF_RANGE
                                      : TB_CA_IMPORTED_EVENT_TIMESTAMP_OUT_OF_RANGE;
                break;
            }
            if (ev.timestamp >= c.batch_ts[b]) {
                status = is_transfers ? TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_ADVANCE
                                      : TB_CA_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_ADVANCE;
                break;
            }
        } else if (ev.timestamp != 0) {
            status = TB_CT_TIMESTAMP_MUST_BE_ZERO;
            break;
        }
        uint64_t ts = ts_event;
        if constexpr (__is_same(Event, tb_transfer_t)) {
            status = replay_create_transfer(R, c, k, ts_event, ev, x, &ts);
            if (status == TB_STATUS_CREATED || status == TB_CT_EXISTS) ts_actual = ts;
        } else {
            status = replay_create_account(R, c, k, ts_event, ev, x, &ts);
            if (status == TB_STATUS_CREATED || status == TB_CA_EXISTS) ts_actual = ts;
        }
    } while (0);

    // The event becomes the holder of its id's slot when it created or orphaned the id.
    const bool transient = is_transfers && status != TB_STATUS_CREATED &&
                           tb_transfer_status_transient(status);
    if ((status == TB_STATUS_CREATED || transient) && x.slot != kNone32) {
        unsigned long long* slots = is_transfers ? T.tr.slots : T.acc.slots;
        slots[x.slot] = (c.row_base + k + 1) | id_tag(ev.id);
    }
    if (status != TB_STATUS_CREATED && chain_open && !chain_broken) {
        chain_broken = true;
        R.scope_close(true);
        for (uint32_t ci = chain_start; ci < k; ci++)
            c.results[ci].status = TB_CT_LINKED_EVENT_FAILED;
    }
    tb_create_result_t res;
    res.timestamp = ts_actual;
    res.status = status;
    res.reserved = 0;
    c.results[k] = res;
    if (chain_open && (!linked || status == TB_CT_LINKED_EVENT_CHAIN_OPEN ||
                       (c.one_chain && last))) {
        if (!chain_broken) R.scope_close(false);
        chain_open = false;
        chain_broken = false;
    }
}

// The event's batch facts, from the batch bounds (serial replay) or precomputed (flow plan).
template <typename Event>
__device__ inline StepInfo step_info(const Call<Event>& c, uint32_t k, uint16_t imported_flag) {
    const uint32_t b = batch_of_guess(c.batch_ends, c.n_batches, c.n, k);
    StepInfo si;
    si.ts_event = ts_event_of(c, b, k);
    si.batch = b;
    si.flags = (k == c.batch_ends[b] - 1 ? StepInfo::kLastOfBatch : 0u) |
               ((c.events[batch_start_of(c, b)].flags & imported_flag) ? StepInfo::kBatchImported
                                                                        : 0u);
    return si;
}

template <typename Event>
__device__ inline void replay_chain_step(Replay& R, const Call<Event>& c, uint32_t k,
                                         bool is_transfers, bool& chain_open,
                                         uint32_t& chain_start, bool& chain_broken) {
    const Event ev = c.events[k];
    const StepInfo si =
        step_info(c, k, is_transfers ? uint16_t(TB_TRANSFER_IMPORTED) : uint16_t(TB_ACCOUNT_IMPORTED));
    replay_chain_step_at<Event>(R, c, k, ev, si, ev_refs(c, k), is_transfers, chain_open,
                                chain_start, chain_broken);
}

template <typename Event>
__global__ void replay_kernel(Tables T, Call<Event> c, int is_transfers) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    Replay R(T);
    if (is_transfers && ((T.scalars->flags & kFlagPostVoid) || c.pnt_force)) R.pnt_ops = c.pnt_call;
    bool chain_open = false, chain_broken = false;
    uint32_t chain_start = 0;
    const uint32_t n = T.scalars->slow_count;
    for (uint32_t i = 0; i < n; i++) {
        replay_chain_step<Event>(R, c, c.slow_list[i], is_transfers != 0, chain_open, chain_start,
                                 chain_broken);
        if (R.overflow) {
            atomicOr(&T.scalars->flags, kFlagUndoOverflow);
            break;
        }
    }
    T.scalars->stats[2] = n;
}

// pulse_next_timestamp of a call with post/void, from the updates recorded per event (Call::
// pnt_call) in call order. `min` updates lower it; a reset fires when the value before it (the
// start value and every earlier `min`, while no reset has fired) equals its expiry, after which the
// value is timestamp_min, which no later update changes. So: prefix minima of the `min` updates,
// then "does any reset meet its prefix?"
__global__ void pnt_prep(const uint64_t* ops, uint32_t n, uint64_t* mins) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint64_t op = ops[k];
    mins[k] = (op == 0 || (op & kPntReset)) ? ~0ull : op;
}
__global__ void pnt_check(Tables T, const uint64_t* ops, uint32_t n, const uint64_t* prefix_min,
                          unsigned long long* fired) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint64_t op = ops[k];
    if (!(op & kPntReset)) return;
    uint64_t before = T.scalars->pulse_next_timestamp;
    if (k > 0 && prefix_min[k - 1] < before) before = prefix_min[k - 1];
    if (before == (op & ~kPntReset)) atomicOr(fired, 1ull);
}
__global__ void pnt_final(Tables T, uint32_t n, const uint64_t* prefix_min,
                          unsigned long long* fired) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    uint64_t v = T.scalars->pulse_next_timestamp;
    if (*fired) v = TB_TIMESTAMP_MIN;
    else if (n && prefix_min[n - 1] < v) v = prefix_min[n - 1];
    T.scalars->pulse_next_timestamp = v;
    *fired = 0;
}

// Id slots and liveness of events: created -> object, transient -> orphan, else tombstone.
template <typename Event>
__device__ inline void finalize_event(const Tables& T, const Call<Event>& c, uint32_t k,
                                      bool is_transfers) {
    const uint64_t row = c.row_base + k;
    const uint32_t status = c.results[k].status;
    const bool created = status == TB_STATUS_CREATED;
    const uint32_t s = c.ev_slot[k];
    unsigned long long* slots = is_transfers ? T.tr.slots : T.acc.slots;
    if (s != kNone32 && (slots[s] & kRefMask) == row + 1) {
        if (created) {
            // the slot names a committed object
        } else if (is_transfers && tb_transfer_status_transient(status)) {
            T.tr_rows[row].id = c.events[k].id;  // orphaned ids keep their key for probes
            slots[s] |= kOrphanBit;
        } else {
            slots[s] = kTomb;
        }
    }
    if (is_transfers) T.tr_live[row] = created;
    else T.acc_live[row] = created;
}

template <typename Event>
__global__ void finalize_slow(Tables T, Call<Event> c, int is_transfers) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= T.scalars->slow_count) return;
    finalize_event(T, c, c.slow_list[i], is_transfers != 0);
}

template <typename Event>
__global__ void finalize_all(Tables T, Call<Event> c, int is_transfers) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= c.n) return;
    finalize_event(T, c, k, is_transfers != 0);
}

// ================================ create_accounts ===========================================

__global__ void acc_prepare(Tables T, Call<tb_account_t> c) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    bool imported = false;
    if (k < c.n) {
        const tb_account_t* ev = c.events;
        const tb_account_t& a = ev[k];
        imported = (a.flags & TB_ACCOUNT_IMPORTED) != 0;
        uint64_t slot = kNone;
        if (!u128_is_zero(a.id) && !u128_is_max(a.id)) {
            const tb_account_t* rows = T.acc_rows;
            const uint64_t base = c.row_base;
            bool dup = false;
            slot = probe_claim(T.acc, a.id, base + k + 1, base, [&](uint64_t r) {
                return r >= base ? ev[r - base].id : rows[r].id;
            }, &dup);
            if (slot == kNone) atomicOr(&T.scalars->flags, kFlagTableFull);
        }
        c.ev_slot[k] = slot == kNone ? kNone32 : uint32_t(slot);
    }
    set_flag_any(T.scalars, imported, kFlagImported);
}

__global__ void acc_classify(Tables T, Call<tb_account_t> c) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    uint8_t cls = kClassDone;
    bool created = false;
    uint64_t ts_created = 0;
    if (k < c.n) {
        const uint32_t b = batch_of(c.batch_ends, c.n_batches, k);
        const uint64_t ts_event = ts_event_of(c, b, k);
        const tb_account_t a = c.events[k];
        const uint32_t bstart = batch_start_of(c, b);
        uint32_t status = 0;
        uint64_t ts = ts_event;
        const uint16_t f = a.flags;
        if (c.force_replay || (T.scalars->flags & kFlagImported) || (f & TB_ACCOUNT_LINKED) ||
            (k > bstart && (c.events[k - 1].flags & TB_ACCOUNT_LINKED))) {
            cls = kClassSlow;
        } else if (a.timestamp != 0) {
            status = TB_CA_TIMESTAMP_MUST_BE_ZERO;
        } else if (a.reserved != 0) {
            status = TB_CA_RESERVED_FIELD;
        } else if (f & TB_ACCOUNT_PADDING_MASK) {
            status = TB_CA_RESERVED_FLAG;
        } else if (u128_is_zero(a.id)) {
            status = TB_CA_ID_MUST_NOT_BE_ZERO;
        } else if (u128_is_max(a.id)) {
            status = TB_CA_ID_MUST_NOT_BE_INT_MAX;
        } else {
            const uint32_t s = c.ev_slot[k];
            if (s == kNone32) {
                cls = kClassSlow;
            } else {
                const uint64_t w = T.acc.slots[s];
                const uint64_t r = (w & kRefMask) - 1;
                if (r < c.row_base) {
                    const tb_account_t e = T.acc_rows[r];
                    status = create_account_exists(a, e, &ts);
                } else if (r != c.row_base + k) {
                    cls = kClassSlow;  // a later duplicate of an in-call id
                } else {
                    status = create_account_checks(a);
                    if (status == TB_STATUS_CREATED) {
                        T.acc_rows[c.row_base + k] = account_row_of(a, ts_event);
                        created = true;
                        ts_created = ts_event;
                    }
                }
            }
        }
        if (cls == kClassDone) {
            tb_create_result_t res;
            res.timestamp = (status == TB_CA_EXISTS || created) ? ts : ts_event;
            res.status = status;
            res.reserved = 0;
            c.results[k] = res;
        }
        c.ev_slow[k] = cls == kClassSlow;
    }
    for (int off = 32; off > 0; off >>= 1) {
        uint64_t o = __shfl_xor(ts_created, off);
        ts_created = o > ts_created ? o : ts_created;
    }
    if ((threadIdx.x & 63) == 0 && ts_created)
        atomicMax(&T.scalars->accounts_key_max, (unsigned long long)ts_created);
    count_stat(T.scalars, 1, created);
    count_stat(T.scalars, 3, k < c.n && cls == kClassDone && !created);
}

// The account index after a create_accounts call: cuckoo insertion of the accounts it created
// (only `ref` words move), then every entry the insertion wrote gets the rest of its image -- id
// low word, flags, hazard, ledger -- from the row it now names, and that row its entry index.
struct IndexBuild {
    uint32_t* dirty;         // entries written by the insertion
    unsigned int* counters;  // [0] dirty entries appended, [1] the dirty list overflowed
    uint32_t dirty_cap;
};

__global__ void acc_index_insert_rows(Tables T, uint64_t row_base, uint32_t n, IndexBuild B) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const uint64_t row = row_base + k;
    if (!T.acc_live[row]) return;
    if (!acc_index_insert(T.acc_index, T.acc_rows, uint32_t(row), B.dirty, &B.counters[0],
                          B.dirty_cap, &B.counters[1]))
        atomicOr(&T.scalars->flags, kFlagTableFull);
}

__device__ inline void acc_index_repair_entry(const Tables& T, uint64_t pos) {
    AccEntry* e = &T.acc_index.entries[pos];
    const uint32_t ref = e->ref;
    if (ref == 0) return;
    const tb_account_t& a = T.acc_rows[ref - 1];
    e->id_lo = a.id.lo;
    e->meta = acc_meta(uint16_t(a.flags & ~TB_ACCOUNT_CLOSED), acc_hazard_of(a), a.ledger);
    T.acc_entry_of[ref - 1] = uint32_t(pos);
}

__global__ void acc_index_repair(Tables T, IndexBuild B) {
    const uint64_t stride = uint64_t(gridDim.x) * blockDim.x;
    const uint64_t i0 = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (B.counters[1]) {  // the dirty list overflowed: every entry
        for (uint64_t p = i0; p <= T.acc_index.mask; p += stride) acc_index_repair_entry(T, p);
        return;
    }
    const uint64_t n = B.counters[0] < B.dirty_cap ? B.counters[0] : B.dirty_cap;
    for (uint64_t i = i0; i < n; i += stride) acc_index_repair_entry(T, B.dirty[i]);
}

// ================================ pulse ======================================================

// kPulseCollectItems expires_at entries per lane (independent loads in flight): drop entries that
// left the index (posted / voided / expired / rolled back), collect the expired ones, and find the
// earliest unexpired expiry. One atomic per workgroup for each list (a counter taken once per wave
// serialised ~5k appends at the L2 for a 300k-entry index).
constexpr uint32_t kPulseCollectThreads = 256, kPulseCollectItems = 4;
constexpr uint32_t kPulseCollectTile = kPulseCollectThreads * kPulseCollectItems;

__global__ void __launch_bounds__(kPulseCollectThreads) pulse_collect(
    Tables T, uint64_t timestamp, uint64_t count, uint64_t* keep, unsigned long long* keep_count,
    uint64_t* cand_expires, uint64_t* cand_ts, uint64_t* cand_row, unsigned long long* cand_count,
    unsigned long long* next_unexpired, unsigned long long* cand_min) {
    constexpr uint32_t kWaves = kPulseCollectThreads / 64;
    __shared__ uint32_t s_keep[kWaves], s_cand[kWaves];
    __shared__ unsigned long long s_base[2], s_next[kWaves], s_min[kWaves];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint64_t base = uint64_t(blockIdx.x) * kPulseCollectTile;
    uint64_t row[kPulseCollectItems], exp[kPulseCollectItems], ts[kPulseCollectItems];
    bool kept[kPulseCollectItems], cand[kPulseCollectItems];
    uint32_t nk = 0, nc = 0;
    uint64_t next = ~0ull, first = ~0ull;
    // (an entry's row fields are loaded with its live / status bytes, not after them: two rounds
    // of dependent loads, not three -- a dropped entry's row is read for nothing)
    uint32_t tmo[kPulseCollectItems];
#pragma unroll
    for (uint32_t j = 0; j < kPulseCollectItems; j++) {
        const uint64_t i = base + j * kPulseCollectThreads + tid;
        row[j] = i < count ? T.expiry[i] : 0;
    }
#pragma unroll
    for (uint32_t j = 0; j < kPulseCollectItems; j++) {
        const uint64_t i = base + j * kPulseCollectThreads + tid;
        kept[j] = i < count && T.tr_live[row[j]] && T.tr_status[row[j]] == TB_PENDING_PENDING;
        ts[j] = i < count ? T.tr_rows[row[j]].timestamp : 0;
        tmo[j] = i < count ? T.tr_rows[row[j]].timeout : 0;
    }
#pragma unroll
    for (uint32_t j = 0; j < kPulseCollectItems; j++) {
        exp[j] = ~0ull;
        cand[j] = false;
        if (!kept[j]) ts[j] = 0;
        if (kept[j]) {
            exp[j] = ts[j] + (uint64_t)tmo[j] * TB_NS_PER_S;
            cand[j] = exp[j] <= timestamp;
            if (!cand[j]) next = exp[j] < next ? exp[j] : next;
            else first = exp[j] < first ? exp[j] : first;
        }
        nk += kept[j];
        nc += cand[j];
    }
    const uint32_t ik = wave_inclusive_u32(nk, lane), ic = wave_inclusive_u32(nc, lane);
    for (int off = 32; off > 0; off >>= 1) {
        const uint64_t o = __shfl_xor(next, off), f = __shfl_xor(first, off);
        next = o < next ? o : next;
        first = f < first ? f : first;
    }
    if (lane == 63) {
        s_keep[wv] = ik;
        s_cand[wv] = ic;
    }
    if (lane == 0) {
        s_next[wv] = next;
        s_min[wv] = first;
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t tk = 0, tc = 0;
        uint64_t tn = ~0ull, tf = ~0ull;
        for (uint32_t w = 0; w < kWaves; w++) {
            tk += s_keep[w];
            tc += s_cand[w];
            tn = s_next[w] < tn ? s_next[w] : tn;
            tf = s_min[w] < tf ? s_min[w] : tf;
        }
        if (tf != ~0ull) atomicMin(cand_min, (unsigned long long)tf);
        s_base[0] = tk ? atomicAdd(keep_count, (unsigned long long)tk) : 0;
        s_base[1] = tc ? atomicAdd(cand_count, (unsigned long long)tc) : 0;
        if (tn != ~0ull) atomicMin(next_unexpired, (unsigned long long)tn);
    }
    __syncthreads();
    uint64_t pk = s_base[0] + ik - nk, pc = s_base[1] + ic - nc;
    for (uint32_t w = 0; w < wv; w++) {
        pk += s_keep[w];
        pc += s_cand[w];
    }
#pragma unroll
    for (uint32_t j = 0; j < kPulseCollectItems; j++) {
        if (kept[j]) keep[pk++] = row[j];
        if (cand[j]) {
            cand_expires[pc] = exp[j];
            cand_ts[pc] = ts[j];
            cand_row[pc] = row[j];
            pc++;
        }
    }
}

// The timestamps of the first n sorted candidates (their index keys' second half).
__global__ void pulse_key_timestamps(Tables T, const uint64_t* rows, uint64_t n, uint64_t* ts) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) ts[i] = T.tr_rows[rows[i]].timestamp;
}

// execute_expire_pending_transfers (:4540-4626) for the selected rows.
// (n_dev: the count on device, n its upper bound)
__device__ inline void pulse_apply_one(Tables T, uint64_t row) {
    const tb_transfer_t& p = T.tr_rows[row];
    const uint64_t dr_row = account_find(T, p.debit_account_id);
    const uint64_t cr_row = account_find(T, p.credit_account_id);
    if (dr_row == kNone || cr_row == kNone) return;
    tb_account_t* dr = &T.acc_rows[dr_row];
    tb_account_t* cr = &T.acc_rows[cr_row];
    // (atomic_sub_u128 on both sides, the two low-word adds in flight together, borrows after)
    const u128 amount = U(p.amount);
    const uint64_t lo = uint64_t(amount), hi = uint64_t(amount >> 64);
    unsigned long long* d = reinterpret_cast<unsigned long long*>(&dr->debits_pending);
    unsigned long long* cw = reinterpret_cast<unsigned long long*>(&cr->credits_pending);
    uint64_t od = 0, oc = 0;
    if (lo) {
        od = atomicAdd(d, 0ull - lo);
        oc = atomicAdd(cw, 0ull - lo);
    }
    const uint64_t hd = hi + (lo && od < lo ? 1u : 0u), hc = hi + (lo && oc < lo ? 1u : 0u);
    if (hd) atomicAdd(d + 1, 0ull - hd);
    if (hc) atomicAdd(cw + 1, 0ull - hc);
    if (p.flags & TB_TRANSFER_CLOSING_DEBIT)
        atomicAnd(account_code_flags_word(dr), ~(uint32_t(TB_ACCOUNT_CLOSED) << 16));
    if (p.flags & TB_TRANSFER_CLOSING_CREDIT)
        atomicAnd(account_code_flags_word(cr), ~(uint32_t(TB_ACCOUNT_CLOSED) << 16));
    T.tr_status[row] = TB_PENDING_EXPIRED;
}

__global__ void pulse_apply(Tables T, const uint64_t* rows, uint64_t n, const unsigned int* n_dev) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n || (n_dev && i >= *n_dev)) return;
    pulse_apply_one(T, rows[i]);
}

// ================================ lookups, dumps, indexes ===================================

__global__ void lookup_accounts_kernel(Tables T, const tb_uint128_t* ids, uint32_t n,
                                       uint64_t* rows, uint8_t* found) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t r = account_find(T, ids[i]);
    found[i] = r != kNone;
    rows[i] = r;
}

__global__ void lookup_transfers_kernel(Tables T, const tb_uint128_t* ids, uint32_t n,
                                        uint64_t* rows, uint8_t* found) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const tb_transfer_t* trs = T.tr_rows;
    const uint64_t s = probe_find(T.tr, ids[i], [&](uint64_t r) { return trs[r].id; });
    uint64_t r = kNone;
    if (s != kNone) {
        const uint64_t w = T.tr.slots[s];
        if (!(w & kOrphanBit)) r = (w & kRefMask) - 1;
    }
    found[i] = r != kNone;
    rows[i] = r;
}

// Orphaned ids back to unknown (a tombstone): a sharded call's probe of a linked chain across
// shards executed an event the reference never reaches (tigerbeetle_amd/shard.py).
__global__ void forget_orphans_kernel(Tables T, const tb_uint128_t* ids, uint32_t n,
                                      unsigned int* forgotten) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const tb_transfer_t* trs = T.tr_rows;
    const uint64_t s = probe_find(T.tr, ids[i], [&](uint64_t r) { return trs[r].id; });
    if (s == kNone) return;
    const uint64_t w = T.tr.slots[s];
    if (w == kTomb || !(w & kOrphanBit)) return;
    T.tr.slots[s] = kTomb;
    atomicAdd(forgotten, 1u);
}

// Whether a live object of a groove has each timestamp (its sorted timestamp index).
__global__ void timestamps_exist_kernel(const uint64_t* index, uint64_t count, const uint64_t* ts,
                                        uint32_t n, uint8_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    out[i] = ts_index_contains(index, count, ts[i]) ? 1 : 0;
}

template <typename Row>
__global__ void gather_rows(const Row* src, const uint64_t* rows, const uint32_t* sel, uint32_t n,
                            Row* dst) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dst[i] = src[rows ? rows[sel[i]] : sel[i]];
}

template <typename Row>
__global__ void gather_timestamps(const Row* src, const uint32_t* sel, uint64_t n, uint64_t* dst) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dst[i] = src[sel[i]].timestamp;
}

__global__ void gather_status(const uint8_t* src, const uint32_t* sel, uint64_t n, uint8_t* dst) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    dst[i] = src[sel[i]];
}

__global__ void set_balances_kernel(Tables T, tb_uint128_t id, tb_uint128_t dp, tb_uint128_t dpo,
                                    tb_uint128_t cp, tb_uint128_t cpo, int* rc) {
    const uint64_t r = account_find(T, id);
    if (r == kNone) {
        *rc = -1;
        return;
    }
    tb_account_t* a = &T.acc_rows[r];
    a->debits_pending = dp;
    a->debits_posted = dpo;
    a->credits_pending = cp;
    a->credits_posted = cpo;
    const uint16_t h = acc_hazard_of(*a);
    if (h) acc_hazard_set(T.acc_index, T.acc_entry_of, r, h);
    *rc = 0;
}

}  // namespace tbg
