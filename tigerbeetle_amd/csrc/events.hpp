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
// accounts; the (account, event) touches are radix-sorted by account with events in descending
// order, and an exclusive scan by key gives every touch the sum of its account's later deltas.
// Chains that were rolled back left no created event, so their events never appear (the groove's
// scope discard). AccountEvents are in timestamp order within a call; the log is kept sorted.
#pragma once

#include "kernels.hpp"

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

// The running sums scanned per account (the four balances and the closed flips).
struct Bal5 {
    u128 dp, dpo, cp, cpo;
    uint32_t flips, pad0;
    uint64_t pad1;
};
struct Bal5Add {
    __device__ Bal5 operator()(const Bal5& a, const Bal5& b) const {
        Bal5 r;
        r.dp = a.dp + b.dp;
        r.dpo = a.dpo + b.dpo;
        r.cp = a.cp + b.cp;
        r.cpo = a.cpo + b.cpo;
        r.flips = a.flips + b.flips;
        r.pad0 = 0;
        r.pad1 = 0;
        return r;
    }
};

struct AeScratch {
    uint64_t* keys;         // per touch: account row << 32 | ~event
    uint32_t* vals;         // per touch: 2 * event + side
    uint64_t* keys_sorted;
    uint32_t* vals_sorted;
    AeDelta* deltas;        // per touch (by 2 * event + side)
    uint32_t* seg;          // per sorted touch: account row
    Bal5* values;           // per sorted touch: its deltas placed in the four fields
    Bal5* scanned;          // exclusive sums by account (the account's later events)
};

__device__ inline void ae_side(const AeScratch& S, uint32_t i, uint32_t side, uint32_t row,
                               u128 pending, u128 posted, uint32_t flip) {
    const uint32_t v = 2 * i + side;
    S.keys[v] = (uint64_t(row) << 32) | (0xFFFFFFFFu - i);
    S.vals[v] = v;
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

__device__ inline uint64_t ae_transfer_row(const Tables& T, const tb_uint128_t& id) {
    const tb_transfer_t* rows = T.tr_rows;
    const uint64_t s = probe_find(T.tr, id, [=](uint64_t r) { return rows[r].id; });
    if (s == kNone) return kNone;
    const uint64_t w = T.tr.slots[s];
    return (w & kOrphanBit) ? kNone : (w & kRefMask) - 1;
}

// Created events of a create_transfers call: list[i] = event index k (call order).
__global__ void ae_created_flags(Call<tb_transfer_t> c, uint8_t* flags) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k < c.n) flags[k] = c.results[k].status == TB_STATUS_CREATED;
}

__global__ void ae_collect_transfers(Tables T, Call<tb_transfer_t> c, const uint32_t* list,
                                     uint32_t m, AeScratch S, tb_account_event_t* log,
                                     AeRef* refs) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint32_t k = list[i];
    const uint64_t row = c.row_base + k;
    const tb_transfer_t& t = T.tr_rows[row];  // the created transfer (amount actual, accounts)
    const uint16_t f = t.flags;
    const uint64_t dr = account_find(T, t.debit_account_id);
    const uint64_t cr = account_find(T, t.credit_account_id);
    const u128 amount = U(t.amount);
    uint8_t status = TB_PENDING_NONE;
    const tb_transfer_t* p = nullptr;
    u128 d_pending = 0, d_posted = 0;
    uint32_t flip_dr = 0, flip_cr = 0;
    if (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) {
        const uint64_t pr = ae_transfer_row(T, t.pending_id);
        p = &T.tr_rows[pr];
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
    ae_side(S, i, 0, uint32_t(dr), d_pending, d_posted, flip_dr);
    ae_side(S, i, 1, uint32_t(cr), d_pending, d_posted, flip_cr);
    ae_event_fields(&log[i], t.timestamp, f, status, p, c.events[k].amount, t.amount, t.ledger);
    refs[i] = AeRef{uint32_t(row), uint32_t(dr), uint32_t(cr), 0};
}

// Expiries of a pulse (execute_expire_pending_transfers :4540-4626): rows[i] in expiry order,
// event i stamped timestamp - m + i + 1.
__global__ void ae_collect_expiry(Tables T, const uint64_t* rows, uint32_t m, uint64_t timestamp,
                                  AeScratch S, tb_account_event_t* log, AeRef* refs) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const uint64_t row = rows[i];
    const tb_transfer_t& p = T.tr_rows[row];
    const uint64_t dr = account_find(T, p.debit_account_id);
    const uint64_t cr = account_find(T, p.credit_account_id);
    const u128 d_pending = u128(0) - U(p.amount);
    ae_side(S, i, 0, uint32_t(dr), d_pending, 0, (p.flags & TB_TRANSFER_CLOSING_DEBIT) != 0);
    ae_side(S, i, 1, uint32_t(cr), d_pending, 0, (p.flags & TB_TRANSFER_CLOSING_CREDIT) != 0);
    ae_event_fields(&log[i], timestamp - m + i + 1, 0, TB_PENDING_EXPIRED, &p,
                    tb_uint128_t{0, 0}, p.amount, p.ledger);
    refs[i] = AeRef{uint32_t(row), uint32_t(dr), uint32_t(cr), 0};
}

// Sorted touches -> their account (the scan key) and their deltas in the four fields.
__global__ void ae_values(AeScratch S, uint32_t touches) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= touches) return;
    const AeDelta d = S.deltas[S.vals_sorted[j]];
    Bal5 b;
    b.dp = d.side == 0 ? d.pending : 0;
    b.dpo = d.side == 0 ? d.posted : 0;
    b.cp = d.side == 1 ? d.pending : 0;
    b.cpo = d.side == 1 ? d.posted : 0;
    b.flips = d.flip;
    b.pad0 = 0;
    b.pad1 = 0;
    S.values[j] = b;
    S.seg[j] = uint32_t(S.keys_sorted[j] >> 32);
}

// One sorted touch: its account after the event = final row - the later events' sums.
__global__ void ae_emit(Tables T, AeScratch S, uint32_t touches, tb_account_event_t* log) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= touches) return;
    const uint32_t v = S.vals_sorted[j];
    const uint32_t i = v >> 1, side = v & 1;
    const tb_account_t& a = T.acc_rows[S.seg[j]];
    const Bal5 later = S.scanned[j];
    tb_account_event_t* e = &log[i];
    const tb_uint128_t dp = W(U(a.debits_pending) - later.dp);
    const tb_uint128_t dpo = W(U(a.debits_posted) - later.dpo);
    const tb_uint128_t cp = W(U(a.credits_pending) - later.cp);
    const tb_uint128_t cpo = W(U(a.credits_posted) - later.cpo);
    const uint16_t flags = uint16_t(a.flags ^ ((later.flips & 1) ? TB_ACCOUNT_CLOSED : 0));
    if (side == 0) {
        e->dr_account_id = a.id;
        e->dr_debits_pending = dp;
        e->dr_debits_posted = dpo;
        e->dr_credits_pending = cp;
        e->dr_credits_posted = cpo;
        e->dr_account_timestamp = a.timestamp;
        e->dr_account_flags = flags;
    } else {
        e->cr_account_id = a.id;
        e->cr_debits_pending = dp;
        e->cr_debits_posted = dpo;
        e->cr_credits_pending = cp;
        e->cr_credits_posted = cpo;
        e->cr_account_timestamp = a.timestamp;
        e->cr_account_flags = flags;
    }
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

// Log order repair (imported transfers may postdate... precede earlier expiries): the log sorted by
// timestamp, stable.
__global__ void ae_sort_keys(const tb_account_event_t* log, uint64_t n, uint64_t* keys,
                             uint32_t* idx) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    keys[i] = log[i].timestamp;
    idx[i] = uint32_t(i);
}
__global__ void ae_permute(const tb_account_event_t* log, const AeRef* refs, const uint32_t* idx,
                           uint64_t n, tb_account_event_t* log_out, AeRef* refs_out) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    log_out[i] = log[idx[i]];
    refs_out[i] = refs[idx[i]];
}

}  // namespace tbg
