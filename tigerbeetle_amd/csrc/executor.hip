// The MI355X batch executor (include/tbg.h): kernels and host API.
//
// A create_transfers call of N events runs as a fixed sequence of stream-ordered launches:
//
//   tr_prepare   one lane per event: batch index, claim of the event's id in the transfer id
//                table (earliest duplicate wins), debit/credit account rows (hash probes)
//   tr_mark      accounts whose `closed` flag may change in this call (closing transfers and
//                voids of pending transfers)
//   tr_classify  the reference's check sequence (state_machine.zig:3029-3104, :3719-3873) up to
//                the first check that depends on in-call state. Events whose outcome is fixed
//                get their result here; events whose outcome is order-dependent are routed to
//                the ordered replay and mark their accounts `hot`; the rest are `fast`
//   tr_fast      fast events touching a hot account join the replay (their balance effect must be
//                ordered); all others commit in parallel: transfer row, result, u128 balance
//                atomics, TransferPending status, expires_at entry, pulse_next_timestamp min
//   select       order-preserving compaction of the replay list (hipcub)
//   tr_replay    one lane executes the replay list in serial order (replay.hpp)
//   tr_finalize  id slots: created -> object, transient failure -> orphan, otherwise tombstone
//
// Exactness argument: a fast event reads only state no other event of the call
// writes (ids unique in the call and absent before, static account flags/ledgers, `closed` of
// accounts no event may close or reopen, no limit flags on the checked side, no balancing, and
// balances/amount below 2^126 / 2^64 so no sum can overflow); its effects on balances are
// commutative additions. Every event that reads state another in-call event writes executes in
// the serial order in the replay, which sees the parallel effects on the accounts it reads
// because any fast event touching those accounts was moved into the replay.

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/tbg.h"
#include "device_common.hpp"
#include "replay.hpp"

using namespace tbg;

namespace {

constexpr int kBlock = 256;

inline uint32_t grid_for(uint64_t n) { return uint32_t((n + kBlock - 1) / kBlock); }

__device__ inline void count_stat(DevScalars* s, int which, bool pred) {
    unsigned long long mask = __ballot(pred);
    if ((threadIdx.x & 63) == 0 && mask) atomicAdd(&s->stats[which], (unsigned long long)__popcll(mask));
}

__device__ inline void set_flag_any(DevScalars* s, bool pred, unsigned int flag) {
    if (__any(pred) && (threadIdx.x & 63) == 0) atomicOr(&s->flags, flag);
}

template <typename Event>
__device__ inline uint64_t ts_event_of(const Call<Event>& c, uint32_t b, uint32_t k) {
    return c.batch_ts[b] - c.batch_ends[b] + k + 1;
}

template <typename Event>
__device__ inline uint32_t batch_start_of(const Call<Event>& c, uint32_t b) {
    return b == 0 ? 0 : c.batch_ends[b - 1];
}

// ================================ create_transfers ==========================================

__global__ void tr_prepare(Tables T, Call<tb_transfer_t> c) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = k < c.n;
    bool imported = false, post_void = false;
    if (active) {
        const tb_transfer_t* ev = c.events;
        const tb_transfer_t& t = ev[k];
        const uint16_t flags = t.flags;
        imported = (flags & TB_TRANSFER_IMPORTED) != 0;
        post_void = (flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) != 0;
        c.ev_batch[k] = batch_of(c.batch_ends, c.n_batches, k);
        const tb_uint128_t id = t.id;
        uint64_t slot = kNone;
        if (!u128_is_zero(id) && !u128_is_max(id)) {
            const tb_transfer_t* rows = T.tr_rows;
            const uint64_t base = c.row_base;
            slot = probe_claim(T.tr, id, base + k + 1, base, [&](uint64_t r) {
                return r >= base ? ev[r - base].id : rows[r].id;
            });
            if (slot == kNone) atomicOr(&T.scalars->flags, kFlagTableFull);
        }
        c.ev_slot[k] = slot;
        const tb_uint128_t dr = t.debit_account_id, cr = t.credit_account_id;
        c.ev_dr[k] = (!u128_is_zero(dr) && !u128_is_max(dr)) ? account_find(T, dr) : kNone;
        c.ev_cr[k] = (!u128_is_zero(cr) && !u128_is_max(cr)) ? account_find(T, cr) : kNone;
    }
    set_flag_any(T.scalars, imported, kFlagImported);
    set_flag_any(T.scalars, post_void, kFlagPostVoid);
}

__global__ void tr_mark(Tables T, Call<tb_transfer_t> c) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= c.n) return;
    const tb_transfer_t& t = c.events[k];
    const uint16_t flags = t.flags;
    if ((flags & TB_TRANSFER_CLOSING_DEBIT) && c.ev_dr[k] != kNone)
        T.acc_closable[c.ev_dr[k]] = c.epoch;
    if ((flags & TB_TRANSFER_CLOSING_CREDIT) && c.ev_cr[k] != kNone)
        T.acc_closable[c.ev_cr[k]] = c.epoch;
    uint64_t p_slot = kNone;
    if ((flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) &&
        !u128_is_zero(t.pending_id) && !u128_is_max(t.pending_id)) {
        p_slot = transfer_slot_find(T, c, t.pending_id);
        if (p_slot != kNone && (flags & TB_TRANSFER_VOID_PENDING)) {
            uint64_t r = (T.tr.slots[p_slot] & kRefMask) - 1;
            const tb_transfer_t& p = r >= c.row_base ? c.events[r - c.row_base] : T.tr_rows[r];
            uint64_t pd = account_find(T, p.debit_account_id);
            uint64_t pc = account_find(T, p.credit_account_id);
            if (pd != kNone) T.acc_closable[pd] = c.epoch;
            if (pc != kNone) T.acc_closable[pc] = c.epoch;
        }
    }
    c.ev_p_slot[k] = p_slot;
}

// Returns a final status, or kClassFast / kClassSlow (encoded as 0 / 1 since no status is 0/1?).
// Statuses are never 0 (deprecated_ok) here, so 0 = fast and 1 is linked_event_failed... use a
// separate out-parameter instead.
__device__ inline uint8_t classify_transfer(const Tables& T, const Call<tb_transfer_t>& c,
                                            uint32_t k, uint32_t b, uint64_t ts_event,
                                            const tb_transfer_t& t, uint32_t* status,
                                            uint64_t* ts_out) {
    const uint16_t f = t.flags;
    const uint32_t bstart = batch_start_of(c, b);
    const bool linked = f & TB_TRANSFER_LINKED;
    if (linked || (k > bstart && (c.events[k - 1].flags & TB_TRANSFER_LINKED))) return kClassSlow;
    // Not in a chain. (Imported calls are routed to the replay before this function.)
    const bool batch_imported = (c.events[bstart].flags & TB_TRANSFER_IMPORTED) != 0;
    const bool imported = (f & TB_TRANSFER_IMPORTED) != 0;
    if (batch_imported != imported) {
        *status = imported ? TB_CT_IMPORTED_EVENT_NOT_EXPECTED : TB_CT_IMPORTED_EVENT_EXPECTED;
        return kClassDone;
    }
    if (!imported && t.timestamp != 0) {
        *status = TB_CT_TIMESTAMP_MUST_BE_ZERO;
        return kClassDone;
    }
    if (f & TB_TRANSFER_PADDING_MASK) { *status = TB_CT_RESERVED_FLAG; return kClassDone; }
    if (u128_is_zero(t.id)) { *status = TB_CT_ID_MUST_NOT_BE_ZERO; return kClassDone; }
    if (u128_is_max(t.id)) { *status = TB_CT_ID_MUST_NOT_BE_INT_MAX; return kClassDone; }

    // Id lookup.
    const uint64_t s = c.ev_slot[k];
    if (s == kNone) return kClassSlow;  // table full: flagged, the call fails
    const uint64_t w = T.tr.slots[s];
    const uint64_t r = (w & kRefMask) - 1;
    if (r < c.row_base) {
        if (w & kOrphanBit) { *status = TB_CT_ID_ALREADY_FAILED; return kClassDone; }
        const tb_transfer_t e = T.tr_rows[r];
        const tb_transfer_t* p = nullptr;
        tb_transfer_t p_copy;
        if (t.flags == e.flags && U(t.pending_id) == U(e.pending_id) && t.timeout == e.timeout &&
            (t.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING))) {
            const uint64_t ps = c.ev_p_slot[k];
            if (ps == kNone) return kClassSlow;
            const uint64_t pw = T.tr.slots[ps];
            const uint64_t pr = (pw & kRefMask) - 1;
            if (pr >= c.row_base || (pw & kOrphanBit)) return kClassSlow;
            p_copy = T.tr_rows[pr];
            p = &p_copy;
        }
        *status = create_transfer_exists(t, e, p, ts_out);
        return kClassDone;
    }
    if (r != c.row_base + k) return kClassSlow;  // a later duplicate of an in-call id

    if (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) return kClassSlow;
    uint32_t st = 0;
    if (u128_is_zero(t.debit_account_id)) st = TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    else if (u128_is_max(t.debit_account_id)) st = TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    else if (u128_is_zero(t.credit_account_id)) st = TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    else if (u128_is_max(t.credit_account_id)) st = TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    else if (u128_eq(t.credit_account_id, t.debit_account_id)) st = TB_CT_ACCOUNTS_MUST_BE_DIFFERENT;
    else if (!u128_is_zero(t.pending_id)) st = TB_CT_PENDING_ID_MUST_BE_ZERO;
    else if (!(f & TB_TRANSFER_PENDING) && t.timeout != 0)
        st = TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
    else if (!(f & TB_TRANSFER_PENDING) && (f & (TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT)))
        st = TB_CT_CLOSING_TRANSFER_MUST_BE_PENDING;
    else if (t.ledger == 0) st = TB_CT_LEDGER_MUST_NOT_BE_ZERO;
    else if (t.code == 0) st = TB_CT_CODE_MUST_NOT_BE_ZERO;
    if (st) { *status = st; return kClassDone; }

    const uint64_t dr_row = c.ev_dr[k], cr_row = c.ev_cr[k];
    if (dr_row == kNone) { *status = TB_CT_DEBIT_ACCOUNT_NOT_FOUND; return kClassDone; }
    if (cr_row == kNone) { *status = TB_CT_CREDIT_ACCOUNT_NOT_FOUND; return kClassDone; }
    const tb_account_t& dr = T.acc_rows[dr_row];
    const tb_account_t& cr = T.acc_rows[cr_row];
    const uint32_t dr_ledger = dr.ledger, cr_ledger = cr.ledger;
    if (dr_ledger != cr_ledger) { *status = TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER; return kClassDone; }
    if (t.ledger != dr_ledger) {
        *status = TB_CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;
        return kClassDone;
    }
    if (T.acc_closable[dr_row] == c.epoch || T.acc_closable[cr_row] == c.epoch) return kClassSlow;
    const uint16_t dr_flags = dr.flags, cr_flags = cr.flags;
    if (dr_flags & TB_ACCOUNT_CLOSED) { *status = TB_CT_DEBIT_ACCOUNT_ALREADY_CLOSED; return kClassDone; }
    if (cr_flags & TB_ACCOUNT_CLOSED) { *status = TB_CT_CREDIT_ACCOUNT_ALREADY_CLOSED; return kClassDone; }
    if (f & (TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT |
             TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT))
        return kClassSlow;
    // Overflow is impossible when every balance is < 2^126 and every amount < 2^64.
    constexpr uint64_t kHiLimit = 1ull << 62;
    if (t.amount.hi != 0 || dr.debits_pending.hi >= kHiLimit || dr.debits_posted.hi >= kHiLimit ||
        cr.credits_pending.hi >= kHiLimit || cr.credits_posted.hi >= kHiLimit)
        return kClassSlow;
    if (ts_event + (uint64_t)t.timeout * TB_NS_PER_S > TB_TIMESTAMP_MAX) {
        *status = TB_CT_OVERFLOWS_TIMEOUT;
        return kClassDone;
    }
    if (dr_flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) return kClassSlow;
    if (cr_flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) return kClassSlow;
    // pulse_next_timestamp is reset by post/void when it equals an expiry: keep its order exact.
    if ((f & TB_TRANSFER_PENDING) && t.timeout > 0 && (T.scalars->flags & kFlagPostVoid))
        return kClassSlow;
    return kClassFast;
}

__global__ void tr_classify(Tables T, Call<tb_transfer_t> c, uint8_t* ev_slow) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    uint8_t cls = kClassDone;
    if (k < c.n) {
        const uint32_t b = c.ev_batch[k];
        const uint64_t ts_event = ts_event_of(c, b, k);
        const tb_transfer_t t = c.events[k];
        uint32_t status = 0;
        uint64_t ts = ts_event;
        if (c.force_replay || (T.scalars->flags & kFlagImported)) {
            cls = kClassSlow;
        } else {
            cls = classify_transfer(T, c, k, b, ts_event, t, &status, &ts);
        }
        if (cls == kClassDone) {
            tb_create_result_t res;
            res.timestamp = status == TB_CT_EXISTS ? ts : ts_event;
            res.status = status;
            res.reserved = 0;
            c.results[k] = res;
        } else if (cls == kClassSlow) {
            // Mark the accounts whose balances/flags this event may read or write in order.
            if (c.ev_dr[k] != kNone) T.acc_hot[c.ev_dr[k]] = c.epoch;
            if (c.ev_cr[k] != kNone) T.acc_hot[c.ev_cr[k]] = c.epoch;
            const uint64_t ps = c.ev_p_slot[k];
            if (ps != kNone) {
                const uint64_t w = T.tr.slots[ps];
                const uint64_t r = (w & kRefMask) - 1;
                const tb_transfer_t& p = r >= c.row_base ? c.events[r - c.row_base] : T.tr_rows[r];
                uint64_t pd = account_find(T, p.debit_account_id);
                uint64_t pc = account_find(T, p.credit_account_id);
                if (pd != kNone) T.acc_hot[pd] = c.epoch;
                if (pc != kNone) T.acc_hot[pc] = c.epoch;
            }
        }
        c.ev_class[k] = cls;
        ev_slow[k] = cls == kClassSlow;
    }
    count_stat(T.scalars, 3, k < c.n && cls == kClassDone);
}

__global__ void tr_fast(Tables T, Call<tb_transfer_t> c, uint8_t* ev_slow) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    bool fast = false;
    if (k < c.n && c.ev_class[k] == kClassFast) {
        const uint64_t dr_row = c.ev_dr[k], cr_row = c.ev_cr[k];
        if (T.acc_hot[dr_row] == c.epoch || T.acc_hot[cr_row] == c.epoch) {
            c.ev_class[k] = kClassSlow;
            ev_slow[k] = 1;
        } else {
            fast = true;
            const uint32_t b = c.ev_batch[k];
            const uint64_t ts = ts_event_of(c, b, k);
            const uint64_t row = c.row_base + k;
            tb_transfer_t o = c.events[k];
            o.timestamp = ts;
            T.tr_rows[row] = o;
            const bool pending = (o.flags & TB_TRANSFER_PENDING) != 0;
            T.tr_status[row] = pending ? TB_PENDING_PENDING : TB_PENDING_NONE;
            tb_create_result_t res;
            res.timestamp = ts;
            res.status = TB_STATUS_CREATED;
            res.reserved = 0;
            c.results[k] = res;
            const u128 amount = U(o.amount);
            if (amount != 0) {
                tb_account_t* dr = &T.acc_rows[dr_row];
                tb_account_t* cr = &T.acc_rows[cr_row];
                if (pending) {
                    atomic_add_u128(&dr->debits_pending, amount);
                    atomic_add_u128(&cr->credits_pending, amount);
                } else {
                    atomic_add_u128(&dr->debits_posted, amount);
                    atomic_add_u128(&cr->credits_posted, amount);
                }
            }
            if (pending && o.timeout > 0) {
                expiry_append(T, row, false);
                atomicMin(&T.scalars->pulse_next_timestamp,
                          (unsigned long long)(ts + (uint64_t)o.timeout * TB_NS_PER_S));
            }
        }
    }
    // transfers objects tree key_range: the largest created timestamp (wave-reduced).
    uint64_t ts_max = 0;
    if (fast) ts_max = ts_event_of(c, c.ev_batch[k], k);
    for (int off = 32; off > 0; off >>= 1) {
        uint64_t o = __shfl_xor(ts_max, off);
        ts_max = o > ts_max ? o : ts_max;
    }
    if ((threadIdx.x & 63) == 0 && ts_max) atomicMax(&T.scalars->transfers_key_max, (unsigned long long)ts_max);
    count_stat(T.scalars, 1, fast);
}

template <typename Event>
__device__ inline void replay_chain_step(Replay& R, const Call<Event>& c, uint32_t k,
                                         bool is_transfers, bool& chain_open, uint32_t& chain_start,
                                         bool& chain_broken) {
    const Tables& T = R.T;
    const Event ev = c.events[k];
    const uint32_t b = c.ev_batch[k];
    const uint32_t bstart = batch_start_of(c, b);
    const uint32_t bend = c.batch_ends[b];
    const uint64_t ts_event = ts_event_of(c, b, k);
    const uint16_t linked_flag = is_transfers ? TB_TRANSFER_LINKED : TB_ACCOUNT_LINKED;
    const uint16_t imported_flag = is_transfers ? TB_TRANSFER_IMPORTED : TB_ACCOUNT_IMPORTED;
    const uint16_t f = ev.flags;
    uint32_t status = 0;
    uint64_t ts_actual = ts_event;

    do {
        if (f & linked_flag) {
            if (!chain_open) {
                chain_open = true;
                chain_start = k;
                chain_broken = false;
                R.scope_open();
            }
            if (k == bend - 1) {
                status = TB_CT_LINKED_EVENT_CHAIN_OPEN;
                break;
            }
        }
        if (chain_broken) {
            status = TB_CT_LINKED_EVENT_FAILED;
            break;
        }
        const bool batch_imported = (c.events[bstart].flags & imported_flag) != 0;
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
        if constexpr (sizeof(Event) == sizeof(tb_transfer_t) &&
                      __is_same(Event, tb_transfer_t)) {
            status = replay_create_transfer(R, c, k, ts_event, ev, &ts);
            if (status == TB_STATUS_CREATED || status == TB_CT_EXISTS) ts_actual = ts;
        } else {
            status = replay_create_account(R, c, k, ts_event, ev, &ts);
            if (status == TB_STATUS_CREATED || status == TB_CA_EXISTS) ts_actual = ts;
        }
    } while (0);

    // This event becomes the holder of its id's slot when it created or orphaned the id.
    const bool transient = is_transfers && status != TB_STATUS_CREATED &&
                           tb_transfer_status_transient(status);
    if ((status == TB_STATUS_CREATED || transient) && c.ev_slot[k] != kNone) {
        unsigned long long* slots = is_transfers ? T.tr.slots : T.acc.slots;
        slots[c.ev_slot[k]] = c.row_base + k + 1;
    }
    if (status != TB_STATUS_CREATED && chain_open && !chain_broken) {
        chain_broken = true;
        R.scope_close(true);
        for (uint32_t ci = chain_start; ci < k; ci++) c.results[ci].status = TB_CT_LINKED_EVENT_FAILED;
    }
    tb_create_result_t res;
    res.timestamp = ts_actual;
    res.status = status;
    res.reserved = 0;
    c.results[k] = res;
    if (chain_open && (!(f & linked_flag) || status == TB_CT_LINKED_EVENT_CHAIN_OPEN)) {
        if (!chain_broken) R.scope_close(false);
        chain_open = false;
        chain_broken = false;
    }
}

template <typename Event>
__global__ void replay_kernel(Tables T, Call<Event> c, int is_transfers) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    Replay R(T);
    bool chain_open = false, chain_broken = false;
    uint32_t chain_start = 0;
    const uint32_t n = T.scalars->slow_count;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t k = c.slow_list[i];
        replay_chain_step<Event>(R, c, k, is_transfers != 0, chain_open, chain_start, chain_broken);
        if (R.overflow) {
            atomicOr(&T.scalars->flags, kFlagUndoOverflow);
            break;
        }
    }
    T.scalars->stats[2] = n;
}

template <typename Event>
__global__ void finalize_kernel(Tables T, Call<Event> c, int is_transfers) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= c.n) return;
    const uint64_t row = c.row_base + k;
    const uint32_t status = c.results[k].status;
    const bool created = status == TB_STATUS_CREATED;
    const uint64_t s = c.ev_slot[k];
    unsigned long long* slots = is_transfers ? T.tr.slots : T.acc.slots;
    if (s != kNone) {
        const uint64_t w = slots[s];
        if (w == row + 1) {
            if (created) {
                // keep: the slot now names a committed object
            } else if (is_transfers && tb_transfer_status_transient(status)) {
                // An orphaned id keeps its key in the row store so later probes can match it.
                T.tr_rows[row].id = c.events[k].id;
                slots[s] = (row + 1) | kOrphanBit;
            } else {
                slots[s] = kTomb;
            }
        }
    }
    if (is_transfers) T.tr_live[row] = created;
    else T.acc_live[row] = created;
}

// ================================ create_accounts ===========================================

__global__ void acc_prepare(Tables T, Call<tb_account_t> c) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    bool imported = false;
    if (k < c.n) {
        const tb_account_t* ev = c.events;
        const tb_account_t& a = ev[k];
        imported = (a.flags & TB_ACCOUNT_IMPORTED) != 0;
        c.ev_batch[k] = batch_of(c.batch_ends, c.n_batches, k);
        uint64_t slot = kNone;
        if (!u128_is_zero(a.id) && !u128_is_max(a.id)) {
            const tb_account_t* rows = T.acc_rows;
            const uint64_t base = c.row_base;
            slot = probe_claim(T.acc, a.id, base + k + 1, base, [&](uint64_t r) {
                return r >= base ? ev[r - base].id : rows[r].id;
            });
            if (slot == kNone) atomicOr(&T.scalars->flags, kFlagTableFull);
        }
        c.ev_slot[k] = slot;
    }
    set_flag_any(T.scalars, imported, kFlagImported);
}

__global__ void acc_classify(Tables T, Call<tb_account_t> c, uint8_t* ev_slow) {
    const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    uint8_t cls = kClassDone;
    bool created = false;
    uint64_t ts_created = 0;
    if (k < c.n) {
        const uint32_t b = c.ev_batch[k];
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
            const uint64_t s = c.ev_slot[k];
            const uint64_t w = s == kNone ? kTomb : T.acc.slots[s];
            const uint64_t r = (w & kRefMask) - 1;
            if (s == kNone) {
                cls = kClassSlow;
            } else if (r < c.row_base) {
                const tb_account_t e = T.acc_rows[r];
                status = create_account_exists(a, e, &ts);
            } else if (r != c.row_base + k) {
                cls = kClassSlow;
            } else {
                status = create_account_checks(a);
                if (status == TB_STATUS_CREATED) {
                    T.acc_rows[c.row_base + k] = account_row_of(a, ts_event);
                    created = true;
                    ts_created = ts_event;
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
        c.ev_class[k] = cls;
        ev_slow[k] = cls == kClassSlow;
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

// ================================ pulse ======================================================

struct ExpiryCandidate {
    uint64_t expires_at;
    uint64_t timestamp;
    uint64_t row;
};

// One lane per expires_at entry: drop entries that left the index (posted / voided / expired /
// rolled back), collect the expired ones, and find the earliest unexpired expiry.
__global__ void pulse_collect(Tables T, uint64_t timestamp, uint64_t count, uint64_t* keep,
                              unsigned long long* keep_count, uint64_t* cand_key_hi,
                              uint64_t* cand_key_lo, uint64_t* cand_row,
                              unsigned long long* cand_count, unsigned long long* next_unexpired) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= count) return;
    const uint64_t row = T.expiry[i];
    if (!T.tr_live[row] || T.tr_status[row] != TB_PENDING_PENDING) return;
    const tb_transfer_t& p = T.tr_rows[row];
    const uint64_t expires_at = p.timestamp + (uint64_t)p.timeout * TB_NS_PER_S;
    keep[atomicAdd(keep_count, 1ull)] = row;
    if (expires_at <= timestamp) {
        unsigned long long j = atomicAdd(cand_count, 1ull);
        cand_key_hi[j] = expires_at;
        cand_key_lo[j] = p.timestamp;
        cand_row[j] = row;
    } else {
        atomicMin(next_unexpired, (unsigned long long)expires_at);
    }
}

__global__ void pulse_apply(Tables T, const uint64_t* rows, uint64_t n) {
    const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint64_t row = rows[i];
    const tb_transfer_t& p = T.tr_rows[row];
    const uint64_t dr_row = account_find(T, p.debit_account_id);
    const uint64_t cr_row = account_find(T, p.credit_account_id);
    if (dr_row == kNone || cr_row == kNone) return;
    tb_account_t* dr = &T.acc_rows[dr_row];
    tb_account_t* cr = &T.acc_rows[cr_row];
    const u128 amount = U(p.amount);
    if (amount) {
        atomic_sub_u128(&dr->debits_pending, amount);
        atomic_sub_u128(&cr->credits_pending, amount);
    }
    if (p.flags & TB_TRANSFER_CLOSING_DEBIT)
        atomicAnd(account_code_flags_word(dr), ~(uint32_t(TB_ACCOUNT_CLOSED) << 16));
    if (p.flags & TB_TRANSFER_CLOSING_CREDIT)
        atomicAnd(account_code_flags_word(cr), ~(uint32_t(TB_ACCOUNT_CLOSED) << 16));
    T.tr_status[row] = TB_PENDING_EXPIRED;
}

// ================================ lookups, dumps, indexes ===================================

__global__ void lookup_accounts_kernel(Tables T, const tb_uint128_t* ids, uint32_t n,
                                       uint64_t* rows, uint8_t* found) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t r = account_find(T, ids[i]);
    found[i] = r != kNone;
    rows[i] = r;
}

__global__ void lookup_transfers_kernel(Tables T, const tb_uint128_t* ids, uint32_t n,
                                        uint64_t* rows, uint8_t* found) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const tb_transfer_t* trs = T.tr_rows;
    uint64_t s = probe_find(T.tr, ids[i], [&](uint64_t r) { return trs[r].id; });
    uint64_t r = kNone;
    if (s != kNone) {
        uint64_t w = T.tr.slots[s];
        if (!(w & kOrphanBit)) r = (w & kRefMask) - 1;
    }
    found[i] = r != kNone;
    rows[i] = r;
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
    uint64_t r = account_find(T, id);
    if (r == kNone) {
        *rc = -1;
        return;
    }
    tb_account_t* a = &T.acc_rows[r];
    a->debits_pending = dp;
    a->debits_posted = dpo;
    a->credits_pending = cp;
    a->credits_posted = cpo;
    *rc = 0;
}

uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

}  // namespace

// ================================ host side ==================================================

struct PulseScratch {
    uint64_t capacity = 0;
    uint64_t *keep = nullptr, *exp = nullptr, *ts = nullptr, *rows = nullptr;
    uint64_t *exp_b = nullptr, *rows_b = nullptr;
    unsigned long long* counters = nullptr;
};

struct tbg_ctx {
    tbg_options opt{};
    PulseScratch pulse;
    hipStream_t stream = nullptr;
    std::string error;
    Tables T{};
    DevScalars* d_scalars = nullptr;
    DevScalars* h_scalars = nullptr;  // pinned
    uint32_t epoch = 0;
    bool force_replay = false;
    tbg_stats stats{};

    // per-call scratch
    uint8_t* d_events = nullptr;
    tb_create_result_t* d_results = nullptr;
    uint32_t* d_batch_ends = nullptr;
    uint64_t* d_batch_ts = nullptr;
    uint32_t* ev_batch = nullptr;
    uint64_t* ev_slot = nullptr;
    uint64_t* ev_dr = nullptr;
    uint64_t* ev_cr = nullptr;
    uint64_t* ev_p_slot = nullptr;
    uint8_t* ev_class = nullptr;
    uint8_t* ev_slow = nullptr;
    uint32_t* slow_list = nullptr;
    void* cub_temp = nullptr;
    size_t cub_temp_bytes = 0;

    // imported-timestamp indexes (rebuilt on demand)
    uint64_t* acc_ts_index = nullptr;
    uint64_t* tr_ts_index = nullptr;
    bool acc_ts_stale = true, tr_ts_stale = true;
    uint32_t* sel_buf = nullptr;  // selection output for dumps / indexes (max rows)

    std::vector<uint32_t> h_ends;

    // Per-kernel timing (tbg_profile): HIP events recorded on the call's stream between launches.
    bool timing = false;
    static constexpr int kMaxMarks = 32;
    hipEvent_t marks[kMaxMarks] = {};
    const char* mark_names[kMaxMarks] = {};
    int n_marks = 0;
    std::vector<std::string> prof_names;
    std::vector<double> prof_ms;
    std::vector<uint64_t> prof_count;
};

namespace {

bool hip_ok(tbg_ctx* ctx, hipError_t e, const char* what) {
    if (e == hipSuccess) return true;
    char buf[256];
    snprintf(buf, sizeof(buf), "%s: %s", what, hipGetErrorString(e));
    ctx->error = buf;
    return false;
}

#define HIP_TRY(ctx, expr)                                  \
    do {                                                    \
        if (!hip_ok((ctx), (expr), #expr)) return TBG_EHIP; \
    } while (0)

template <typename T>
bool dev_alloc(tbg_ctx* ctx, T** p, uint64_t count, bool zero) {
    size_t bytes = std::max<size_t>(size_t(count) * sizeof(T), 16);
    if (!hip_ok(ctx, hipMalloc(reinterpret_cast<void**>(p), bytes), "hipMalloc")) return false;
    if (zero && !hip_ok(ctx, hipMemsetAsync(*p, 0, bytes, ctx->stream), "hipMemset")) return false;
    return true;
}

// Order-preserving selection of indices [0, n) whose flag is nonzero.
int select_flagged(tbg_ctx* ctx, const uint8_t* flags, uint64_t n, uint32_t* out,
                   unsigned int* d_count) {
    hipcub::CountingInputIterator<uint32_t> it(0);
    size_t bytes = 0;
    HIP_TRY(ctx, hipcub::DeviceSelect::Flagged(nullptr, bytes, it, flags, out, d_count, int(n),
                                               ctx->stream));
    if (bytes > ctx->cub_temp_bytes) {
        if (ctx->cub_temp) (void)hipFree(ctx->cub_temp);
        ctx->cub_temp = nullptr;
        HIP_TRY(ctx, hipMalloc(&ctx->cub_temp, bytes));
        ctx->cub_temp_bytes = bytes;
    }
    HIP_TRY(ctx, hipcub::DeviceSelect::Flagged(ctx->cub_temp, bytes, it, flags, out, d_count,
                                               int(n), ctx->stream));
    return 0;
}

int sync_scalars(tbg_ctx* ctx) {
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_scalars, ctx->d_scalars, sizeof(DevScalars),
                                hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

// Sorted timestamps of live rows (creation order is timestamp order for each groove).
template <typename Row>
int rebuild_ts_index(tbg_ctx* ctx, const Row* rows, const uint8_t* live, uint64_t used,
                     uint64_t* index, uint64_t* count) {
    if (used == 0) {
        *count = 0;
        return 0;
    }
    unsigned int* d_count = &ctx->d_scalars->slow_count;  // scratch word (not in a call)
    int rc = select_flagged(ctx, live, used, ctx->sel_buf, d_count);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->h_scalars->slow_count, d_count, 4, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *count = ctx->h_scalars->slow_count;
    if (*count)
        hipLaunchKernelGGL(gather_timestamps<Row>, dim3(grid_for(*count)), dim3(kBlock), 0,
                           ctx->stream, rows, ctx->sel_buf, *count, index);
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

template <typename Event>
Call<Event> make_call(tbg_ctx* ctx, const Event* d_events, uint32_t n, const uint32_t* d_ends,
                      const uint64_t* d_ts, uint32_t nb, tb_create_result_t* d_results,
                      uint64_t row_base) {
    Call<Event> c;
    c.events = d_events;
    c.n = n;
    c.batch_ends = d_ends;
    c.batch_ts = d_ts;
    c.n_batches = nb;
    c.results = d_results;
    c.row_base = row_base;
    c.epoch = ++ctx->epoch;
    c.force_replay = ctx->force_replay ? 1 : 0;
    c.ev_batch = ctx->ev_batch;
    c.ev_slot = ctx->ev_slot;
    c.ev_dr = ctx->ev_dr;
    c.ev_cr = ctx->ev_cr;
    c.ev_p_slot = ctx->ev_p_slot;
    c.ev_class = ctx->ev_class;
    c.slow_list = ctx->slow_list;
    return c;
}

void tmark(tbg_ctx* ctx, const char* name) {
    if (!ctx->timing || ctx->n_marks >= tbg_ctx::kMaxMarks) return;
    if (!ctx->marks[ctx->n_marks]) (void)hipEventCreate(&ctx->marks[ctx->n_marks]);
    (void)hipEventRecord(ctx->marks[ctx->n_marks], ctx->stream);
    ctx->mark_names[ctx->n_marks++] = name;
}

// After the stream is synchronised: accumulate the time between consecutive marks per name.
void tcollect(tbg_ctx* ctx) {
    if (!ctx->timing) return;
    for (int i = 1; i < ctx->n_marks; i++) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, ctx->marks[i - 1], ctx->marks[i]) != hipSuccess) continue;
        const std::string name = ctx->mark_names[i];
        size_t j = 0;
        while (j < ctx->prof_names.size() && ctx->prof_names[j] != name) j++;
        if (j == ctx->prof_names.size()) {
            ctx->prof_names.push_back(name);
            ctx->prof_ms.push_back(0);
            ctx->prof_count.push_back(0);
        }
        ctx->prof_ms[j] += ms;
        ctx->prof_count[j] += 1;
    }
    ctx->n_marks = 0;
}

int begin_call(tbg_ctx* ctx) {
    // Reset the per-call words of the scalars block: flags, slow_count, stats.
    ctx->n_marks = 0;
    HIP_TRY(ctx, hipMemsetAsync(&ctx->d_scalars->flags, 0,
                                sizeof(DevScalars) - offsetof(DevScalars, flags), ctx->stream));
    tmark(ctx, "begin");
    return 0;
}

int end_call(tbg_ctx* ctx, uint32_t n) {
    int rc = sync_scalars(ctx);
    if (rc) return rc;
    tcollect(ctx);
    const DevScalars& s = *ctx->h_scalars;
    ctx->stats.events = n;
    ctx->stats.fast = s.stats[1];
    ctx->stats.replayed = s.stats[2];
    ctx->stats.static_fail = s.stats[3];
    if (s.flags & kFlagTableFull) {
        ctx->error = "table capacity exceeded";
        return TBG_ENOSPC;
    }
    if (s.flags & kFlagUndoOverflow) {
        ctx->error = "linked chain longer than the undo log";
        return TBG_ENOSPC;
    }
    return 0;
}

// Shared tail of both create_* paths once the call is classified.
template <typename Event>
int run_replay_and_finalize(tbg_ctx* ctx, Call<Event>& c, bool is_transfers) {
    Tables T = ctx->T;
    int rc = select_flagged(ctx, ctx->ev_slow, c.n, ctx->slow_list, &ctx->d_scalars->slow_count);
    if (rc) return rc;
    tmark(ctx, "select_replay_list");
    hipLaunchKernelGGL(replay_kernel<Event>, dim3(1), dim3(64), 0, ctx->stream, T, c,
                       is_transfers ? 1 : 0);
    tmark(ctx, is_transfers ? "tr_replay" : "acc_replay");
    hipLaunchKernelGGL(finalize_kernel<Event>, dim3(grid_for(c.n)), dim3(kBlock), 0, ctx->stream,
                       T, c, is_transfers ? 1 : 0);
    tmark(ctx, is_transfers ? "tr_finalize" : "acc_finalize");
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

int check_imported_indexes(tbg_ctx* ctx, bool is_transfers) {
    // Imported events look up the *other* groove by timestamp (indirect_lookup).
    if (is_transfers && ctx->acc_ts_stale) {
        int rc = rebuild_ts_index(ctx, ctx->T.acc_rows, ctx->T.acc_live, ctx->T.acc_rows_used,
                                  ctx->acc_ts_index, &ctx->T.acc_ts_count);
        if (rc) return rc;
        ctx->acc_ts_stale = false;
    }
    if (!is_transfers && ctx->tr_ts_stale) {
        int rc = rebuild_ts_index(ctx, ctx->T.tr_rows, ctx->T.tr_live, ctx->T.tr_rows_used,
                                  ctx->tr_ts_index, &ctx->T.tr_ts_count);
        if (rc) return rc;
        ctx->tr_ts_stale = false;
    }
    return 0;
}

int ensure_pulse_scratch(tbg_ctx* ctx, uint64_t count) {
    PulseScratch& S = ctx->pulse;
    if (S.counters && count <= S.capacity) return 0;
    for (void* p : {(void*)S.keep, (void*)S.exp, (void*)S.ts, (void*)S.rows, (void*)S.exp_b,
                    (void*)S.rows_b, (void*)S.counters})
        if (p) (void)hipFree(p);
    S = PulseScratch();
    const uint64_t cap = std::max<uint64_t>(count + count / 2, 1024);
    if (!(dev_alloc(ctx, &S.keep, cap, false) && dev_alloc(ctx, &S.exp, cap, false) &&
          dev_alloc(ctx, &S.ts, cap, false) && dev_alloc(ctx, &S.rows, cap, false) &&
          dev_alloc(ctx, &S.exp_b, cap, false) && dev_alloc(ctx, &S.rows_b, cap, false) &&
          dev_alloc(ctx, &S.counters, 3, false)))
        return TBG_ENOMEM;
    S.capacity = cap;
    return 0;
}

template <typename Row>
int64_t dump_impl(tbg_ctx* ctx, const Row* rows, const uint8_t* live, uint64_t used,
                         Row* out, uint8_t* status_out) {
    if (used == 0) return 0;
    unsigned int* d_count = &ctx->d_scalars->slow_count;
    int rc = select_flagged(ctx, live, used, ctx->sel_buf, d_count);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->h_scalars->slow_count, d_count, 4, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t count = ctx->h_scalars->slow_count;
    if (!out || count == 0) return int64_t(count);
    Row* d_out = nullptr;
    if (!dev_alloc(ctx, &d_out, count, false)) return TBG_ENOMEM;
    hipLaunchKernelGGL(gather_rows<Row>, dim3(grid_for(count)), dim3(kBlock), 0, ctx->stream, rows,
                       (const uint64_t*)nullptr, ctx->sel_buf, uint32_t(count), d_out);
    int64_t result = int64_t(count);
    if (!hip_ok(ctx, hipMemcpyAsync(out, d_out, count * sizeof(Row), hipMemcpyDeviceToHost,
                                    ctx->stream), "dump copy"))
        result = TBG_EHIP;
    if (status_out && result >= 0) {
        uint8_t* d_status = nullptr;
        if (!dev_alloc(ctx, &d_status, count, false)) {
            result = TBG_ENOMEM;
        } else {
            hipLaunchKernelGGL(gather_status, dim3(grid_for(count)), dim3(kBlock), 0, ctx->stream,
                               ctx->T.tr_status, ctx->sel_buf, count, d_status);
            if (!hip_ok(ctx, hipMemcpyAsync(status_out, d_status, count, hipMemcpyDeviceToHost,
                                            ctx->stream), "dump status"))
                result = TBG_EHIP;
            (void)hipStreamSynchronize(ctx->stream);
            (void)hipFree(d_status);
        }
    }
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(d_out);
    return result;
}

}  // namespace

extern "C" {

tbg_ctx* tbg_open(const tbg_options* options) {
    if (!options || options->account_capacity == 0 || options->transfer_capacity == 0 ||
        options->batch_events_max == 0 || options->batch_count_max == 0 ||
        options->pulse_batch_max == 0)
        return nullptr;
    tbg_ctx* ctx = new tbg_ctx();
    ctx->opt = *options;
    bool ok = hip_ok(ctx, hipSetDevice(int(options->device)), "hipSetDevice") &&
              hip_ok(ctx, hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking),
                     "hipStreamCreate");
    const uint64_t acc_cap = options->account_capacity, tr_cap = options->transfer_capacity;
    const uint64_t ev_max = options->batch_events_max;
    const uint64_t acc_slots = next_pow2(acc_cap * 2), tr_slots = next_pow2(tr_cap * 2);
    Tables& T = ctx->T;
    ok = ok && dev_alloc(ctx, &T.acc.slots, acc_slots, true) &&
         dev_alloc(ctx, &T.acc_rows, acc_cap, true) && dev_alloc(ctx, &T.acc_live, acc_cap, true) &&
         dev_alloc(ctx, &T.acc_hot, acc_cap, true) && dev_alloc(ctx, &T.acc_closable, acc_cap, true) &&
         dev_alloc(ctx, &T.tr.slots, tr_slots, true) && dev_alloc(ctx, &T.tr_rows, tr_cap, false) &&
         dev_alloc(ctx, &T.tr_live, tr_cap, true) && dev_alloc(ctx, &T.tr_status, tr_cap, true) &&
         dev_alloc(ctx, &T.expiry, tr_cap, false) && dev_alloc(ctx, &ctx->d_scalars, 1, true);
    const uint64_t undo_cap = 3 * std::min<uint64_t>(ev_max, 65536);
    ok = ok && dev_alloc(ctx, &T.undo, undo_cap, false);
    ok = ok && dev_alloc(ctx, &ctx->d_events, ev_max * 128, false) &&
         dev_alloc(ctx, &ctx->d_results, ev_max, false) &&
         dev_alloc(ctx, &ctx->d_batch_ends, options->batch_count_max, false) &&
         dev_alloc(ctx, &ctx->d_batch_ts, options->batch_count_max, false) &&
         dev_alloc(ctx, &ctx->ev_batch, ev_max, false) && dev_alloc(ctx, &ctx->ev_slot, ev_max, false) &&
         dev_alloc(ctx, &ctx->ev_dr, ev_max, false) && dev_alloc(ctx, &ctx->ev_cr, ev_max, false) &&
         dev_alloc(ctx, &ctx->ev_p_slot, ev_max, false) &&
         dev_alloc(ctx, &ctx->ev_class, ev_max, false) && dev_alloc(ctx, &ctx->ev_slow, ev_max, false) &&
         dev_alloc(ctx, &ctx->slow_list, ev_max, false);
    ok = ok && dev_alloc(ctx, &ctx->acc_ts_index, acc_cap, false) &&
         dev_alloc(ctx, &ctx->tr_ts_index, tr_cap, false) &&
         dev_alloc(ctx, &ctx->sel_buf, std::max(acc_cap, tr_cap), false);
    ok = ok && hip_ok(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->h_scalars), sizeof(DevScalars)),
                      "hipHostMalloc");
    if (!ok) {
        fprintf(stderr, "tbg_open: %s\n", ctx->error.c_str());
        tbg_close(ctx);
        return nullptr;
    }
    T.acc.mask = acc_slots - 1;
    T.tr.mask = tr_slots - 1;
    T.expiry_capacity = tr_cap;
    T.undo_capacity = undo_cap;
    T.scalars = ctx->d_scalars;
    T.acc_ts_index = ctx->acc_ts_index;
    T.tr_ts_index = ctx->tr_ts_index;
    DevScalars init{};
    init.pulse_next_timestamp = options->pulse_next_timestamp_init;
    if (!hip_ok(ctx, hipMemcpyAsync(ctx->d_scalars, &init, sizeof(init), hipMemcpyHostToDevice,
                                    ctx->stream), "init") ||
        !hip_ok(ctx, hipStreamSynchronize(ctx->stream), "init sync")) {
        tbg_close(ctx);
        return nullptr;
    }
    return ctx;
}

void tbg_close(tbg_ctx* ctx) {
    if (!ctx) return;
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    void* ptrs[] = {ctx->T.acc.slots, ctx->T.acc_rows, ctx->T.acc_live, ctx->T.acc_hot,
                    ctx->T.acc_closable, ctx->T.tr.slots, ctx->T.tr_rows, ctx->T.tr_live,
                    ctx->T.tr_status, ctx->T.expiry, ctx->d_scalars, ctx->T.undo, ctx->d_events,
                    ctx->d_results, ctx->d_batch_ends, ctx->d_batch_ts, ctx->ev_batch,
                    ctx->ev_slot, ctx->ev_dr, ctx->ev_cr, ctx->ev_p_slot, ctx->ev_class,
                    ctx->ev_slow, ctx->slow_list, ctx->cub_temp, ctx->acc_ts_index,
                    ctx->tr_ts_index, ctx->sel_buf};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (void* p : {(void*)ctx->pulse.keep, (void*)ctx->pulse.exp, (void*)ctx->pulse.ts,
                    (void*)ctx->pulse.rows, (void*)ctx->pulse.exp_b, (void*)ctx->pulse.rows_b,
                    (void*)ctx->pulse.counters})
        if (p) (void)hipFree(p);
    for (hipEvent_t e : ctx->marks)
        if (e) (void)hipEventDestroy(e);
    if (ctx->h_scalars) (void)hipHostFree(ctx->h_scalars);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* tbg_last_error(const tbg_ctx* ctx) { return ctx ? ctx->error.c_str() : "null ctx"; }

int tbg_create_transfers_device(tbg_ctx* ctx, const tb_transfer_t* d_events, uint32_t n,
                                const uint32_t* d_batch_ends, const uint64_t* d_batch_ts,
                                uint32_t n_batches, tb_create_result_t* d_results, void* stream) {
    if (!ctx || n > ctx->opt.batch_events_max || n_batches > ctx->opt.batch_count_max)
        return TBG_EINVAL;
    if (ctx->T.tr_rows_used + n > ctx->opt.transfer_capacity) {
        ctx->error = "transfer capacity exceeded";
        return TBG_ENOSPC;
    }
    if (n == 0) return 0;
    hipStream_t user = static_cast<hipStream_t>(stream);
    hipStream_t saved = ctx->stream;
    if (user) ctx->stream = user;
    int rc = begin_call(ctx);
    Call<tb_transfer_t> c =
        make_call(ctx, d_events, n, d_batch_ends, d_batch_ts, n_batches, d_results, ctx->T.tr_rows_used);
    Tables T = ctx->T;
    const dim3 grid(grid_for(n)), block(kBlock);
    if (!rc) {
        hipLaunchKernelGGL(tr_prepare, grid, block, 0, ctx->stream, T, c);
        tmark(ctx, "tr_prepare");
        hipLaunchKernelGGL(tr_mark, grid, block, 0, ctx->stream, T, c);
        tmark(ctx, "tr_mark");
        // Imported events need the accounts' timestamp index; find out whether any are present.
        rc = sync_scalars(ctx);
        tmark(ctx, "host_sync");
    }
    if (!rc && (ctx->h_scalars->flags & kFlagImported)) {
        rc = check_imported_indexes(ctx, true);
        T = ctx->T;
    }
    if (!rc) {
        hipLaunchKernelGGL(tr_classify, grid, block, 0, ctx->stream, T, c, ctx->ev_slow);
        tmark(ctx, "tr_classify");
        hipLaunchKernelGGL(tr_fast, grid, block, 0, ctx->stream, T, c, ctx->ev_slow);
        tmark(ctx, "tr_fast");
        rc = hip_ok(ctx, hipGetLastError(), "launch") ? 0 : TBG_EHIP;
    }
    if (!rc) rc = run_replay_and_finalize(ctx, c, true);
    if (!rc) rc = end_call(ctx, n);
    ctx->stream = saved;
    // Rows are consumed whether or not the events created objects.
    ctx->T.tr_rows_used += n;
    ctx->tr_ts_stale = true;
    return rc;
}

int tbg_create_accounts_device(tbg_ctx* ctx, const tb_account_t* d_events, uint32_t n,
                               const uint32_t* d_batch_ends, const uint64_t* d_batch_ts,
                               uint32_t n_batches, tb_create_result_t* d_results, void* stream) {
    if (!ctx || n > ctx->opt.batch_events_max || n_batches > ctx->opt.batch_count_max)
        return TBG_EINVAL;
    if (ctx->T.acc_rows_used + n > ctx->opt.account_capacity) {
        ctx->error = "account capacity exceeded";
        return TBG_ENOSPC;
    }
    if (n == 0) return 0;
    hipStream_t user = static_cast<hipStream_t>(stream);
    hipStream_t saved = ctx->stream;
    if (user) ctx->stream = user;
    int rc = begin_call(ctx);
    Call<tb_account_t> c =
        make_call(ctx, d_events, n, d_batch_ends, d_batch_ts, n_batches, d_results, ctx->T.acc_rows_used);
    Tables T = ctx->T;
    const dim3 grid(grid_for(n)), block(kBlock);
    if (!rc) {
        hipLaunchKernelGGL(acc_prepare, grid, block, 0, ctx->stream, T, c);
        rc = sync_scalars(ctx);
    }
    if (!rc && (ctx->h_scalars->flags & kFlagImported)) {
        rc = check_imported_indexes(ctx, false);
        T = ctx->T;
    }
    if (!rc) {
        hipLaunchKernelGGL(acc_classify, grid, block, 0, ctx->stream, T, c, ctx->ev_slow);
        rc = hip_ok(ctx, hipGetLastError(), "launch") ? 0 : TBG_EHIP;
    }
    if (!rc) rc = run_replay_and_finalize(ctx, c, false);
    if (!rc) rc = end_call(ctx, n);
    ctx->stream = saved;
    ctx->T.acc_rows_used += n;
    ctx->acc_ts_stale = true;
    return rc;
}

static int upload_batches(tbg_ctx* ctx, uint32_t n, const uint32_t* batch_lens,
                          const uint64_t* batch_ts, uint32_t nb) {
    if (nb == 0 || nb > ctx->opt.batch_count_max) return TBG_EINVAL;
    ctx->h_ends.resize(nb);
    uint64_t total = 0;
    for (uint32_t b = 0; b < nb; b++) {
        total += batch_lens[b];
        ctx->h_ends[b] = uint32_t(total);
    }
    if (total != n) return TBG_EINVAL;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_batch_ends, ctx->h_ends.data(), nb * 4,
                                hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_batch_ts, batch_ts, nb * 8, hipMemcpyHostToDevice,
                                ctx->stream));
    return 0;
}

int tbg_create_transfers(tbg_ctx* ctx, const tb_transfer_t* events, uint32_t n,
                         const uint32_t* batch_lens, const uint64_t* batch_ts, uint32_t nb,
                         tb_create_result_t* results) {
    if (!ctx || n > ctx->opt.batch_events_max) return TBG_EINVAL;
    if (n == 0) return 0;
    int rc = upload_batches(ctx, n, batch_lens, batch_ts, nb);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_events, events, size_t(n) * 128, hipMemcpyHostToDevice,
                                ctx->stream));
    rc = tbg_create_transfers_device(ctx, reinterpret_cast<const tb_transfer_t*>(ctx->d_events), n,
                                     ctx->d_batch_ends, ctx->d_batch_ts, nb, ctx->d_results, nullptr);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(results, ctx->d_results, size_t(n) * 16, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

int tbg_create_accounts(tbg_ctx* ctx, const tb_account_t* events, uint32_t n,
                        const uint32_t* batch_lens, const uint64_t* batch_ts, uint32_t nb,
                        tb_create_result_t* results) {
    if (!ctx || n > ctx->opt.batch_events_max) return TBG_EINVAL;
    if (n == 0) return 0;
    int rc = upload_batches(ctx, n, batch_lens, batch_ts, nb);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_events, events, size_t(n) * 128, hipMemcpyHostToDevice,
                                ctx->stream));
    rc = tbg_create_accounts_device(ctx, reinterpret_cast<const tb_account_t*>(ctx->d_events), n,
                                    ctx->d_batch_ends, ctx->d_batch_ts, nb, ctx->d_results, nullptr);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(results, ctx->d_results, size_t(n) * 16, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

int64_t tbg_pulse(tbg_ctx* ctx, uint64_t timestamp) {
    if (!ctx) return TBG_EINVAL;
    int rc = sync_scalars(ctx);
    if (rc) return rc;
    const uint64_t count = std::min<uint64_t>(ctx->h_scalars->expiry_count, ctx->T.expiry_capacity);
    rc = ensure_pulse_scratch(ctx, count);
    if (rc) return rc;
    PulseScratch& S = ctx->pulse;
    unsigned long long h_counters[3] = {0, 0, ~0ull};  // kept, candidates, next unexpired
    HIP_TRY(ctx, hipMemcpyAsync(S.counters, h_counters, sizeof(h_counters), hipMemcpyHostToDevice,
                                ctx->stream));
    if (count)
        hipLaunchKernelGGL(pulse_collect, dim3(grid_for(count)), dim3(kBlock), 0, ctx->stream,
                           ctx->T, timestamp, count, S.keep, &S.counters[0], S.exp, S.ts, S.rows,
                           &S.counters[1], &S.counters[2]);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemcpyAsync(h_counters, S.counters, sizeof(h_counters), hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t kept = h_counters[0], cands = h_counters[1];
    const uint64_t batch_max = ctx->opt.pulse_batch_max;
    const uint64_t expired = std::min<uint64_t>(cands, batch_max);
    uint64_t pulse_next = h_counters[2] == ~0ull ? TB_TIMESTAMP_MAX : h_counters[2];
    const uint64_t* apply_rows = S.rows;
    if (cands >= batch_max) {
        // The expires_at index is ordered by (expires_at, timestamp) and the scan stops with
        // buffer_finished after batch_max values (scan_lookup.zig:150-175): expire the first
        // batch_max in that order. Row order is timestamp order, so a stable sort by row and
        // then a stable sort by expires_at yields the index order.
        size_t bytes = 0;
        HIP_TRY(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, S.rows, S.rows_b, S.exp,
                                                        S.exp_b, int(cands), 0, 64, ctx->stream));
        if (bytes > ctx->cub_temp_bytes) {
            if (ctx->cub_temp) (void)hipFree(ctx->cub_temp);
            ctx->cub_temp = nullptr;
            HIP_TRY(ctx, hipMalloc(&ctx->cub_temp, bytes));
            ctx->cub_temp_bytes = bytes;
        }
        HIP_TRY(ctx, hipcub::DeviceRadixSort::SortPairs(ctx->cub_temp, bytes, S.rows, S.rows_b,
                                                        S.exp, S.exp_b, int(cands), 0, 64,
                                                        ctx->stream));
        size_t bytes2 = 0;
        HIP_TRY(ctx, hipcub::DeviceRadixSort::SortPairs(nullptr, bytes2, S.exp_b, S.exp, S.rows_b,
                                                        S.rows, int(cands), 0, 64, ctx->stream));
        if (bytes2 > ctx->cub_temp_bytes) {
            if (ctx->cub_temp) (void)hipFree(ctx->cub_temp);
            ctx->cub_temp = nullptr;
            HIP_TRY(ctx, hipMalloc(&ctx->cub_temp, bytes2));
            ctx->cub_temp_bytes = bytes2;
        }
        HIP_TRY(ctx, hipcub::DeviceRadixSort::SortPairs(ctx->cub_temp, bytes2, S.exp_b, S.exp,
                                                        S.rows_b, S.rows, int(cands), 0, 64,
                                                        ctx->stream));
        uint64_t last = 0;
        HIP_TRY(ctx, hipMemcpyAsync(&last, S.exp + (batch_max - 1), 8, hipMemcpyDeviceToHost,
                                    ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        pulse_next = last;
        apply_rows = S.rows;
    }
    if (expired)
        hipLaunchKernelGGL(pulse_apply, dim3(grid_for(expired)), dim3(kBlock), 0, ctx->stream,
                           ctx->T, apply_rows, expired);
    HIP_TRY(ctx, hipGetLastError());
    // The index keeps the entries still pending (those just expired are filtered next time).
    if (kept)
        HIP_TRY(ctx, hipMemcpyAsync(ctx->T.expiry, S.keep, kept * 8, hipMemcpyDeviceToDevice,
                                    ctx->stream));
    unsigned long long kept_ull = kept;
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->d_scalars->expiry_count, &kept_ull, 8, hipMemcpyHostToDevice,
                                ctx->stream));
    unsigned long long next_ull = pulse_next;
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->d_scalars->pulse_next_timestamp, &next_ull, 8,
                                hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return int64_t(expired);
}

uint64_t tbg_pulse_next_timestamp(tbg_ctx* ctx) {
    if (!ctx || sync_scalars(ctx)) return 0;
    return ctx->h_scalars->pulse_next_timestamp;
}

static int64_t lookup_impl(tbg_ctx* ctx, const tb_uint128_t* ids, uint32_t n, void* out,
                           bool accounts) {
    if (!ctx) return TBG_EINVAL;
    if (n == 0) return 0;
    if (n > ctx->opt.batch_events_max) return TBG_EINVAL;
    // Scratch: ids in d_events, rows in ev_slot, found flags in ev_slow, selection in slow_list.
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_events, ids, size_t(n) * 16, hipMemcpyHostToDevice,
                                ctx->stream));
    const tb_uint128_t* d_ids = reinterpret_cast<const tb_uint128_t*>(ctx->d_events);
    if (accounts)
        hipLaunchKernelGGL(lookup_accounts_kernel, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream,
                           ctx->T, d_ids, n, ctx->ev_slot, ctx->ev_slow);
    else
        hipLaunchKernelGGL(lookup_transfers_kernel, dim3(grid_for(n)), dim3(kBlock), 0,
                           ctx->stream, ctx->T, d_ids, n, ctx->ev_slot, ctx->ev_slow);
    HIP_TRY(ctx, hipGetLastError());
    unsigned int* d_count = &ctx->d_scalars->slow_count;
    int rc = select_flagged(ctx, ctx->ev_slow, n, ctx->slow_list, d_count);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->h_scalars->slow_count, d_count, 4, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint32_t found = ctx->h_scalars->slow_count;
    if (found == 0) return 0;
    void* d_out = ctx->d_events + size_t(n) * 16;  // after the ids (128 B per event available)
    if (accounts)
        hipLaunchKernelGGL(gather_rows<tb_account_t>, dim3(grid_for(found)), dim3(kBlock), 0,
                           ctx->stream, ctx->T.acc_rows, ctx->ev_slot, ctx->slow_list, found,
                           static_cast<tb_account_t*>(d_out));
    else
        hipLaunchKernelGGL(gather_rows<tb_transfer_t>, dim3(grid_for(found)), dim3(kBlock), 0,
                           ctx->stream, ctx->T.tr_rows, ctx->ev_slot, ctx->slow_list, found,
                           static_cast<tb_transfer_t*>(d_out));
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemcpyAsync(out, d_out, size_t(found) * 128, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return found;
}

int64_t tbg_lookup_accounts(tbg_ctx* ctx, const tb_uint128_t* ids, uint32_t n, tb_account_t* out) {
    return lookup_impl(ctx, ids, n, out, true);
}

int64_t tbg_lookup_transfers(tbg_ctx* ctx, const tb_uint128_t* ids, uint32_t n,
                             tb_transfer_t* out) {
    return lookup_impl(ctx, ids, n, out, false);
}

int64_t tbg_dump_accounts(tbg_ctx* ctx, tb_account_t* out) {
    if (!ctx) return TBG_EINVAL;
    return dump_impl(ctx, ctx->T.acc_rows, ctx->T.acc_live, ctx->T.acc_rows_used, out, nullptr);
}

int64_t tbg_dump_transfers(tbg_ctx* ctx, tb_transfer_t* out, uint8_t* pending_status) {
    if (!ctx) return TBG_EINVAL;
    return dump_impl(ctx, ctx->T.tr_rows, ctx->T.tr_live, ctx->T.tr_rows_used, out,
                     pending_status);
}

int tbg_debug_set_account_balances(tbg_ctx* ctx, tb_uint128_t id, tb_uint128_t debits_pending,
                                   tb_uint128_t debits_posted, tb_uint128_t credits_pending,
                                   tb_uint128_t credits_posted) {
    if (!ctx) return TBG_EINVAL;
    int* d_rc = reinterpret_cast<int*>(&ctx->d_scalars->slow_count);
    hipLaunchKernelGGL(set_balances_kernel, dim3(1), dim3(1), 0, ctx->stream, ctx->T, id,
                       debits_pending, debits_posted, credits_pending, credits_posted, d_rc);
    HIP_TRY(ctx, hipGetLastError());
    int rc = 0;
    HIP_TRY(ctx, hipMemcpyAsync(&rc, d_rc, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return rc;
}

int tbg_last_stats(tbg_ctx* ctx, tbg_stats* out) {
    if (!ctx || !out) return TBG_EINVAL;
    *out = ctx->stats;
    return 0;
}

int tbg_debug_force_replay(tbg_ctx* ctx, int enable) {
    if (!ctx) return TBG_EINVAL;
    ctx->force_replay = enable != 0;
    return 0;
}

int tbg_profile(tbg_ctx* ctx, int enable) {
    if (!ctx) return TBG_EINVAL;
    ctx->timing = enable != 0;
    ctx->prof_names.clear();
    ctx->prof_ms.clear();
    ctx->prof_count.clear();
    return 0;
}

int tbg_profile_read(tbg_ctx* ctx, uint32_t index, char* name, uint32_t name_len,
                     double* total_ms, uint64_t* launches) {
    if (!ctx || index >= ctx->prof_names.size()) return 0;
    if (name && name_len) {
        snprintf(name, name_len, "%s", ctx->prof_names[index].c_str());
    }
    if (total_ms) *total_ms = ctx->prof_ms[index];
    if (launches) *launches = ctx->prof_count[index];
    return 1;
}

}  // extern "C"
