// The scans over the HBM tables: get_account_transfers, get_account_balances, query_accounts,
// query_transfers (state_machine.zig:1482-2123 prefetch scans, :3294-3393 execution).
//
// The reference answers these from the grooves' secondary indexes (LSM trees keyed by
// (field value, timestamp)): intersections of index scans in timestamp order. Here every live row
// is tested against the filter in one coalesced pass (one lane per row, 128-B rows read once), the
// matches are selected in row order -- which is timestamp order: rows are appended as objects are
// created and timestamps only grow, imported ones included -- and the first `limit` (or the last,
// reversed) are gathered. A scan is HBM-bound: 129 bytes per live row.
#pragma once

#include "events.hpp"

namespace tbg {

// A filter as the match kernels see it (AccountFilter or QueryFilter).
struct ScanFilter {
    u128 account_id;   // AccountFilter only (0: a QueryFilter)
    u128 user_data_128;
    uint64_t user_data_64;
    uint32_t user_data_32;
    uint32_t ledger;   // QueryFilter only
    uint32_t code;
    uint32_t sides;    // TB_ACCOUNT_FILTER_DEBITS | _CREDITS (AccountFilter)
    uint64_t ts_lo, ts_hi;
};

template <typename Row>
__device__ inline bool scan_common_match(const ScanFilter& f, const Row& o) {
    return o.timestamp >= f.ts_lo && o.timestamp <= f.ts_hi &&
           (f.user_data_128 == 0 || f.user_data_128 == U(o.user_data_128)) &&
           (f.user_data_64 == 0 || f.user_data_64 == o.user_data_64) &&
           (f.user_data_32 == 0 || f.user_data_32 == o.user_data_32) &&
           (f.code == 0 || f.code == o.code);
}

// get_scan_from_account_filter (:1737-1841): (debit OR credit account) AND the nonzero fields.
__global__ void scan_match_account_transfers(const tb_transfer_t* rows, const uint8_t* live,
                                             uint64_t used, ScanFilter f, uint8_t* match) {
    const uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r >= used) return;
    bool m = false;
    if (live[r]) {
        const tb_transfer_t& t = rows[r];
        const bool side = ((f.sides & TB_ACCOUNT_FILTER_DEBITS) && U(t.debit_account_id) == f.account_id) ||
                          ((f.sides & TB_ACCOUNT_FILTER_CREDITS) && U(t.credit_account_id) == f.account_id);
        m = side && scan_common_match(f, t);
    }
    match[r] = m;
}

// get_scan_from_query_filter (:2054-2123): the nonzero fields, ledger included.
template <typename Row>
__global__ void scan_match_query(const Row* rows, const uint8_t* live, uint64_t used, ScanFilter f,
                                 uint8_t* match) {
    const uint64_t r = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (r >= used) return;
    bool m = false;
    if (live[r]) {
        const Row& o = rows[r];
        m = (f.ledger == 0 || f.ledger == o.ledger) && scan_common_match(f, o);
    }
    match[r] = m;
}

// Result j: the j-th selected row, or the j-th from the end when reversed.
__device__ inline uint32_t scan_pick(const uint32_t* sel, uint32_t count, uint32_t j, bool reversed) {
    return sel[reversed ? count - 1 - j : j];
}

template <typename Row>
__global__ void scan_gather(const Row* rows, const uint32_t* sel, uint32_t count, uint32_t n,
                            int reversed, Row* out) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j < n) copy_row(&out[j], &rows[scan_pick(sel, count, j, reversed != 0)]);
}

// execute_get_account_balances (:3312-3357) over AccountBalancesScanLookup (:619-624): each
// selected transfer's AccountEvent -- the one with its timestamp, found by binary search in the
// timestamp-ordered log -- as the filter account's side of it.
__global__ void scan_balances(const tb_transfer_t* rows, const uint32_t* sel, uint32_t count,
                              uint32_t n, int reversed, const tb_account_event_t* log,
                              uint64_t log_n, u128 account_id, tb_account_balance_t* out,
                              unsigned int* missing) {
    const uint32_t j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t ts = rows[scan_pick(sel, count, j, reversed != 0)].timestamp;
    uint64_t lo = 0, hi = log_n;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (log[mid].timestamp < ts) lo = mid + 1;
        else hi = mid;
    }
    tb_account_balance_t b;
    memset(&b, 0, sizeof(b));
    b.timestamp = ts;
    if (lo < log_n && log[lo].timestamp == ts) {
        const tb_account_event_t& e = log[lo];
        if (U(e.dr_account_id) == account_id) {
            b.debits_pending = e.dr_debits_pending;
            b.debits_posted = e.dr_debits_posted;
            b.credits_pending = e.dr_credits_pending;
            b.credits_posted = e.dr_credits_posted;
        } else {
            b.debits_pending = e.cr_debits_pending;
            b.debits_posted = e.cr_debits_posted;
            b.credits_pending = e.cr_credits_pending;
            b.credits_posted = e.cr_credits_posted;
        }
    } else {
        atomicAdd(missing, 1u);  // (every created transfer has its AccountEvent)
    }
    out[j] = b;
}

}  // namespace tbg
