/*
 * tb_oracle.h -- CPU oracle for the create_accounts / create_transfers commit path.
 *
 * TEST INFRASTRUCTURE ONLY. This is a serial, single-threaded C restatement of the reference's
 * state machine (src/state_machine.zig) used as the parity checker for the HIP executor and as
 * the CPU baseline leg of bench.py. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline may load it; the product path (tigerbeetle_amd/, libtbg.so) never does.
 *
 * Parity is pinned by the reference's own table-driven tests (src/state_machine_tests.zig,
 * transcribed as data under tests/golden/tables/ by tests/golden/extract_tables.py).
 */
#ifndef TB_ORACLE_H
#define TB_ORACLE_H

#include "../include/tb_types.h"
#include "../include/tb_state_machine.h"
#include "../include/tbg_group.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tbo_ctx tbo_ctx;

/* pulse_batch_max: transfers expired per pulse (batch_max.create_transfers; 8190 in production,
 * 30 under the reference's test config). pulse_next_timestamp_init: TB_TIMESTAMP_MIN in
 * production (state_machine.zig:4908), TB_TIMESTAMP_MAX in the unit-test harness
 * (state_machine_tests.zig:148-157). */
tbo_ctx* tbo_open(uint32_t pulse_batch_max, uint64_t pulse_next_timestamp_init);
void tbo_close(tbo_ctx* ctx);

/* execute_create (state_machine.zig:3002-3213) for one batch whose highest timestamp is
 * `timestamp`; event i gets timestamp - n + i + 1. Writes n dense results. */
void tbo_create_accounts(tbo_ctx* ctx, const tb_account_t* events, uint32_t n, uint64_t timestamp,
                         tb_create_result_t* results);
void tbo_create_transfers(tbo_ctx* ctx, const tb_transfer_t* events, uint32_t n,
                          uint64_t timestamp, tb_create_result_t* results);

/* Sharded calls (test instrumentation; the shard executor contract of tigerbeetle_amd/shard.py,
 * include/tbg.h): a multi-batch call (batch b: lens[b] events, timestamp batch_ts[b]) whose
 * pulse_next_timestamp log (tbo_pnt_ops) covers the call; a one-batch call whose events carry
 * their own timestamps `stamps` (`timestamp` = the batch's, 0 = the last stamp; options bit 0: one
 * linked chain closed at the last event, whatever the linked flags); orphaned ids
 * returned to unknown; whether live objects of a groove hold timestamps (out[i] = 0/1). */
void tbo_create_accounts_batches(tbo_ctx* ctx, const tb_account_t* events, const uint32_t* lens,
                                 const uint64_t* batch_ts, uint32_t nb,
                                 tb_create_result_t* results);
void tbo_create_transfers_batches(tbo_ctx* ctx, const tb_transfer_t* events, const uint32_t* lens,
                                  const uint64_t* batch_ts, uint32_t nb,
                                  tb_create_result_t* results);
void tbo_create_accounts_stamped(tbo_ctx* ctx, const tb_account_t* events, uint32_t n,
                                 const uint64_t* stamps, uint64_t timestamp, uint32_t options,
                                 tb_create_result_t* results);
void tbo_create_transfers_stamped(tbo_ctx* ctx, const tb_transfer_t* events, uint32_t n,
                                  const uint64_t* stamps, uint64_t timestamp, uint32_t options,
                                  tb_create_result_t* results);
uint64_t tbo_forget_orphans(tbo_ctx* ctx, const tb_uint128_t* ids, uint32_t n);
void tbo_key_max(const tbo_ctx* ctx, uint64_t* accounts_key_max, uint64_t* transfers_key_max);
uint64_t tbo_timestamps_exist(const tbo_ctx* ctx, int transfers, const uint64_t* ts, uint32_t n,
                              uint8_t* out);

/* pulse: prefetch_expire_pending_transfers + execute_expire_pending_transfers
 * (state_machine.zig:2436-2562, :4511-4628, :4875-5029). Returns the number expired. */
uint32_t tbo_pulse(tbo_ctx* ctx, uint64_t timestamp);
/* Sharded pulses: the expired-eligible entries of this shard's expires_at index,
 * in (expires_at, timestamp) order -- their count, and the first `max` keys; then the pulse that
 * expires exactly the entries up to a cut key (the global pulse_batch_max-th across shards) and
 * sets pulse_next_timestamp (the cut's expires_at, as ExpirePendingTransfers.finish does when its
 * buffer fills). */
uint64_t tbo_pulse_candidates(tbo_ctx* ctx, uint64_t timestamp, uint64_t* expires_at,
                              uint64_t* timestamps, uint32_t max);
uint32_t tbo_pulse_cut(tbo_ctx* ctx, uint64_t timestamp, uint64_t cut_expires_at,
                       uint64_t cut_timestamp, uint64_t pulse_next_timestamp,
                       const uint64_t* stamps);
int tbo_pulse_needed(const tbo_ctx* ctx, uint64_t timestamp);
uint64_t tbo_pulse_next_timestamp(const tbo_ctx* ctx);

/* execute_lookup_accounts / execute_lookup_transfers (state_machine.zig:3255-3292):
 * found objects only, in request order. Returns the count written. */
uint32_t tbo_lookup_accounts(const tbo_ctx* ctx, const tb_uint128_t* ids, uint32_t n,
                             tb_account_t* out);
uint32_t tbo_lookup_transfers(const tbo_ctx* ctx, const tb_uint128_t* ids, uint32_t n,
                              tb_transfer_t* out);

/* Test-harness `setup` action (state_machine_tests.zig:657-676): overwrite balances. */
int tbo_set_account_balances(tbo_ctx* ctx, tb_uint128_t id, tb_uint128_t debits_pending,
                             tb_uint128_t debits_posted, tb_uint128_t credits_pending,
                             tb_uint128_t credits_posted);

/* Dumps for parity checks. Returns counts; `out` may be NULL to query the count. */
uint64_t tbo_account_count(const tbo_ctx* ctx);
uint64_t tbo_transfer_count(const tbo_ctx* ctx);
uint64_t tbo_dump_accounts(const tbo_ctx* ctx, tb_account_t* out);   /* creation order */
uint64_t tbo_dump_transfers(const tbo_ctx* ctx, tb_transfer_t* out); /* creation order */
uint64_t tbo_dump_pending_status(const tbo_ctx* ctx, uint8_t* out);  /* per transfer */

/* Sharded imported batches: raises the objects trees' key_range.key_max to the
 * maxima over every shard (0 = leave), so that imported `must_not_regress` checks see them. */
void tbo_raise_key_max(tbo_ctx* ctx, uint64_t accounts_key_max, uint64_t transfers_key_max);

/* The account_events groove in insertion order (AccountEvent, state_machine.zig:104-220). */
uint64_t tbo_dump_account_events(const tbo_ctx* ctx, tb_account_event_t* out);
/* get_change_events (state_machine.zig:2396-2434, :3395-3527): ChangeEvents with timestamps in the
 * filter's range, ascending, at most min(filter->limit, limit_max); 0 for an invalid filter. */
int64_t tbo_get_change_events(const tbo_ctx* ctx, const tb_change_events_filter_t* filter,
                              uint32_t limit_max, tb_change_event_t* out);

/* The scans (state_machine.zig:1482-2123, :3294-3393): see tbg.h. */
int64_t tbo_get_account_transfers(const tbo_ctx* ctx, const tb_account_filter_t* filter,
                                  uint32_t limit_max, tb_transfer_t* out);
int64_t tbo_get_account_balances(const tbo_ctx* ctx, const tb_account_filter_t* filter,
                                 uint32_t limit_max, tb_account_balance_t* out);
int64_t tbo_query_accounts(const tbo_ctx* ctx, const tb_query_filter_t* filter,
                           uint32_t limit_max, tb_account_t* out);
int64_t tbo_query_transfers(const tbo_ctx* ctx, const tb_query_filter_t* filter,
                            uint32_t limit_max, tb_transfer_t* out);

/* Sharded pulse_next_timestamp (test instrumentation for the ledger shards, shard.py): with
 * `on`, every update of create_transfer (:3975-3982, `min`, applied) and of
 * post_or_void_pending_transfer (:4227-4229, reset-if-equal: logged, not applied) is logged with
 * its event's timestamp; tbo_pnt_ops returns the log since the last read (count; with ts / ops
 * non-null it copies and clears) and the value before its first entry; the caller resolves the
 * resets across shards and sets the value. Op encoding: expires_at, | 1 << 63 for a reset. */
void tbo_pnt_sharded(tbo_ctx* ctx, int on);
uint64_t tbo_pnt_ops(tbo_ctx* ctx, uint64_t* ts, uint64_t* ops, uint64_t* start);
void tbo_set_pulse_next_timestamp(tbo_ctx* ctx, uint64_t value);

/* Binds this oracle as a tb_executor (tb_state_machine.h) for the StateMachine mirror. */
void tbo_executor_fill(tbo_ctx* ctx, tb_executor* ex);
/* The shard executor interface (tbg_group.h) over tbo_ctx shards: tbg_group_open_shards. */
void tbo_shard_ops_fill(tbg_shard_ops* ops);

#ifdef __cplusplus
}
#endif

#endif /* TB_ORACLE_H */
