/*
 * tbg.h -- C ABI of the MI355X batch executor for TigerBeetle's commit path.
 *
 * The executor holds the state the reference keeps in its Forest grooves for this path, resident
 * in HBM: the account table (groove `accounts`), the transfer table with orphaned ids (groove
 * `transfers`), TransferPending statuses (groove `transfers_pending`), the `expires_at` index and
 * `pulse_next_timestamp`. It executes create_accounts / create_transfers / pulse with results
 * bit-identical to the reference's serial execution.
 *
 * Entry points and the reference interface each one replaces (all in src/state_machine.zig):
 *   tbg_create_accounts   <- execute_create(.create_accounts)   :3002-3213, create_account :3613
 *   tbg_create_transfers  <- execute_create(.create_transfers)  :3002-3213, create_transfer :3719
 *   tbg_pulse             <- prefetch_expire_pending_transfers  :2436-2562 +
 *                            execute_expire_pending_transfers   :4511-4628
 *   tbg_pulse_next_timestamp <- ExpirePendingTransfers.pulse_next_timestamp :4906-4909
 *   tbg_lookup_accounts   <- execute_lookup_accounts            :3255-3272
 *   tbg_lookup_transfers  <- execute_lookup_transfers           :3274-3292
 *   tbg_get_change_events <- execute_get_change_events          :3395-3527 (the account_events
 *                            groove written by account_event    :4384-4465)
 *   tbg_get_account_transfers / _balances, tbg_query_accounts / _transfers <- the scans
 *                            :1482-2123, :3294-3393 (below)
 * prefetch (:1146-1420) has no counterpart: every table is HBM-resident, nothing is staged.
 *
 * Batches: one call executes `n_batches` consecutive batches (a multi-batch body, or any sequence
 * of commits). Batch b holds batch_lens[b] events and `batch_timestamps[b]` is the `timestamp`
 * argument execute_create receives for it (its highest event timestamp); event i of batch b is
 * stamped batch_timestamps[b] - batch_lens[b] + i + 1. Batches are executed in order; linked
 * chains and the imported flag are scoped to a batch exactly as in the reference.
 *
 * Conventions: the caller owns every buffer. Calls are synchronous (results are on the host when
 * the call returns) except the *_device variants, which are stream-ordered and take device
 * pointers. A ctx is single-thread-affine (the reference state machine is single-threaded).
 * Return values: 0 (or a count) on success, a negative errno-style value on API misuse or a HIP
 * failure. Domain failures are per-event statuses in the results, never return codes.
 */
#ifndef TBG_H
#define TBG_H

#include "tb_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tbg_ctx tbg_ctx;

typedef struct tbg_options {
    uint64_t account_capacity;  /* max accounts ever submitted (rows + 2x hash slots) */
    uint64_t transfer_capacity; /* max transfer events ever submitted (rows + 2x hash slots) */
    uint32_t batch_events_max;  /* max events per call */
    uint32_t batch_count_max;   /* max batches per call */
    uint32_t pulse_batch_max;   /* batch_max.create_transfers: 8190 in production */
    uint32_t device;            /* HIP device ordinal */
    uint64_t pulse_next_timestamp_init; /* TB_TIMESTAMP_MIN in production */
    /* AccountEvents kept (the account_events groove, state_machine.zig:104-220: one per created
     * transfer, post/void and expiry); 0 = none are recorded (get_change_events returns none). */
    uint64_t account_events_capacity;
} tbg_options;

/* Errors (negative). */
#define TBG_EINVAL (-22)
#define TBG_ENOMEM (-12)
#define TBG_ENOSPC (-28)
#define TBG_EHIP (-5)

tbg_ctx* tbg_open(const tbg_options* options);
void tbg_close(tbg_ctx* ctx);
/* Last HIP / API error message of this ctx (never NULL). */
const char* tbg_last_error(const tbg_ctx* ctx);

int tbg_create_accounts(tbg_ctx* ctx, const tb_account_t* events, uint32_t n,
                        const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                        uint32_t n_batches, tb_create_result_t* results);
int tbg_create_transfers(tbg_ctx* ctx, const tb_transfer_t* events, uint32_t n,
                         const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                         uint32_t n_batches, tb_create_result_t* results);

/* Device-resident variants: every pointer is device memory; batch_ends[b] = exclusive end index
 * of batch b (prefix sum of batch_lens). Enqueued on `stream` (a hipStream_t, NULL = the ctx's
 * stream); results are complete when the stream reaches this point. */
int tbg_create_accounts_device(tbg_ctx* ctx, const tb_account_t* d_events, uint32_t n,
                               const uint32_t* d_batch_ends, const uint64_t* d_batch_timestamps,
                               uint32_t n_batches, tb_create_result_t* d_results, void* stream);
int tbg_create_transfers_device(tbg_ctx* ctx, const tb_transfer_t* d_events, uint32_t n,
                                const uint32_t* d_batch_ends, const uint64_t* d_batch_timestamps,
                                uint32_t n_batches, tb_create_result_t* d_results, void* stream);

/* A ledger shard's slice of a routed call (tigerbeetle_amd/shard.py): the events keep their
 * global commit timestamps, given per event (increasing, not necessarily contiguous); the slice is
 * one batch for linked-chain and imported semantics. Device pointers, stream-ordered. */
int tbg_create_transfers_stamped_device(tbg_ctx* ctx, const tb_transfer_t* d_events, uint32_t n,
                                        const uint64_t* d_event_timestamps,
                                        tb_create_result_t* d_results, void* stream);

/* The same with host buffers, synchronous, for create_accounts too: the router's exact path
 * (shard.py) sends a shard its events of an imported batch, or its part of a linked chain that
 * spans shards, this way -- every event keeps its global timestamp and the events are one batch.
 * `batch_timestamp` is the batch's `timestamp` (execute_create :3002-3104: imported events'
 * must_not_advance bound; 0 = the last event's). Timestamps must be nonzero and increasing (else
 * TBG_EINVAL). `options`: TBG_ONE_CHAIN -- the batch is one linked chain closed at its last event,
 * whatever the events' linked flags (which are stored and compared unchanged): a shard's part of a
 * chain across shards, probed with a failing last event or committed (executed by the ordered
 * replay on one lane). */
#define TBG_ONE_CHAIN 1u
int tbg_create_transfers_stamped(tbg_ctx* ctx, const tb_transfer_t* events, uint32_t n,
                                 const uint64_t* event_timestamps, uint64_t batch_timestamp,
                                 uint32_t options, tb_create_result_t* results);
int tbg_create_accounts_stamped(tbg_ctx* ctx, const tb_account_t* events, uint32_t n,
                                const uint64_t* event_timestamps, uint64_t batch_timestamp,
                                uint32_t options, tb_create_result_t* results);

/* Sharded linked chains (shard.py): a shard probes its part of a chain that spans shards, and the
 * chain's first failure across shards decides it (execute_create :3116-3172). An event the probe
 * executed past that failure may have orphaned its id (transient_error :3215-3252) although the
 * reference never executes it: tbg_forget_orphans returns such ids to unknown (a tombstone, as a
 * failed claim leaves). Returns the count forgotten (ids not orphaned are left alone). */
int64_t tbg_forget_orphans(tbg_ctx* ctx, const tb_uint128_t* ids, uint32_t n);

/* Sharded imported events: whether a live object of a groove (transfers != 0: transfers, else
 * accounts) holds each timestamp -- the `indirect_lookup` by timestamp that imported events'
 * must_not_regress checks make into the *other* groove (:3661-3665, :3813-3817), asked of every
 * shard by the router. out[i] = 0/1; returns the count found. */
int64_t tbg_timestamps_exist(tbg_ctx* ctx, int transfers, const uint64_t* timestamps, uint32_t n,
                             uint8_t* out);

/* Pins and maps a host buffer the caller reuses across calls (a replica's message bodies and
 * reply buffers; hipHostRegister, mapped): a host-buffer call whose events or results lie in a
 * registered range has its kernels read the body (tr_ingest, small calls) and write the results
 * over PCIe on the call's own stream -- no staged copy of pageable memory and no DMA-engine
 * hand-off. Unregistered at tbg_unregister_host or tbg_close. */
int tbg_register_host(tbg_ctx* ctx, void* ptr, uint64_t size);
int tbg_unregister_host(tbg_ctx* ctx, void* ptr);

/* Waits for every kernel and copy the ctx has queued on its own stream (e.g. the AccountEvents
 * appends a *_device call leaves behind it) -- for callers that reuse the call's device buffers
 * from other streams. */
int tbg_synchronize(tbg_ctx* ctx);

/* Returns the number of pending transfers expired (<= pulse_batch_max). */
int64_t tbg_pulse(tbg_ctx* ctx, uint64_t timestamp);
uint64_t tbg_pulse_next_timestamp(tbg_ctx* ctx);

/* Sharded pulses (one executor per ledger shard; the reference's single expires_at scan,
 * ExpirePendingTransfersType :4875-5029, spans all shards): the count of this shard's
 * expired-eligible pending transfers at `timestamp` and the first `max` of their index keys
 * (expires_at, timestamp) in order; then the pulse that expires exactly this shard's entries up to
 * and including a cut key -- the pulse_batch_max-th key across all shards, or the last key when
 * fewer expire -- and sets pulse_next_timestamp to `pulse_next_timestamp` (the cut's expires_at:
 * the scan's buffer filled), or, when it is 0, to this shard's first unexpired expires_at.
 * `event_timestamps` (NULL: timestamp - m + i + 1 locally) stamps this shard's i-th expiry with
 * its position in the pulse's expiry order over all shards, timestamp - E + position + 1
 * (execute_expire_pending_transfers :4540-4546): its AccountEvent's timestamp. Both return a
 * count or a negative error. */
int64_t tbg_pulse_candidates(tbg_ctx* ctx, uint64_t timestamp, uint64_t* expires_at,
                             uint64_t* timestamps, uint32_t max);
int64_t tbg_pulse_cut(tbg_ctx* ctx, uint64_t timestamp, uint64_t cut_expires_at,
                      uint64_t cut_timestamp, uint64_t pulse_next_timestamp,
                      const uint64_t* event_timestamps);

/* Sharded imported batches: raises the accounts / transfers objects trees' key_range.key_max
 * (read only by imported events' must_not_regress checks) to the maxima over every shard. */
int tbg_raise_key_max(tbg_ctx* ctx, uint64_t accounts_key_max, uint64_t transfers_key_max);
/* ... and reads this shard's (0: no key range yet), which the router raises every shard to. */
int tbg_key_max(tbg_ctx* ctx, uint64_t* accounts_key_max, uint64_t* transfers_key_max);

/* Sharded pulse_next_timestamp (one executor per ledger shard). A post/void of a pending transfer
 * with a timeout resets pulse_next_timestamp when it equals the transfer's expiry
 * (post_or_void_pending_transfer :4227-4229): a comparison against the value over *all* shards at
 * that point of the call. With tbg_set_pnt_sharded(ctx, 1) every create_transfers call records
 * each update at its event -- min(expires_at) of a pending transfer with a timeout
 * (create_transfer :3975-3982) or a reset-if-equal of a post/void -- applies the mins only, and
 * tbg_pnt_ops returns the last call's updates as (event timestamp, op) pairs in call order (op:
 * expires_at, with bit 63 set for a reset) and the value at the call's start. The caller merges
 * the shards' updates by timestamp, replays them from the minimum of the starts and, when a reset
 * fires, sets every shard's value to timestamp_min (tbg_set_pulse_next_timestamp). Returns the
 * count (at most `max` copied) or a negative error. */
int tbg_set_pnt_sharded(tbg_ctx* ctx, int on);
int64_t tbg_pnt_ops(tbg_ctx* ctx, uint64_t* timestamps, uint64_t* ops, uint64_t max,
                    uint64_t* start);
int tbg_set_pulse_next_timestamp(tbg_ctx* ctx, uint64_t value);

/* Found objects only, in request order; returns the count written. */
int64_t tbg_lookup_accounts(tbg_ctx* ctx, const tb_uint128_t* ids, uint32_t n, tb_account_t* out);
int64_t tbg_lookup_transfers(tbg_ctx* ctx, const tb_uint128_t* ids, uint32_t n,
                             tb_transfer_t* out);

/* Parity dumps: live objects in creation order; `out` may be NULL to query the count. */
int64_t tbg_dump_accounts(tbg_ctx* ctx, tb_account_t* out);
int64_t tbg_dump_transfers(tbg_ctx* ctx, tb_transfer_t* out, uint8_t* pending_status);
/* Every transfer id the transfers' id table holds -- created transfers and orphaned ids
 * (transient failures, :3215-3252), not tombstones -- in row order; out NULL: the count. A group
 * reopened from its shards' checkpoints rebuilds its router's directory from these
 * (tbg_group_open_checkpoint). */
int64_t tbg_dump_transfer_ids(tbg_ctx* ctx, tb_uint128_t* out);

/* The account_events groove (AccountEvent, state_machine.zig:104-220; written by account_event
 * :4384-4465 for every created transfer, post/void and expiry), in timestamp order; `out` may be
 * NULL to query the count. */
int64_t tbg_dump_account_events(tbg_ctx* ctx, tb_account_event_t* out);
/* get_change_events (state_machine.zig:2396-2434, :3395-3527): the ChangeEvents whose timestamps
 * lie in the filter's range, ascending, at most min(filter->limit, limit_max); 0 for an invalid
 * filter. Returns the count written. */
int64_t tbg_get_change_events(tbg_ctx* ctx, const tb_change_events_filter_t* filter,
                              uint32_t limit_max, tb_change_event_t* out);

/* Durability (the reference persists these tables through its Forest).
 *   tbg_compact          <- StateMachine.compact (state_machine.zig:2912-2935): drops the rows of
 *                           transfer events that created no object and orphaned no id (rows are
 *                           consumed by every event), rebuilds the transfer id index without the
 *                           tombstones of failed claims, keeps row order (= timestamp order).
 *                           Returns the rows freed (>= 0) or an error. Results of later calls are
 *                           unchanged by it. A failure once rows have begun to move leaves the
 *                           tables undefined: every later call on the ctx returns TBG_EHIP.
 *   tbg_checkpoint       <- StateMachine.checkpoint (:2937-2958): writes an image of every
 *                           persistent table (accounts, transfers, TransferPending, expires_at,
 *                           AccountEvents, pulse_next_timestamp, key ranges) with a checksum of
 *                           its header and of every section to `path`.tmp, fsyncs it, renames it
 *                           over `path` and fsyncs the directory (an atomic, durable switch).
 *   tbg_open_checkpoint  <- StateMachine.open (:964-978): opens a ctx with `options` (the same
 *                           capacities as the ctx that wrote the image) and loads the image; NULL
 *                           if the image is unreadable, does not fit, or fails a checksum
 *                           (nothing of a torn image is installed). */
int64_t tbg_compact(tbg_ctx* ctx);
int tbg_checkpoint(tbg_ctx* ctx, const char* path);
tbg_ctx* tbg_open_checkpoint(const tbg_options* options, const char* path);

/* The scans (state_machine.zig, prefetch_*_scan + execute_*): objects in timestamp order
 * (descending with the filter's `reversed` flag) within [timestamp_min, timestamp_max], at most
 * min(filter->limit, limit_max); 0 results for an invalid filter. Returns the count written.
 *   tbg_get_account_transfers <- get_scan_from_account_filter :1737-1841 (the transfers whose
 *                                debit and/or credit account is filter->account_id, AND the
 *                                nonzero user_data_128/64/32 and code), execute :3294-3310
 *   tbg_get_account_balances  <- prefetch_get_account_balances_scan :1608-1675 (the account must
 *                                exist with flags.history; the same transfer scan, each mapped to
 *                                its AccountEvent by timestamp), execute :3312-3357. Needs
 *                                account_events_capacity > 0 (else TBG_EINVAL).
 *   tbg_query_accounts        <- get_scan_from_query_filter :2054-2123 over the accounts groove
 *   tbg_query_transfers       <- the same over the transfers groove (ledger, code, user data) */
int64_t tbg_get_account_transfers(tbg_ctx* ctx, const tb_account_filter_t* filter,
                                  uint32_t limit_max, tb_transfer_t* out);
int64_t tbg_get_account_balances(tbg_ctx* ctx, const tb_account_filter_t* filter,
                                 uint32_t limit_max, tb_account_balance_t* out);
int64_t tbg_query_accounts(tbg_ctx* ctx, const tb_query_filter_t* filter, uint32_t limit_max,
                           tb_account_t* out);
int64_t tbg_query_transfers(tbg_ctx* ctx, const tb_query_filter_t* filter, uint32_t limit_max,
                            tb_transfer_t* out);

/* Test-harness `setup` action (src/state_machine_tests.zig:657-676). */
int tbg_debug_set_account_balances(tbg_ctx* ctx, tb_uint128_t id, tb_uint128_t debits_pending,
                                   tb_uint128_t debits_posted, tb_uint128_t credits_pending,
                                   tb_uint128_t credits_posted);

/* Per-call execution statistics of the last create_* call (diagnostics / bench). */
typedef struct tbg_stats {
    uint64_t events;       /* events in the call */
    uint64_t fast;         /* applied by the parallel path */
    uint64_t replayed;     /* executed by the ordered replay */
    uint64_t static_fail;  /* failed on checks that depend on no in-call state */
    uint64_t ae_window;    /* the call's AccountEvents in one pass: 1 balance-window emit, 2 dense
                            * emit (general calls, dense key spaces), 3 balance-window emit with
                            * u128 sums (wide amounts); 0 the general appends or the side stream
                            * (small calls) */
    uint64_t ingest_finished;  /* 1: the call ended in tr_ingest's last workgroup (a small call
                                * whose events were all FAST: no tr_commit or stage_out work) */
} tbg_stats;
int tbg_last_stats(tbg_ctx* ctx, tbg_stats* out);

/* The executor's overflow predicate, sum_overflows (state_machine.zig:5144-5149), on `n` operand
 * pairs of `bits` = 64 (low words only) or 128: out[i] = 1 iff a[i] + b[i] overflows. ctx NULL
 * evaluates it on the host; otherwise a kernel on the ctx's device (the code the replay runs).
 * Pins the predicate to the reference's "sum_overflows" test (:5151-5166). */
int tbg_sum_overflows(tbg_ctx* ctx, uint32_t bits, const tb_uint128_t* a, const tb_uint128_t* b,
                      uint32_t n, uint8_t* out);

/* Forces every event through the ordered replay (self-check of the fast path). */
int tbg_debug_force_replay(tbg_ctx* ctx, int enable);

/* Runs every ordered replay of create_transfers on one lane in call order (replay_kernel) instead
 * of the flow replay (many lanes, units ordered by the keys they share): a self-check of the
 * flow replay's exactness. */
int tbg_debug_serial_replay(tbg_ctx* ctx, int enable);
/* Debug / A-B: 1 = every AccountEvents append on the call's stream (no side stream; the default
 * hands a call of <= 8192 events' appends to a side stream behind the next call). */
int tbg_debug_ae_sync(tbg_ctx* ctx, int enable);

/* Per-kernel timing with HIP events on the call's stream (off by default; resets the totals);
 * enable == 2 records only the host-wall phases of host-buffer calls (host:*), no HIP events;
 * enable == 3 records only the marks that bound a call's device spans (no per-kernel entries: each
 * mark recorded between two launches idles the GPU a few microseconds).
 * tbg_profile_read returns 1 and fills name / accumulated milliseconds / launches for entry
 * `index`, or 0 past the last entry. */
int tbg_profile(tbg_ctx* ctx, int enable);
int tbg_profile_read(tbg_ctx* ctx, uint32_t index, char* name, uint32_t name_len,
                     double* total_ms, uint64_t* launches);

#ifdef __cplusplus
}
#endif

#endif /* TBG_H */
