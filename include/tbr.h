/*
 * tbr.h -- C ABI of the device-side ledger router (multi-GPU).
 *
 * A client call (create_transfers over any number of batches) enters at one GPU; the router
 * assigns every event to the ledger shard (GPU) that holds its accounts, and scatters the call
 * into per-shard slices that keep every event's global commit timestamp (executed there with
 * tbg_create_transfers_stamped_device). Its directories -- account id -> shard, transfer id ->
 * shard (created and orphaned ids) -- are HBM open-addressing tables probed like the executor's
 * id tables. The group (tbg_group.h) drives it.
 *
 * The device path (tbr_route_device) places:
 *  * an event whose id already exists: on its holder (create_transfer_exists / id_already_failed,
 *    :3733-3738, come before any account lookup);
 *  * an event whose status follows from itself alone (nonzero padding, id 0 / maxInt, a nonzero
 *    timestamp; an unknown debit and credit account; a post/void whose pending transfer exists
 *    nowhere): on any shard (k mod shards, or its chain's);
 *  * a transfer: on its accounts' shard, the known one's if the other is unknown; accounts on two
 *    shards: a surrogate (credit := debit, accounts_must_be_different) whose status settle patches
 *    to the reference's (:3756-3798);
 *  * a post/void: on its pending transfer's shard (in the directory or created earlier in the
 *    call);
 *  * an id repeated in the call: on its first occurrence's shard, when its own placement allows;
 *  * a linked chain: whole on one shard, closed within its batch;
 *  * imported events: when every event of the call is imported, their timestamps increase
 *    through the call, lie below their own commit timestamps and above the imported floor
 *    (tbr_set_imported_floor).
 * Any other event is a *hazard*: the call is left to the exact engine (tbg_group.h, engine.cpp),
 * which reads the same directories through tbr_account_shards / tbr_transfer_shards and records its
 * outcome with tbr_record_*.
 *
 * Reference: the shard boundary follows `accounts_must_have_the_same_ledger` /
 * `transfer_must_have_the_same_ledger_as_accounts` (src/state_machine.zig:3795-3798); transfer
 * ids are global (create_transfer's id lookup, :3733-3760).
 */
#ifndef TBR_H
#define TBR_H

#include "tb_types.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tbr_ctx tbr_ctx;

tbr_ctx* tbr_open(uint32_t shards, uint64_t account_capacity, uint64_t transfer_capacity,
                  uint32_t events_max, uint32_t device);
void tbr_close(tbr_ctx* ctx);

/* Directory access (host buffers). Lookups write the shard or -1. */
int tbr_record_accounts(tbr_ctx* ctx, const tb_uint128_t* ids, const uint8_t* shards, uint32_t n);
int tbr_record_transfers(tbr_ctx* ctx, const tb_uint128_t* ids, const uint8_t* shards, uint32_t n);
int64_t tbr_account_shards(tbr_ctx* ctx, const tb_uint128_t* ids, uint32_t n, int32_t* out);
int64_t tbr_transfer_shards(tbr_ctx* ctx, const tb_uint128_t* ids, uint32_t n, int32_t* out);

/* Imported events on the fast path (execute_create :3066-3078, create_transfer :3800-3830): their
 * must_not_regress checks read the objects trees' key ranges and the accounts' timestamps over all
 * shards. The caller keeps `floor` at or above the largest timestamp of any account or transfer on
 * any shard (tbg_key_max over the shards; raised by the created_timestamp_max of each settled
 * call); an imported timestamp above it, in a call whose imported timestamps increase, collides
 * with nothing and regresses past nothing on any shard. UINT64_MAX (the initial value): every
 * imported event is a hazard. */
int tbr_set_imported_floor(tbr_ctx* ctx, uint64_t floor);

/* The fast path (device pointers, synchronous). Returns 0 when the call was routed: slices in
 * shard order at d_out_events / d_out_timestamps (event i of shard s at offset
 * sum(shard_counts[< s]) + i), d_out_positions = each slice event's position in the call,
 * shard_counts[shards] on the host; the call's ids are held for it until tbr_settle_device.
 * Returns 2 instead of 0 when the call posts or voids: its shards' pulse_next_timestamp updates
 * are then resolved across shards after it (tbg_pnt_ops, post_or_void_pending_transfer
 * :4227-4229). Returns 1 when the call holds a hazard (nothing routed, nothing held); < 0 on
 * error. */
int64_t tbr_route_device(tbr_ctx* ctx, const tb_transfer_t* d_events, uint32_t n,
                         const uint32_t* d_batch_ends, const uint64_t* d_batch_timestamps,
                         uint32_t n_batches, tb_transfer_t* d_out_events,
                         uint64_t* d_out_timestamps, uint32_t* d_out_positions,
                         uint32_t* shard_counts);
/* A shard's slice of a routed call (device pointers, possibly in another GPU's HBM: the scatter
 * stores and settle reads across xGMI, no staging copy): where its events and their global
 * commit timestamps go, and where its executor writes their results. */
typedef struct tbr_slice {
    tb_transfer_t* events;
    uint64_t* timestamps;
    const tb_create_result_t* results;
    uint64_t capacity; /* events the slice holds: a call that routes more to it returns -22 */
} tbr_slice;
/* tbr_route_device with every shard's slice at its own `slices[s]` (host array of `shards`
 * entries); d_out_positions = each slice event's position in the call, in shard order. Settle with
 * d_shard_results NULL (the results are read from the slices). */
int64_t tbr_route_device_slices(tbr_ctx* ctx, const tb_transfer_t* d_events, uint32_t n,
                                const uint32_t* d_batch_ends, const uint64_t* d_batch_timestamps,
                                uint32_t n_batches, const tbr_slice* slices,
                                uint32_t* d_out_positions, uint32_t* shard_counts);
/* The routed call's results (in shard order) back to call order; records the ids that now exist
 * on their shard (created, or orphaned by a transient failure) and releases the others.
 * *created_timestamp_max (if not NULL) receives the largest timestamp of a created transfer (0 if
 * none): the transfers objects tree's key_range.key_max the host router keeps for imported
 * events' must_not_regress checks (:3808-3817). */
int tbr_settle_device(tbr_ctx* ctx, const tb_create_result_t* d_shard_results,
                      const uint32_t* d_positions, uint32_t n, tb_create_result_t* d_results,
                      uint64_t* created_timestamp_max);
/* The last tbr_route_device call's counts: out[0] events placed anywhere, out[1] surrogates,
 * out[2] repeats of an id of the call. */
int tbr_route_stats(tbr_ctx* ctx, uint64_t* out);

#ifdef __cplusplus
}
#endif

#endif /* TBR_H */
