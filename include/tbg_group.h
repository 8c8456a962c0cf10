/*
 * tbg_group.h -- C ABI of the ledger-sharded executor group: one process owns N executors (one
 * per GPU of a node, or several on one GPU) and executes every call exactly as the reference's
 * single serial state machine would.
 *
 * The reference commits from one StateMachine inside one replica process (ReplicaType(StateMachine,
 * ...), src/vsr/replica.zig:144-152; a synchronous commit, src/state_machine.zig:2564-2669). A
 * group is that StateMachine's executor over N GPUs: the replica's shim calls tbg_group_* where a
 * single-GPU shim calls tbg_* (or binds the group as a tb_executor, tbg_group_executor, under
 * tb_sm_open). Debit and credit accounts share the transfer's ledger
 * (accounts_must_have_the_same_ledger / transfer_must_have_the_same_ledger_as_accounts,
 * :3795-3798), so every shard owns a contiguous range of ledgers: their accounts, transfer ids,
 * transfer rows, TransferPending statuses and expiries.
 *
 *   tbg_group_create_accounts      <- execute_create(.create_accounts)  :3002-3213, :3613-3703
 *   tbg_group_create_transfers(_device) <- execute_create(.create_transfers) :3002-3213, :3719-4382
 *   tbg_group_pulse                <- execute_expire_pending_transfers  :4511-4628, :4875-5029
 *   tbg_group_pulse_next_timestamp <- ExpirePendingTransfers.pulse_next_timestamp :4906-4909
 *   tbg_group_lookup_accounts / _transfers <- execute_lookup_*          :3255-3292
 *
 * A call takes one of two paths:
 *  * the device path (groups of HIP executors): the device router (router.hip) assigns every event
 *    a shard from HBM directories (account id -> shard, transfer id -> shard), scatters the call
 *    into per-shard slices that keep every event's global commit timestamp, copies each slice to
 *    its shard's GPU (peer copies over xGMI), every shard executes its slice on its own host
 *    thread, and the 16-byte results come back in call order. Events whose status follows from
 *    themselves alone (a nonzero padding, an id 0 / maxInt, a nonzero timestamp, an unknown
 *    account, a pending transfer found nowhere) run on any shard; a transfer between two shards'
 *    accounts runs as a surrogate whose status is patched to the reference's; an id repeated in the
 *    call runs on its first occurrence's shard.
 *  * the exact engine (every group; the only path of a group opened over other executors): a call
 *    the router cannot place -- a linked chain across shards, an imported batch that could regress
 *    past another shard's objects, a repeated id that may run elsewhere -- is cut into segments
 *    executed shard by shard, with the chain protocol for chains across shards (probe, first
 *    failure across shards, commit or roll back), key-range sync for imported events, surrogates
 *    for cross-shard transfers and pulse_next_timestamp resolved across shards.
 * Both give every event the status and timestamp the reference's serial execution gives it.
 *
 * Conventions: as tbg.h -- the caller owns every buffer, calls are synchronous, a group is
 * single-thread-affine, returns are 0 / a count or a negative TBG_E* code.
 */
#ifndef TBG_GROUP_H
#define TBG_GROUP_H

#include "tb_state_machine.h"
#include "tb_types.h"
#include "tbg.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tbg_group tbg_group;

#define TBG_GROUP_SHARDS_MAX 64

/* The shard executor interface: every member has the signature and meaning of the tbg.h function
 * of the same name (`self` in place of the tbg_ctx). A group over HIP executors binds the tbg_*
 * functions themselves; tests bind another executor with the same semantics (the CPU oracle). */
typedef struct tbg_shard_ops {
    int (*create_accounts)(void* self, const tb_account_t* events, uint32_t n,
                           const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                           uint32_t n_batches, tb_create_result_t* results);
    int (*create_transfers)(void* self, const tb_transfer_t* events, uint32_t n,
                            const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                            uint32_t n_batches, tb_create_result_t* results);
    int (*create_accounts_stamped)(void* self, const tb_account_t* events, uint32_t n,
                                   const uint64_t* event_timestamps, uint64_t batch_timestamp,
                                   uint32_t options, tb_create_result_t* results);
    int (*create_transfers_stamped)(void* self, const tb_transfer_t* events, uint32_t n,
                                    const uint64_t* event_timestamps, uint64_t batch_timestamp,
                                    uint32_t options, tb_create_result_t* results);
    int64_t (*forget_orphans)(void* self, const tb_uint128_t* ids, uint32_t n);
    int64_t (*timestamps_exist)(void* self, int transfers, const uint64_t* timestamps, uint32_t n,
                                uint8_t* out);
    int (*key_max)(void* self, uint64_t* accounts_key_max, uint64_t* transfers_key_max);
    int (*raise_key_max)(void* self, uint64_t accounts_key_max, uint64_t transfers_key_max);
    int (*set_pnt_sharded)(void* self, int on);
    int64_t (*pnt_ops)(void* self, uint64_t* timestamps, uint64_t* ops, uint64_t max,
                       uint64_t* start);
    uint64_t (*pulse_next_timestamp)(void* self);
    int (*set_pulse_next_timestamp)(void* self, uint64_t value);
    int64_t (*pulse_candidates)(void* self, uint64_t timestamp, uint64_t* expires_at,
                                uint64_t* timestamps, uint32_t max);
    int64_t (*pulse_cut)(void* self, uint64_t timestamp, uint64_t cut_expires_at,
                         uint64_t cut_timestamp, uint64_t pulse_next_timestamp,
                         const uint64_t* event_timestamps);
    int64_t (*lookup_accounts)(void* self, const tb_uint128_t* ids, uint32_t n, tb_account_t* out);
    int64_t (*lookup_transfers)(void* self, const tb_uint128_t* ids, uint32_t n,
                                tb_transfer_t* out);
} tbg_shard_ops;

typedef struct tbg_group_options {
    uint32_t shards;          /* 1..TBG_GROUP_SHARDS_MAX */
    uint32_t ledgers;         /* ledgers 1..ledgers map to shards by contiguous ranges (64 / G in
                               * config 5); any other ledger to ledger % shards */
    uint32_t events_max;      /* max events per call (a shard's part of a call must fit its
                               * batch_events_max, else the call fails with TBG_EINVAL) */
    uint32_t batch_count_max; /* max batches per shard call (<= every shard's batch_count_max) */
    uint32_t pulse_batch_max; /* batch_max.create_transfers: 8190 in production */
    uint32_t router_device;   /* the device router's GPU: device-buffer calls enter here */
    uint64_t router_account_capacity;  /* accounts ever created through the group */
    uint64_t router_transfer_capacity; /* transfer events ever routed (< 2^31) */
} tbg_group_options;

/* Opens `options->shards` HIP executors, shard s with shard_options[s] (its device, capacities),
 * the device router on options->router_device, and peer access between the router's GPU and
 * every shard's. A group of one shard passes every call straight to its executor. */
tbg_group* tbg_group_open(const tbg_group_options* options, const tbg_options* shard_options);
/* The shard operations of HIP executors (tbg_ctx*), for a group over executors the caller owns --
 * e.g. executors in other processes reached through the caller's transport (remote.py). */
void tbg_group_hip_shard_ops(tbg_shard_ops* out);
/* A group over executors the caller owns (`ops` applied to shards[s]): host directories and the
 * exact engine only (no device path); shard calls are made one at a time from the caller's
 * thread. */
tbg_group* tbg_group_open_shards(const tbg_group_options* options, const tbg_shard_ops* ops,
                                 void* const* shards);
/* Durability (StateMachine.checkpoint :2937-2958 / open :964-978, for a group): every shard
 * writes its image to paths[s] (tbg_checkpoint: tables, AccountEvents, pulse_next_timestamp, key
 * ranges), between calls; tbg_group_open_checkpoint opens each shard from paths[s]
 * (tbg_open_checkpoint) and rebuilds the router's directories from the shards' accounts and
 * transfer ids, orphaned ids included (tbg_dump_transfer_ids). Groups of HIP executors only
 * (tbg_group_open). */
int tbg_group_checkpoint(tbg_group* g, const char* const* paths);
tbg_group* tbg_group_open_checkpoint(const tbg_group_options* options,
                                     const tbg_options* shard_options, const char* const* paths);
void tbg_group_close(tbg_group* g);
const char* tbg_group_last_error(const tbg_group* g);
/* Shard s's executor (a tbg_ctx* for tbg_group_open, the caller's pointer otherwise): dumps,
 * AccountEvents and scans of the shard's own tables. */
void* tbg_group_shard(tbg_group* g, uint32_t s);

int tbg_group_create_accounts(tbg_group* g, const tb_account_t* events, uint32_t n,
                              const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                              uint32_t n_batches, tb_create_result_t* results);
int tbg_group_create_transfers(tbg_group* g, const tb_transfer_t* events, uint32_t n,
                               const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                               uint32_t n_batches, tb_create_result_t* results);
/* Device-buffer form (tbg_group_open only): every pointer is memory of the router's GPU,
 * batch_ends[b] = exclusive end of batch b; synchronous (results complete on return). */
int tbg_group_create_transfers_device(tbg_group* g, const tb_transfer_t* d_events, uint32_t n,
                                      const uint32_t* d_batch_ends,
                                      const uint64_t* d_batch_timestamps, uint32_t n_batches,
                                      tb_create_result_t* d_results);

int64_t tbg_group_pulse(tbg_group* g, uint64_t timestamp);
uint64_t tbg_group_pulse_next_timestamp(tbg_group* g);
/* Found objects only, in request order; returns the count written. */
int64_t tbg_group_lookup_accounts(tbg_group* g, const tb_uint128_t* ids, uint32_t n,
                                  tb_account_t* out);
int64_t tbg_group_lookup_transfers(tbg_group* g, const tb_uint128_t* ids, uint32_t n,
                                   tb_transfer_t* out);

/* Binds the group as a tb_executor (tb_state_machine.h: create_*, pulse, pulse_next_timestamp,
 * lookups; the scans and get_change_events merge the shards' answers by timestamp), so that
 * tb_sm_open(options, &executor) is the reference's StateMachine over N GPUs. */
void tbg_group_executor(tbg_group* g, tb_executor* out);

/* Counters since open (diagnostics / bench). */
typedef struct tbg_group_stats {
    uint64_t calls;            /* create_* calls */
    uint64_t device_calls;     /* create_transfers calls executed by the device path */
    uint64_t engine_calls;     /* calls executed by the exact engine */
    uint64_t segments;         /* segments the exact engine executed */
    uint64_t chain_segments;   /* of them linked chains across shards */
    uint64_t surrogates;       /* device-path events with a patched status (cross-shard accounts) */
    uint64_t anywhere;         /* device-path events whose status followed from themselves */
    uint64_t repeats;          /* device-path events repeating an id of the call */
    uint64_t route_ns;         /* device path, host wall time: routing (tbr_route_device) */
    uint64_t execute_ns;       /* ... the shards' slices (copies in, execution, copies out) */
    uint64_t settle_ns;        /* ... settle and the pulse_next_timestamp resolution */
    uint64_t engine_ns;        /* the exact engine's calls */
} tbg_group_stats;
int tbg_group_stats_read(tbg_group* g, tbg_group_stats* out);

/* Test hook: the exact engine's segments for a call planned against the current directories
 * without executing anything (every segment planned with the directories as they are).
 * seg_ends[i] = end of segment i, seg_flags[i] bit 0 = a linked chain across shards;
 * shard_of[k] = event k's shard. Returns the segment count (<= max_segments) or an error. */
int64_t tbg_group_plan(tbg_group* g, int transfers, const void* events, uint32_t n,
                       const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                       uint32_t n_batches, uint32_t* seg_ends, uint8_t* seg_flags,
                       int32_t* shard_of, uint32_t max_segments);
/* Test hook: records directory entries (accounts: id -> shard) as if created there. */
int tbg_group_record_accounts(tbg_group* g, const tb_uint128_t* ids, const uint8_t* shards,
                              uint32_t n);
int tbg_group_record_transfers(tbg_group* g, const tb_uint128_t* ids, const uint8_t* shards,
                               uint32_t n);

#ifdef __cplusplus
}
#endif

#endif /* TBG_GROUP_H */
