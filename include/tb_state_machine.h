/*
 * tb_state_machine.h -- the reference's StateMachine contract for the commit path, as a C ABI.
 *
 * Mirrors `StateMachineType(Storage)` (src/state_machine.zig:222-2958) as consumed by
 * `ReplicaType(StateMachine, ...)` (src/vsr/replica.zig:144-152) for the operations of this path:
 * pulse, create_accounts, create_transfers, lookup_accounts, lookup_transfers,
 * get_change_events (the account_events groove's reader, CDC) and the scans over the same tables:
 * get_account_transfers, get_account_balances, query_accounts, query_transfers -- and their
 * deprecated encodings (the unbatched bodies and the sparse create results older clients send,
 * execute :2671-2700, execute_create :3116-3194). Bodies are multi-batch encoded exactly as
 * src/vsr/multi_batch.zig; replies are multi-batch encoded the same way. The executor underneath is pluggable (tb_executor): the product binds the HIP
 * executor (tbg.h) with tb_sm_open_gpu; tests may bind another executor with the same semantics.
 *
 *   tb_sm_input_valid     <- StateMachine.input_valid   :980-1032 (+ batch_valid :1036-1067)
 *   tb_sm_event_max / tb_sm_result_max <- Operation.event_max / result_max
 *                            (src/tigerbeetle.zig:853-931) under the bound message_body_size_max
 *   tb_sm_prepare         <- StateMachine.prepare       :1070-1101
 *   tb_sm_pulse_needed    <- StateMachine.pulse_needed  :1138-1144
 *   tb_sm_prefetch        <- StateMachine.prefetch      :1146-1226 (completes immediately:
 *                            the tables are HBM-resident; the callback runs before return)
 *   tb_sm_commit          <- StateMachine.commit        :2564-2669 / execute_multi_batch :2702
 *   tb_sm_compact         <- StateMachine.compact       :2912-2935 (the HIP executor's tables
 *                            are compacted at the last op of each bar, TB_SM_COMPACTION_OPS)
 *   tb_sm_checkpoint      <- StateMachine.checkpoint    :2937-2958 (an image of the tables)
 *   tb_sm_open_gpu_checkpoint <- StateMachine.open      :964-978 (tables loaded from an image)
 *   tb_sm_{get,set}_*_timestamp <- fields prepare_timestamp / commit_timestamp /
 *                            prefetch_timestamp (:229-231), written by the replica.
 */
#ifndef TB_STATE_MACHINE_H
#define TB_STATE_MACHINE_H

#include "tb_types.h"
#include "tbg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Operation numbers (src/tigerbeetle.zig:685-716, vsr_operations_reserved = 128): every operation
 * of the reference's StateMachine, the deprecated encodings included (older clients). */
enum {
    TB_OPERATION_PULSE = 128,
    TB_OPERATION_DEPRECATED_CREATE_ACCOUNTS_UNBATCHED = 129,
    TB_OPERATION_DEPRECATED_CREATE_TRANSFERS_UNBATCHED = 130,
    TB_OPERATION_DEPRECATED_LOOKUP_ACCOUNTS_UNBATCHED = 131,
    TB_OPERATION_DEPRECATED_LOOKUP_TRANSFERS_UNBATCHED = 132,
    TB_OPERATION_DEPRECATED_GET_ACCOUNT_TRANSFERS_UNBATCHED = 133,
    TB_OPERATION_DEPRECATED_GET_ACCOUNT_BALANCES_UNBATCHED = 134,
    TB_OPERATION_DEPRECATED_QUERY_ACCOUNTS_UNBATCHED = 135,
    TB_OPERATION_DEPRECATED_QUERY_TRANSFERS_UNBATCHED = 136,
    TB_OPERATION_GET_CHANGE_EVENTS = 137,
    TB_OPERATION_DEPRECATED_CREATE_ACCOUNTS_SPARSE = 138,
    TB_OPERATION_DEPRECATED_CREATE_TRANSFERS_SPARSE = 139,
    TB_OPERATION_LOOKUP_ACCOUNTS = 140,
    TB_OPERATION_LOOKUP_TRANSFERS = 141,
    TB_OPERATION_GET_ACCOUNT_TRANSFERS = 142,
    TB_OPERATION_GET_ACCOUNT_BALANCES = 143,
    TB_OPERATION_QUERY_ACCOUNTS = 144,
    TB_OPERATION_QUERY_TRANSFERS = 145,
    TB_OPERATION_CREATE_ACCOUNTS = 146,
    TB_OPERATION_CREATE_TRANSFERS = 147,
};

/* An executor of the path: create_* take all batches of one commit. */
typedef struct tb_executor {
    void* self;
    int (*create_accounts)(void* self, const tb_account_t* events, uint32_t n,
                           const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                           uint32_t n_batches, tb_create_result_t* results);
    int (*create_transfers)(void* self, const tb_transfer_t* events, uint32_t n,
                            const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                            uint32_t n_batches, tb_create_result_t* results);
    int64_t (*pulse)(void* self, uint64_t timestamp);
    uint64_t (*pulse_next_timestamp)(void* self);
    int64_t (*lookup_accounts)(void* self, const tb_uint128_t* ids, uint32_t n, tb_account_t* out);
    int64_t (*lookup_transfers)(void* self, const tb_uint128_t* ids, uint32_t n,
                                tb_transfer_t* out);
    /* ChangeEvents of the filter, at most min(filter->limit, limit_max); 0 if invalid. */
    int64_t (*get_change_events)(void* self, const tb_change_events_filter_t* filter,
                                 uint32_t limit_max, tb_change_event_t* out);
    /* The scans of one filter, at most min(filter->limit, limit_max) results; 0 if invalid. */
    int64_t (*get_account_transfers)(void* self, const tb_account_filter_t* filter,
                                     uint32_t limit_max, tb_transfer_t* out);
    int64_t (*get_account_balances)(void* self, const tb_account_filter_t* filter,
                                    uint32_t limit_max, tb_account_balance_t* out);
    int64_t (*query_accounts)(void* self, const tb_query_filter_t* filter, uint32_t limit_max,
                              tb_account_t* out);
    int64_t (*query_transfers)(void* self, const tb_query_filter_t* filter, uint32_t limit_max,
                               tb_transfer_t* out);
} tb_executor;

typedef struct tb_sm tb_sm;

typedef struct tb_sm_options {
    uint32_t batch_size_limit;      /* Options.batch_size_limit (<= message_body_size_max) */
    uint32_t message_body_size_max; /* constants.message_body_size_max (1 MiB - 256 in prod) */
    uint32_t pulse_batch_max;       /* batch_max.create_transfers (prepare delta of a pulse) */
} tb_sm_options;

/* Binds an executor (copied). */
tb_sm* tb_sm_open(const tb_sm_options* options, const tb_executor* executor);
/* Opens the HIP executor (tbg_open) and binds it; the tb_sm owns it. */
tb_sm* tb_sm_open_gpu(const tb_sm_options* options, const tbg_options* executor_options);
/* Opens the HIP executor from a checkpoint image (tbg_open_checkpoint) and binds it. */
tb_sm* tb_sm_open_gpu_checkpoint(const tb_sm_options* options,
                                 const tbg_options* executor_options, const char* path);
void tb_sm_close(tb_sm* sm);
/* The bound HIP executor of a tb_sm_open_gpu state machine (NULL otherwise). */
tbg_ctx* tb_sm_executor_gpu(tb_sm* sm);
/* Registers a host buffer the replica passes as bodies or reply outputs (its message pool) with
 * the HIP executor (tbg_register_host): page-locked and mapped, so the executor's kernels read a
 * body and write a reply over PCIe on the call's stream, with no DMA-engine hand-off; a no-op
 * returning 0 for another executor. */
int tb_sm_register_buffer(tb_sm* sm, void* ptr, uint64_t size);

int tb_sm_input_valid(const tb_sm* sm, uint8_t operation, const void* body, uint32_t size);
/* Operation.event_max / result_max (tigerbeetle.zig:853-931) for this state machine's
 * message_body_size_max; 0 for pulse, an unknown operation or a batch_size_limit outside
 * (0, message_body_size_max]. */
uint32_t tb_sm_event_max(const tb_sm* sm, uint8_t operation, uint32_t batch_size_limit);
uint32_t tb_sm_result_max(const tb_sm* sm, uint8_t operation, uint32_t batch_size_limit);
void tb_sm_prepare(tb_sm* sm, uint8_t operation, const void* body, uint32_t size);
int tb_sm_pulse_needed(const tb_sm* sm, uint64_t timestamp);

typedef void (*tb_sm_prefetch_callback)(void* context);
void tb_sm_prefetch(tb_sm* sm, tb_sm_prefetch_callback callback, void* context, uint64_t op,
                    uint64_t snapshot, uint8_t operation, const void* body, uint32_t size);

/* Returns the reply size in bytes written to `output` (>= message_body_size_max bytes), or a
 * negative value on executor failure. `client` is u128 {lo, hi}; client == 0 only for pulse. */
int64_t tb_sm_commit(tb_sm* sm, uint64_t client_lo, uint64_t client_hi, uint64_t op,
                     uint64_t timestamp, uint8_t operation, const void* body, uint32_t size,
                     void* output);

/* Ops per bar (constants.lsm_compaction_ops, src/constants.zig:647; 32 in the production
 * config): the LSM spreads a bar's compaction over its ops, the executor compacts its transfer
 * store (tbg_compact) at the bar's last op. Returns 0 or a negative executor error. */
#define TB_SM_COMPACTION_OPS 32
int tb_sm_compact(tb_sm* sm, uint64_t op);
/* Writes the executor's checkpoint image to `path` (tbg_checkpoint); -22 for a non-HIP executor. */
int tb_sm_checkpoint(tb_sm* sm, const char* path);

uint64_t tb_sm_get_prepare_timestamp(const tb_sm* sm);
uint64_t tb_sm_get_commit_timestamp(const tb_sm* sm);
uint64_t tb_sm_get_prefetch_timestamp(const tb_sm* sm);
void tb_sm_set_prepare_timestamp(tb_sm* sm, uint64_t v);
void tb_sm_set_commit_timestamp(tb_sm* sm, uint64_t v);
void tb_sm_set_prefetch_timestamp(tb_sm* sm, uint64_t v);

/* Multi-batch codec (src/vsr/multi_batch.zig), exported for clients/tests.
 * encode: writes the payload of `n_batches` batches (element counts `counts`) laid out
 * contiguously in `buffer` followed by the trailer; returns the total body size.
 * decode: returns the batch count (>0) and fills counts[] (capacity `counts_max`) and
 * *payload_size; returns -1 if the body is not a valid multi-batch encoding. */
int64_t tb_multi_batch_encode_trailer(void* buffer, uint32_t payload_size, uint32_t element_size,
                                      const uint16_t* counts, uint32_t n_batches);
int64_t tb_multi_batch_decode(const void* body, uint32_t size, uint32_t element_size,
                              uint16_t* counts, uint32_t counts_max, uint32_t* payload_size);
uint32_t tb_multi_batch_trailer_total_size(uint32_t element_size, uint32_t batch_count);

#ifdef __cplusplus
}
#endif

#endif /* TB_STATE_MACHINE_H */
