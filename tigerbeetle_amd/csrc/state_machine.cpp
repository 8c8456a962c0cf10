// StateMachine mirror for the commit path (include/tb_state_machine.h).
//
// Restates the host-side control of src/state_machine.zig for the operations of this path:
// input_valid / batch_valid (:980-1067), prepare / prepare_delta_nanoseconds (:1070-1136),
// pulse_needed (:1138-1144), prefetch (:1146-1226; a no-op here), commit (:2564-2669) and
// execute_multi_batch (:2702-2762), plus the multi-batch codec (src/vsr/multi_batch.zig). The
// per-event work is delegated to a tb_executor: the HIP executor (tbg.h) in production.

#include "../../include/tb_state_machine.h"

#include <algorithm>
#include <chrono>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

namespace {

constexpr uint16_t kBatchCountMax = 0xFFFF - 1;  // Postamble.batch_count_max
constexpr uint16_t kTrailerPadding = 0xFFFF;      // TrailerItem.padding

uint32_t div_ceil(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

// Operation's comptime facts (src/tigerbeetle.zig:717-849): EventType / ResultType sizes,
// is_batchable, is_multi_batch.
struct OperationInfo {
    uint32_t event_size;
    uint32_t result_size;
    bool batchable;
    bool multi_batch;
};

bool operation_info(uint8_t operation, OperationInfo* info) {
    switch (operation) {
        case TB_OPERATION_PULSE: *info = {0, 0, false, false}; return true;
        case TB_OPERATION_DEPRECATED_CREATE_ACCOUNTS_UNBATCHED:
        case TB_OPERATION_DEPRECATED_CREATE_TRANSFERS_UNBATCHED:
            *info = {128, 8, true, false}; return true;
        case TB_OPERATION_DEPRECATED_LOOKUP_ACCOUNTS_UNBATCHED:
        case TB_OPERATION_DEPRECATED_LOOKUP_TRANSFERS_UNBATCHED:
            *info = {16, 128, true, false}; return true;
        case TB_OPERATION_DEPRECATED_GET_ACCOUNT_TRANSFERS_UNBATCHED:
        case TB_OPERATION_DEPRECATED_GET_ACCOUNT_BALANCES_UNBATCHED:
            *info = {128, 128, false, false}; return true;
        case TB_OPERATION_DEPRECATED_QUERY_ACCOUNTS_UNBATCHED:
        case TB_OPERATION_DEPRECATED_QUERY_TRANSFERS_UNBATCHED:
            *info = {64, 128, false, false}; return true;
        case TB_OPERATION_GET_CHANGE_EVENTS: *info = {64, 384, false, false}; return true;
        case TB_OPERATION_DEPRECATED_CREATE_ACCOUNTS_SPARSE:
        case TB_OPERATION_DEPRECATED_CREATE_TRANSFERS_SPARSE:
            *info = {128, 8, true, true}; return true;
        case TB_OPERATION_LOOKUP_ACCOUNTS:
        case TB_OPERATION_LOOKUP_TRANSFERS: *info = {16, 128, true, true}; return true;
        case TB_OPERATION_GET_ACCOUNT_TRANSFERS:
        case TB_OPERATION_GET_ACCOUNT_BALANCES: *info = {128, 128, false, true}; return true;
        case TB_OPERATION_QUERY_ACCOUNTS:
        case TB_OPERATION_QUERY_TRANSFERS: *info = {64, 128, false, true}; return true;
        case TB_OPERATION_CREATE_ACCOUNTS:
        case TB_OPERATION_CREATE_TRANSFERS: *info = {128, 16, true, true}; return true;
        default: return false;
    }
}

bool is_create(uint8_t operation) {
    switch (operation) {
        case TB_OPERATION_CREATE_ACCOUNTS:
        case TB_OPERATION_CREATE_TRANSFERS:
        case TB_OPERATION_DEPRECATED_CREATE_ACCOUNTS_SPARSE:
        case TB_OPERATION_DEPRECATED_CREATE_TRANSFERS_SPARSE:
        case TB_OPERATION_DEPRECATED_CREATE_ACCOUNTS_UNBATCHED:
        case TB_OPERATION_DEPRECATED_CREATE_TRANSFERS_UNBATCHED: return true;
        default: return false;
    }
}

bool creates_accounts(uint8_t operation) {
    return operation == TB_OPERATION_CREATE_ACCOUNTS ||
           operation == TB_OPERATION_DEPRECATED_CREATE_ACCOUNTS_SPARSE ||
           operation == TB_OPERATION_DEPRECATED_CREATE_ACCOUNTS_UNBATCHED;
}

// A query filter's `limit` (Operation.result_count_expected, tigerbeetle.zig:966-990): the
// AccountFilter, QueryFilter or ChangeEventsFilter of the (non-batchable) operation.
uint32_t filter_limit(uint8_t operation, const uint8_t* filter) {
    uint32_t limit = 0;
    size_t at = offsetof(tb_account_filter_t, limit);
    if (operation == TB_OPERATION_QUERY_ACCOUNTS || operation == TB_OPERATION_QUERY_TRANSFERS ||
        operation == TB_OPERATION_DEPRECATED_QUERY_ACCOUNTS_UNBATCHED ||
        operation == TB_OPERATION_DEPRECATED_QUERY_TRANSFERS_UNBATCHED)
        at = offsetof(tb_query_filter_t, limit);
    if (operation == TB_OPERATION_GET_CHANGE_EVENTS) at = offsetof(tb_change_events_filter_t, limit);
    std::memcpy(&limit, filter + at, 4);
    return limit;
}

}  // namespace

extern "C" uint32_t tb_multi_batch_trailer_total_size(uint32_t element_size,
                                                      uint32_t batch_count) {
    // multi_batch.zig:101-118
    uint32_t unpadded = batch_count * 2 + 2;
    if (element_size == 0) return unpadded;
    return div_ceil(unpadded, element_size) * element_size;
}

extern "C" int64_t tb_multi_batch_decode(const void* body_, uint32_t size, uint32_t element_size,
                                         uint16_t* counts, uint32_t counts_max,
                                         uint32_t* payload_size) {
    // MultiBatchDecoder.init, multi_batch.zig:135-230. Parses suffixes from the end.
    const uint8_t* body = static_cast<const uint8_t*>(body_);
    if (size < 2 || (reinterpret_cast<uintptr_t>(body + size - 2) & 1u)) return -1;
    uint16_t batch_count;
    std::memcpy(&batch_count, body + size - 2, 2);
    if (batch_count == 0 || batch_count > kBatchCountMax) return -1;
    uint32_t trailer_size = tb_multi_batch_trailer_total_size(element_size, batch_count);
    uint32_t items_size = uint32_t(batch_count) * 2;
    if (size < 2 + items_size) return -1;
    if (trailer_size > size) return -1;
    // Padding between the used items and the start of the trailer must be all 0xFF.
    uint32_t padding_size = trailer_size - 2 - items_size;
    const uint8_t* trailer = body + size - trailer_size;
    for (uint32_t i = 0; i < padding_size; i++)
        if (trailer[i] != 0xFF) return -1;
    const uint8_t* items = body + size - 2 - items_size;
    uint64_t total = 0;
    if (counts_max < batch_count) return -1;
    for (uint32_t b = 0; b < batch_count; b++) {
        // The last item corresponds to the first batch.
        uint16_t c;
        std::memcpy(&c, items + (uint32_t(batch_count) - 1 - b) * 2, 2);
        if (c == kTrailerPadding) return -1;
        counts[b] = c;
        total += c;
    }
    if (element_size == 0 && total != 0) return -1;
    uint64_t payload = total * element_size;
    if (payload > 0xFFFFFFFFull) return -1;
    uint32_t trailer_pad = uint32_t(payload % 2);  // only for 1-byte elements
    if (trailer_pad) {
        if (size < trailer_size + trailer_pad) return -1;
        if (body[size - trailer_size - 1] != 0xFF) return -1;
    }
    if (payload != uint64_t(size) - trailer_size - trailer_pad) return -1;
    *payload_size = uint32_t(payload);
    return batch_count;
}

extern "C" int64_t tb_multi_batch_encode_trailer(void* buffer_, uint32_t payload_size,
                                                 uint32_t element_size, const uint16_t* counts,
                                                 uint32_t n_batches) {
    // MultiBatchEncoder.finish, multi_batch.zig:428-490.
    if (n_batches == 0 || n_batches > kBatchCountMax) return -1;
    uint8_t* buffer = static_cast<uint8_t*>(buffer_);
    uint32_t padding = payload_size % 2;
    if (padding) buffer[payload_size] = 0xFF;
    uint32_t trailer_size = tb_multi_batch_trailer_total_size(element_size, n_batches);
    uint8_t* trailer = buffer + payload_size + padding;
    uint32_t items = (trailer_size - 2) / 2;
    for (uint32_t i = 0; i < items - n_batches; i++)
        std::memcpy(trailer + i * 2, &kTrailerPadding, 2);
    for (uint32_t b = 0; b < n_batches; b++) {
        uint16_t c = counts[b];
        std::memcpy(trailer + (items - 1 - b) * 2, &c, 2);
    }
    uint16_t bc = uint16_t(n_batches);
    std::memcpy(trailer + trailer_size - 2, &bc, 2);
    return int64_t(payload_size) + padding + trailer_size;
}

struct tb_sm {
    tb_sm_options options;
    tb_executor executor;
    tbg_ctx* gpu = nullptr;  // owned when opened with tb_sm_open_gpu

    uint64_t prepare_timestamp = 0;
    uint64_t commit_timestamp = 0;
    uint64_t prefetch_timestamp = 0;

    std::vector<uint16_t> counts;
    std::vector<uint32_t> lens;
    std::vector<uint64_t> batch_ts;
    std::vector<tb_create_result_t> results;

    // Operation.event_max (src/tigerbeetle.zig:853-901).
    uint32_t event_max(const OperationInfo& info, uint32_t batch_size_limit) const {
        const uint32_t mbsm = options.message_body_size_max;
        if (!info.multi_batch) {
            return info.event_size == 0 ? mbsm / info.result_size
                                        : std::min(batch_size_limit / info.event_size,
                                                   mbsm / info.result_size);
        }
        const uint32_t reply_trailer_min = tb_multi_batch_trailer_total_size(info.result_size, 1);
        if (info.event_size == 0) return (mbsm - reply_trailer_min) / info.result_size;
        const uint32_t request_trailer_min = tb_multi_batch_trailer_total_size(info.event_size, 1);
        return std::min((batch_size_limit - request_trailer_min) / info.event_size,
                        (mbsm - reply_trailer_min) / info.result_size);
    }

    // Operation.result_max (tigerbeetle.zig:907-931).
    uint32_t result_max(const OperationInfo& info, uint32_t batch_size_limit) const {
        if (info.batchable) return event_max(info, batch_size_limit);
        const uint32_t mbsm = options.message_body_size_max;
        if (!info.multi_batch) return mbsm / info.result_size;
        return (mbsm - tb_multi_batch_trailer_total_size(info.result_size, 1)) / info.result_size;
    }

    // StateMachine.batch_valid (state_machine.zig:1036-1067): one (decoded) batch.
    bool batch_valid(uint8_t operation, const OperationInfo& info, uint32_t batch_size) const {
        if (operation == TB_OPERATION_PULSE) return batch_size == 0;
        if (!info.batchable) return batch_size == info.event_size;
        if (batch_size % info.event_size != 0) return false;
        return batch_size / info.event_size <= event_max(info, options.batch_size_limit);
    }

    // prepare_delta_nanoseconds (:1106-1136): the logical time one batch advances.
    uint64_t prepare_delta(uint8_t operation, uint32_t batch_size) const {
        if (operation == TB_OPERATION_PULSE) return options.pulse_batch_max;
        return is_create(operation) ? batch_size / 128u : 0;
    }
};

namespace {

int gpu_create_accounts(void* self, const tb_account_t* e, uint32_t n, const uint32_t* lens,
                        const uint64_t* ts, uint32_t nb, tb_create_result_t* r) {
    return tbg_create_accounts(static_cast<tbg_ctx*>(self), e, n, lens, ts, nb, r);
}
int gpu_create_transfers(void* self, const tb_transfer_t* e, uint32_t n, const uint32_t* lens,
                         const uint64_t* ts, uint32_t nb, tb_create_result_t* r) {
    return tbg_create_transfers(static_cast<tbg_ctx*>(self), e, n, lens, ts, nb, r);
}
int64_t gpu_pulse(void* self, uint64_t ts) { return tbg_pulse(static_cast<tbg_ctx*>(self), ts); }
uint64_t gpu_pulse_next(void* self) {
    return tbg_pulse_next_timestamp(static_cast<tbg_ctx*>(self));
}
int64_t gpu_lookup_accounts(void* self, const tb_uint128_t* ids, uint32_t n, tb_account_t* out) {
    return tbg_lookup_accounts(static_cast<tbg_ctx*>(self), ids, n, out);
}
int64_t gpu_lookup_transfers(void* self, const tb_uint128_t* ids, uint32_t n,
                             tb_transfer_t* out) {
    return tbg_lookup_transfers(static_cast<tbg_ctx*>(self), ids, n, out);
}
int64_t gpu_get_change_events(void* self, const tb_change_events_filter_t* filter,
                              uint32_t limit_max, tb_change_event_t* out) {
    return tbg_get_change_events(static_cast<tbg_ctx*>(self), filter, limit_max, out);
}
int64_t gpu_get_account_transfers(void* self, const tb_account_filter_t* f, uint32_t m,
                                  tb_transfer_t* out) {
    return tbg_get_account_transfers(static_cast<tbg_ctx*>(self), f, m, out);
}
int64_t gpu_get_account_balances(void* self, const tb_account_filter_t* f, uint32_t m,
                                 tb_account_balance_t* out) {
    return tbg_get_account_balances(static_cast<tbg_ctx*>(self), f, m, out);
}
int64_t gpu_query_accounts(void* self, const tb_query_filter_t* f, uint32_t m, tb_account_t* out) {
    return tbg_query_accounts(static_cast<tbg_ctx*>(self), f, m, out);
}
int64_t gpu_query_transfers(void* self, const tb_query_filter_t* f, uint32_t m,
                            tb_transfer_t* out) {
    return tbg_query_transfers(static_cast<tbg_ctx*>(self), f, m, out);
}

}  // namespace

extern "C" tb_sm* tb_sm_open(const tb_sm_options* options, const tb_executor* executor) {
    if (!options || !executor) return nullptr;
    if (options->batch_size_limit == 0 || options->batch_size_limit > options->message_body_size_max)
        return nullptr;
    tb_sm* sm = new (std::nothrow) tb_sm();
    if (!sm) return nullptr;
    sm->options = *options;
    sm->executor = *executor;
    return sm;
}

namespace {
tb_sm* bind_gpu(const tb_sm_options* options, tbg_ctx* ctx) {
    if (!ctx) return nullptr;
    tb_executor ex;
    ex.self = ctx;
    ex.create_accounts = gpu_create_accounts;
    ex.create_transfers = gpu_create_transfers;
    ex.pulse = gpu_pulse;
    ex.pulse_next_timestamp = gpu_pulse_next;
    ex.lookup_accounts = gpu_lookup_accounts;
    ex.lookup_transfers = gpu_lookup_transfers;
    ex.get_change_events = gpu_get_change_events;
    ex.get_account_transfers = gpu_get_account_transfers;
    ex.get_account_balances = gpu_get_account_balances;
    ex.query_accounts = gpu_query_accounts;
    ex.query_transfers = gpu_query_transfers;
    tb_sm* sm = tb_sm_open(options, &ex);
    if (!sm) {
        tbg_close(ctx);
        return nullptr;
    }
    sm->gpu = ctx;
    return sm;
}
}  // namespace

extern "C" tb_sm* tb_sm_open_gpu(const tb_sm_options* options, const tbg_options* executor_options) {
    return bind_gpu(options, tbg_open(executor_options));
}

extern "C" tb_sm* tb_sm_open_gpu_checkpoint(const tb_sm_options* options,
                                            const tbg_options* executor_options, const char* path) {
    return bind_gpu(options, tbg_open_checkpoint(executor_options, path));
}

extern "C" int tb_sm_compact(tb_sm* sm, uint64_t op) {
    if (!sm) return TBG_EINVAL;
    if (!sm->gpu || (op + 1) % TB_SM_COMPACTION_OPS != 0) return 0;
    const int64_t rc = tbg_compact(sm->gpu);
    return rc < 0 ? int(rc) : 0;
}

extern "C" int tb_sm_checkpoint(tb_sm* sm, const char* path) {
    if (!sm || !sm->gpu) return TBG_EINVAL;
    return tbg_checkpoint(sm->gpu, path);
}

extern "C" void tb_sm_close(tb_sm* sm) {
    if (!sm) return;
    if (sm->gpu) tbg_close(sm->gpu);
    delete sm;
}

extern "C" tbg_ctx* tb_sm_executor_gpu(tb_sm* sm) { return sm ? sm->gpu : nullptr; }

extern "C" int tb_sm_register_buffer(tb_sm* sm, void* ptr, uint64_t size) {
    if (!sm) return TBG_EINVAL;
    return sm->gpu ? tbg_register_host(sm->gpu, ptr, size) : 0;
}

extern "C" uint32_t tb_sm_event_max(const tb_sm* sm, uint8_t operation, uint32_t batch_size_limit) {
    OperationInfo info;
    if (!sm || !operation_info(operation, &info) || info.result_size == 0) return 0;
    if (batch_size_limit == 0 || batch_size_limit > sm->options.message_body_size_max) return 0;
    return sm->event_max(info, batch_size_limit);
}

extern "C" uint32_t tb_sm_result_max(const tb_sm* sm, uint8_t operation, uint32_t batch_size_limit) {
    OperationInfo info;
    if (!sm || !operation_info(operation, &info) || info.result_size == 0) return 0;
    if (batch_size_limit == 0 || batch_size_limit > sm->options.message_body_size_max) return 0;
    return sm->result_max(info, batch_size_limit);
}

extern "C" int tb_sm_input_valid(const tb_sm* sm, uint8_t operation, const void* body,
                                 uint32_t size) {
    // StateMachine.input_valid (:980-1032). The reference asserts size <= batch_size_limit (the
    // replica checked it); here an oversize body is simply invalid.
    OperationInfo info;
    if (!operation_info(operation, &info)) return 0;
    if (size > sm->options.batch_size_limit) return 0;
    if (!info.multi_batch) return sm->batch_valid(operation, info, size) ? 1 : 0;

    std::vector<uint16_t> counts(kBatchCountMax);
    uint32_t payload = 0;
    int64_t nb = tb_multi_batch_decode(body, size, info.event_size, counts.data(),
                                       uint32_t(counts.size()), &payload);
    if (nb <= 0) return 0;
    uint64_t result_count_expected = 0;
    // Replies are not constrained by the runtime batch_size_limit (:1013-1017).
    const uint32_t result_max = sm->result_max(info, sm->options.message_body_size_max);
    const uint8_t* batch = static_cast<const uint8_t*>(body);
    for (int64_t b = 0; b < nb; b++) {
        const uint32_t batch_size = uint32_t(counts[b]) * info.event_size;
        if (!sm->batch_valid(operation, info, batch_size)) return 0;
        // Operation.result_count_expected (tigerbeetle.zig:936-992): one result per event, or
        // up to the filter's limit.
        const uint32_t expected = info.batchable ? counts[b] : filter_limit(operation, batch);
        result_count_expected += std::min<uint32_t>(expected, result_max);
        batch += batch_size;
    }
    uint64_t reply_trailer = tb_multi_batch_trailer_total_size(info.result_size, uint32_t(nb));
    if (sm->options.message_body_size_max < result_count_expected * info.result_size + reply_trailer)
        return 0;
    return 1;
}

extern "C" void tb_sm_prepare(tb_sm* sm, uint8_t operation, const void* body, uint32_t size) {
    // StateMachine.prepare (:1070-1101): the sum of the batches' deltas.
    OperationInfo info;
    if (!operation_info(operation, &info)) return;
    uint64_t delta = 0;
    if (!info.multi_batch) {
        delta = sm->prepare_delta(operation, size);
    } else {
        uint32_t payload = 0;
        sm->counts.resize(kBatchCountMax);
        int64_t nb = tb_multi_batch_decode(body, size, info.event_size, sm->counts.data(),
                                           uint32_t(sm->counts.size()), &payload);
        for (int64_t b = 0; b < nb; b++)
            delta += sm->prepare_delta(operation, uint32_t(sm->counts[b]) * info.event_size);
    }
    sm->prepare_timestamp += delta;
}

extern "C" int tb_sm_pulse_needed(const tb_sm* sm, uint64_t timestamp) {
    return sm->executor.pulse_next_timestamp(sm->executor.self) <= timestamp;
}

extern "C" void tb_sm_prefetch(tb_sm* sm, tb_sm_prefetch_callback callback, void* context,
                               uint64_t op, uint64_t snapshot, uint8_t operation,
                               const void* body, uint32_t size) {
    (void)sm;
    (void)op;
    (void)snapshot;
    (void)operation;
    (void)body;
    (void)size;
    // Every table is resident in HBM: nothing is staged. (The body itself is read by the commit's
    // create kernel across PCIe from the registered message pool; a copy started here measured
    // slower back to back with the commit -- DESIGN.md §13.)
    if (callback) callback(context);
}

namespace {

// The sparse results of the deprecated create operations (CreateAccountErrorResult /
// CreateTransferErrorResult, tigerbeetle.zig:496-515): execute_create (:3116-3194) appends
// {index, status} for every event whose final status is not `created` -- a broken chain's earlier
// events (linked_event_failed) are appended, in order, before the event that broke it -- which is
// the dense results' non-created entries in index order. Returns the bytes written.
uint32_t sparse_results(const tb_create_result_t* dense, uint32_t n, uint8_t* out) {
    uint32_t count = 0;
    for (uint32_t i = 0; i < n; i++) {
        if (dense[i].status == TB_STATUS_CREATED) continue;
        const uint32_t entry[2] = {i, dense[i].status};
        std::memcpy(out + 8u * count, entry, 8);
        count++;
    }
    return 8u * count;
}

// One query filter's scan through the executor: results written to `dst`, their count returned
// (at most min(filter.limit, limit_max); 0 for an invalid filter).
int64_t execute_scan(const tb_executor& ex, uint8_t operation, const uint8_t* filter,
                     uint32_t limit_max, void* dst) {
    switch (operation) {
        case TB_OPERATION_GET_ACCOUNT_TRANSFERS:
        case TB_OPERATION_DEPRECATED_GET_ACCOUNT_TRANSFERS_UNBATCHED:
            return ex.get_account_transfers(ex.self,
                                            reinterpret_cast<const tb_account_filter_t*>(filter),
                                            limit_max, static_cast<tb_transfer_t*>(dst));
        case TB_OPERATION_GET_ACCOUNT_BALANCES:
        case TB_OPERATION_DEPRECATED_GET_ACCOUNT_BALANCES_UNBATCHED:
            return ex.get_account_balances(ex.self,
                                           reinterpret_cast<const tb_account_filter_t*>(filter),
                                           limit_max, static_cast<tb_account_balance_t*>(dst));
        case TB_OPERATION_QUERY_ACCOUNTS:
        case TB_OPERATION_DEPRECATED_QUERY_ACCOUNTS_UNBATCHED:
            return ex.query_accounts(ex.self, reinterpret_cast<const tb_query_filter_t*>(filter),
                                     limit_max, static_cast<tb_account_t*>(dst));
        default:
            return ex.query_transfers(ex.self, reinterpret_cast<const tb_query_filter_t*>(filter),
                                      limit_max, static_cast<tb_transfer_t*>(dst));
    }
}

}  // namespace

extern "C" int64_t tb_sm_commit(tb_sm* sm, uint64_t client_lo, uint64_t client_hi, uint64_t op,
                                uint64_t timestamp, uint8_t operation, const void* body,
                                uint32_t size, void* output) {
    (void)client_lo;
    (void)client_hi;
    (void)op;
    OperationInfo info;
    if (!operation_info(operation, &info)) return TBG_EINVAL;
    const tb_executor& ex = sm->executor;
    uint8_t* out = static_cast<uint8_t*>(output);
    if (operation == TB_OPERATION_PULSE) {
        // execute_expire_pending_transfers (:4511-4628): scans with expires_at_max =
        // prefetch_timestamp (:2463); no output.
        int64_t expired = ex.pulse(ex.self, timestamp);
        if (expired < 0) return expired;
        if (expired > 0) sm->commit_timestamp = timestamp;
        return 0;
    }

    if (operation == TB_OPERATION_GET_CHANGE_EVENTS) {
        // execute_query(.get_change_events) (:2770-2800, :3395-3422): not multi-batch; the scan
        // limit is capped by the reply size and the prefetches available per scanned result
        // (prefetch_get_change_events_scan, :2232-2265): transfers, and 2 accounts per event.
        if (size != sizeof(tb_change_events_filter_t) || !ex.get_change_events) return TBG_EINVAL;
        tb_change_events_filter_t filter;
        std::memcpy(&filter, body, sizeof(filter));
        const OperationInfo lookup{16, 128, true, false};  // deprecated_lookup_*_unbatched
        const uint32_t prefetch = sm->event_max(lookup, sm->options.batch_size_limit);
        const uint32_t limit_max = std::min({sm->options.message_body_size_max / 384u, prefetch,
                                             prefetch / 2});
        if (limit_max == 0) return 0;
        int64_t count = ex.get_change_events(ex.self, &filter, limit_max,
                                             static_cast<tb_change_event_t*>(output));
        return count < 0 ? count : count * int64_t(sizeof(tb_change_event_t));
    }

    // The batches of the body: the multi-batch decoding, or the whole body as one batch for the
    // deprecated unbatched operations (execute, :2671-2700; execute_query, :2764-2821).
    uint32_t payload = size;
    int64_t nb = 1;
    sm->counts.resize(kBatchCountMax);
    if (info.multi_batch) {
        nb = tb_multi_batch_decode(body, size, info.event_size, sm->counts.data(),
                                   uint32_t(sm->counts.size()), &payload);
        if (nb <= 0) return TBG_EINVAL;
    } else {
        if (size % info.event_size != 0 || (!info.batchable && size != info.event_size))
            return TBG_EINVAL;
        sm->counts[0] = uint16_t(size / info.event_size);
    }
    const uint32_t n = payload / info.event_size;

    if (is_create(operation)) {
        // execute_multi_batch: execute_timestamp starts at timestamp - delta(payload) and each
        // batch advances it by its own delta before executing (:2717-2737); an unbatched body
        // is one batch stamped `timestamp` (execute, :2671-2700).
        sm->lens.resize(size_t(nb));
        sm->batch_ts.resize(size_t(nb));
        uint64_t execute_timestamp = timestamp - n;
        for (int64_t b = 0; b < nb; b++) {
            sm->lens[b] = sm->counts[b];
            execute_timestamp += sm->counts[b];
            sm->batch_ts[b] = execute_timestamp;
        }
        const bool dense = info.result_size == sizeof(tb_create_result_t);
        tb_create_result_t* results = reinterpret_cast<tb_create_result_t*>(out);
        if (!dense) {
            sm->results.resize(n);
            results = sm->results.data();
        }
        int rc = n == 0 ? 0
                 : creates_accounts(operation)
                     ? ex.create_accounts(ex.self, static_cast<const tb_account_t*>(body), n,
                                          sm->lens.data(), sm->batch_ts.data(), uint32_t(nb),
                                          results)
                     : ex.create_transfers(ex.self, static_cast<const tb_transfer_t*>(body), n,
                                           sm->lens.data(), sm->batch_ts.data(), uint32_t(nb),
                                           results);
        if (rc < 0) return rc;
        if (dense)
            return tb_multi_batch_encode_trailer(out, n * 16u, 16, sm->counts.data(), uint32_t(nb));
        // Sparse: each batch's errors, indexed within the batch (execute_create runs per batch).
        uint32_t written = 0, offset = 0;
        std::vector<uint16_t> reply_counts(static_cast<size_t>(nb));
        for (int64_t b = 0; b < nb; b++) {
            const uint32_t bytes = sparse_results(results + offset, sm->counts[b], out + written);
            reply_counts[b] = uint16_t(bytes / 8);
            written += bytes;
            offset += sm->counts[b];
        }
        if (!info.multi_batch) return written;
        return tb_multi_batch_encode_trailer(out, written, 8, reply_counts.data(), uint32_t(nb));
    }

    if (!info.batchable) {
        // The scans (execute_query_multi_batch :2823-2910, execute_query :2764-2821): each batch
        // is one filter, its results (at most min(filter.limit, result_max)) one reply batch.
        if (!ex.get_account_transfers || !ex.get_account_balances || !ex.query_accounts ||
            !ex.query_transfers)
            return TBG_EINVAL;
        const uint32_t limit_max = sm->result_max(info, sm->options.message_body_size_max);
        const uint8_t* filter = static_cast<const uint8_t*>(body);
        std::vector<uint16_t> reply_counts(static_cast<size_t>(nb));
        uint32_t written = 0;
        for (int64_t b = 0; b < nb; b++, filter += info.event_size) {
            const int64_t count = execute_scan(ex, operation, filter, limit_max, out + written);
            if (count < 0) return count;
            reply_counts[b] = uint16_t(count);
            written += uint32_t(count) * info.result_size;
        }
        if (!info.multi_batch) return written;
        return tb_multi_batch_encode_trailer(out, written, info.result_size, reply_counts.data(),
                                             uint32_t(nb));
    }

    // lookup_accounts / lookup_transfers: per batch, found objects only (:3255-3292).
    const bool accounts = operation == TB_OPERATION_LOOKUP_ACCOUNTS ||
                          operation == TB_OPERATION_DEPRECATED_LOOKUP_ACCOUNTS_UNBATCHED;
    const tb_uint128_t* ids = static_cast<const tb_uint128_t*>(body);
    uint32_t written = 0, offset = 0;
    std::vector<uint16_t> reply_counts(static_cast<size_t>(nb));
    for (int64_t b = 0; b < nb; b++) {
        int64_t found = sm->counts[b] == 0 ? 0
                        : accounts ? ex.lookup_accounts(ex.self, ids + offset, sm->counts[b],
                                                        reinterpret_cast<tb_account_t*>(out + written))
                                   : ex.lookup_transfers(ex.self, ids + offset, sm->counts[b],
                                                         reinterpret_cast<tb_transfer_t*>(out + written));
        if (found < 0) return found;
        reply_counts[b] = uint16_t(found);
        written += uint32_t(found) * 128u;
        offset += sm->counts[b];
    }
    if (!info.multi_batch) return written;
    return tb_multi_batch_encode_trailer(out, written, 128, reply_counts.data(), uint32_t(nb));
}

extern "C" uint64_t tb_sm_get_prepare_timestamp(const tb_sm* sm) { return sm->prepare_timestamp; }
extern "C" uint64_t tb_sm_get_commit_timestamp(const tb_sm* sm) { return sm->commit_timestamp; }
extern "C" uint64_t tb_sm_get_prefetch_timestamp(const tb_sm* sm) {
    return sm->prefetch_timestamp;
}
extern "C" void tb_sm_set_prepare_timestamp(tb_sm* sm, uint64_t v) { sm->prepare_timestamp = v; }
extern "C" void tb_sm_set_commit_timestamp(tb_sm* sm, uint64_t v) { sm->commit_timestamp = v; }
extern "C" void tb_sm_set_prefetch_timestamp(tb_sm* sm, uint64_t v) {
    sm->prefetch_timestamp = v;
}
