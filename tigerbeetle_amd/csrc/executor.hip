// The MI355X batch executor (include/tbg.h): host orchestration of the kernels in kernels.hpp.
//
// All tables live in HBM for the lifetime of a tbg_ctx. A create_* call enqueues a
// fixed launch sequence on the ctx's stream and synchronises once at the end (plus once after the
// ingest pass, to learn whether the call holds imported events, which need timestamp indexes).

#include <hip/hip_runtime.h>

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/tbg.h"
#include "group.hpp"
#include "events.hpp"
#include "durability.hpp"
#include "queries.hpp"
#include "hostio.hpp"
#include "pulse.hpp"

using namespace tbg;

namespace {

inline uint32_t grid_for(uint64_t n) { return uint32_t((n + kBlock - 1) / kBlock); }

uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// Calls at least this large accumulate balances by sort + reduce instead of atomics.
constexpr uint32_t kSortThreshold = 1u << 16;
// Balance items use u128 atomics instead of the sort when the key space has more than this many
// account fields per item.
constexpr uint64_t kAtomicKeysPerItem = 8;
// The pinned blocks kernels write for the spinning host (scalars, results, the sequence word):
// coherent, so that their write-back does not depend on the memory type.
constexpr unsigned int kCoherentHost = hipHostMallocMapped | hipHostMallocCoherent;
// Calls up to this many events find their chunks' batch bounds inside tr_ingest.
constexpr uint32_t kInlineChunkMax = 1u << 16;
constexpr size_t kFlowDebugBytes = 8 * (16 + 8 * 1000);  // TBG_FLOW_DEBUG counters (+ per owner)

struct PulseScratch {
    uint64_t capacity = 0;  // a multiple of kPulseRun (pulse.hpp's sorted runs)
    uint64_t *keep = nullptr, *exp = nullptr, *ts = nullptr, *rows = nullptr;
    uint64_t *exp_b = nullptr, *rows_b = nullptr;
    uint32_t* run_len = nullptr;  // two arrays of capacity / kPulseSortRun + 1
    bool counters_clean = false;  // (tbg_pulse's report clears them for the next pulse)
    unsigned long long* counters = nullptr;  // kept, candidates, earliest unexpired, expired
    unsigned long long* counters_next = nullptr;  // (the other set of two: tbg_pulse alternates)
    unsigned long long* counters_base = nullptr;  // (the allocation holding both)
    unsigned int* expired = nullptr;
    uint64_t* sel = nullptr;  // tbg_pulse's expired rows, in order (kPulseRun)
    PulseRuns first{}, second{};  // the last selection's buffers (pulse_apply_root)
};

// Flow replay scratch (flow.hpp, group.hpp), grown on demand to the largest replay list seen.
struct FlowScratch {
    uint64_t cap = 0;          // positions
    uint64_t slots = 0;        // grouping hash slots
    uint8_t *head8 = nullptr, *barrier8 = nullptr;
    uint32_t *heads = nullptr, *unit_of = nullptr, *barriers = nullptr, *vals = nullptr,
             *vals_sorted = nullptr, *succ = nullptr, *indeg = nullptr, *indeg0 = nullptr;
    uint64_t* keys_sorted = nullptr;
    Step* steps = nullptr;
    tb_transfer_t* evs = nullptr;  // per position: its event (flow_replay loads it with the step)
    uint32_t* queue = nullptr;
    uint8_t* outcome = nullptr;  // account lanes' verdicts
    // the grouping (group.hpp)
    unsigned long long* hkeys = nullptr;
    uint32_t *hcnt = nullptr, *hoff = nullptr, *loc = nullptr, *rank = nullptr;
    uint4* big = nullptr;
    uint32_t* chunk_seg = nullptr;
    unsigned long long* chunk_sum = nullptr;
    unsigned int* seg_done = nullptr;
    // account lanes (lanes.hpp)
    LaneRec* recs = nullptr;
    uint32_t *mailbox = nullptr, *owner_starts = nullptr, *mb_index = nullptr;
    unsigned int* lane_counts = nullptr;
    uint32_t* dup_mark = nullptr;  // per event (batch_events_max)
    unsigned int* counts = nullptr;  // [0] units [1] barriers [2] ready; [4..8] the grouping's
    unsigned long long* words = nullptr;  // [1] expiry_count at the plan's start
    UndoEntry* lane_undo = nullptr;
    unsigned int* engine = nullptr;  // flow engine queue counters
    uint32_t* exp_flag = nullptr;
    uint32_t* acc_free = nullptr;  // per account (lanes.hpp free owners)
    unsigned long long* acc_pot = nullptr;  // per account (group.hpp doomed debits)
    uint32_t* doom_off = nullptr;
};

}  // namespace

// Makes a ctx's device current for the length of an entry point (a process may drive executors on
// several GPUs from one thread, tbg_group.h) and restores the caller's.
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int device) {
        if (device < 0 || hipGetDevice(&prev) != hipSuccess) {
            prev = -1;
            return;
        }
        if (prev != device) (void)hipSetDevice(device);
        else prev = -1;
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};
#define TBG_DEVICE_SCOPE(ctx) DeviceScope tbg_device_scope_((ctx) ? int((ctx)->opt.device) : -1)

struct tbg_ctx {
    tbg_options opt{};
    hipStream_t stream = nullptr;
    std::string error;
    Tables T{};
    DevScalars* d_scalars = nullptr;
    DevScalars* h_scalars = nullptr;  // pinned
    tb_create_result_t* h_results = nullptr;  // pinned: host-buffer calls' results land here first
    hipEvent_t results_ready = nullptr;
    // pinned staging of a host-buffer call's batch ends and timestamps (batch_count_max each)
    uint32_t* h_batch_ends = nullptr;
    uint64_t* h_batch_ts = nullptr;
    // The pinned blocks as the GPU addresses them (hostio.hpp kernels read / write them).
    DevScalars* dh_scalars = nullptr;
    // A call's end as the host sees it without the runtime's stream synchronisation: stage_out's
    // last workgroup writes the call's sequence number into a pinned word (spin_wait).
    unsigned int* h_seq = nullptr;
    unsigned int* dh_seq = nullptr;
    unsigned int* d_stage_done = nullptr;  // stage_out's finished workgroups; [1] tr_ingest's
    unsigned int seq = 0;
    bool spin_sync = false;
    double call_timeout_ms = 60000;  // spin_wait's bound (TBG_CALL_TIMEOUT_MS)
    // The environment knobs (README), read once at tbg_open: a call reads these, not the
    // environment (a getenv scans every variable; a replayed call consulted ~18 of them).
    struct Knobs {
        bool no_pv_fast, no_lanes, no_additive, no_doom, no_free_owners, flow_debug, walk_seq,
            lanes_one_lane, no_window, no_lean_lookup, no_ingest_finish;
        uint32_t flow_lpw, flow_waves, flow_blocks, flow_xcd, flow_backoff;
    } knobs{};
    // The expires_at index's length as of the last create_transfers call or pulse (the pulse's
    // first kernels need no synchronisation for it); cleared by anything else that changes it.
    bool expiry_known = false;
    uint64_t expiry_host = 0;
    unsigned long long* h_pulse = nullptr;   // pinned: a pulse's expired count, the index length
    unsigned long long* dh_pulse = nullptr;
    tb_create_result_t* dh_results = nullptr;
    uint32_t* dh_batch_ends = nullptr;
    uint64_t* dh_batch_ts = nullptr;
    // Host ranges the caller registered (tbg_register_host), mapped for the GPU: bodies are read
    // and results written by kernels over PCIe (hostio.hpp).
    struct Mapped {
        uintptr_t host;
        uint64_t size;
        uintptr_t dev;
    };
    std::vector<Mapped> registered;
    // A host-buffer create_transfers call queues its results' download before its one host
    // synchronisation (create_transfers_impl); valid when the call needed no replay.
    tb_create_result_t* early_dst = nullptr;
    bool early_done = false;
    // The next create_transfers call's scalar words were reset by its staging kernel.
    bool scalars_reset = false;
    // The call's scalar words are zero on device: the last create_transfers call queued
    // tr_reset_scalars at its end and nothing has written them since (create_accounts and the
    // other entry points that may clear this flag).
    bool scalars_clean = true;
    // ... and its body is read by tr_ingest from mapped host memory (the GPU's address), null: the
    // body is in d_events.
    const tb_transfer_t* events_host = nullptr;
    // ... and so are its batch bounds, from the pinned staging (dh_batch_ends / dh_batch_ts): the
    // call has no stage_in launch.
    bool batches_host = false;
    uint32_t epoch = 0;
    // Sticky: a compaction failed after it began moving rows; the tables are undefined and every
    // later call fails (tbg_compact).
    bool failed = false;
    bool force_replay = false;
    bool serial_replay = false;  // debug: every replay on one lane (replay_kernel)
    bool call_one_chain = false;  // the next call is one chain (TBG_ONE_CHAIN): serial replay
    tbg_stats stats{};

    // per-call scratch (capacity batch_events_max)
    uint8_t* d_events = nullptr;
    tb_create_result_t* d_results = nullptr;
    uint32_t* d_batch_ends = nullptr;
    uint64_t* d_batch_ts = nullptr;
    uint32_t* ev_slot = nullptr;
    uint32_t* ev_dr = nullptr;
    uint32_t* ev_cr = nullptr;
    uint64_t* ev_amount = nullptr;
    uint64_t* ev_prow = nullptr;
    uint8_t* ev_info = nullptr;
    uint8_t* ev_slow = nullptr;
    uint32_t* slow_list = nullptr;
    uint32_t* fix_slots = nullptr;  // tr_commit's fixed failures' id slots (Call::fix_slots)
    unsigned long long* chain_planes = nullptr;  // (Call::chain_planes, calls past kInlineChunkMax)
    bool chain_hint = true;  // the last large call had linked chains (tr_chain_planes is launched)
    bool replay_hint = false;  // the last large call replayed (its results were downloaded twice)
    uint64_t* pnt_call = nullptr;           // pulse_next_timestamp updates per event (post/void)
    bool pnt_sharded = false;               // tbg_set_pnt_sharded: every call records its updates
    Call<tb_transfer_t> pnt_last{};         // the last create_transfers call (tbg_pnt_ops)
    bool pnt_last_valid = false;
    unsigned long long* pnt_fired = nullptr;
    uint64_t* pnt_tiles = nullptr;          // pnt_resolve's per-tile minima (its own scratch)
    uint64_t* d_stamps = nullptr;           // per-event timestamps of a host stamped call
    unsigned long long* pv_slots = nullptr;  // pending-id claims of post/void events (kernels.hpp)
    uint64_t pv_mask = 0;
    // balance items (2 per event, packed u64) and their sorted copy
    uint64_t* bal_items = nullptr;
    uint4* chunk_info = nullptr;     // per 64-event chunk of a create_transfers call
    uint64_t* bal_items_sorted = nullptr;  // sorted (large key spaces) or bucketed items
    unsigned int* bucket_words = nullptr;  // counts, cursors, offsets, slice bases
    uint64_t* bucket_partials = nullptr;   // per slice: kBucketKeys partial sums
    uint64_t bucket_slices_max = 0;
    uint32_t* window_partials = nullptr;   // balance window: per workgroup, kWindowKeys u32 sums
    unsigned long long* window_carry = nullptr;  // per window key (zero between calls)
    unsigned int* window_counts = nullptr;  // per workgroup: its slice's items; [kWindowGridMax] done
    unsigned long long* window_ts = nullptr;  // per workgroup: first / last created timestamp
    // The last create_transfers call's balance window (its AccountEvents may take ae_window_emit).
    struct WindowCall {
        uint32_t epoch = 0, nwg = 0, ps = 0, wkeys = 0;
    } win;
    // account index build (cuckoo insertion + repair)
    uint32_t* idx_dirty = nullptr;
    unsigned int* idx_counters = nullptr;
    uint32_t idx_dirty_cap = 0;
    // chained scans (prims.hpp): per-tile status words, the tile ticket, launch sequence
    unsigned long long* scan_status = nullptr;
    uint64_t scan_tiles_cap = 0;
    unsigned int* scan_ticket = nullptr;
    uint32_t scan_ticket_base = 0;
    uint32_t scan_seq = 0;

    // imported-timestamp indexes (rebuilt on demand)
    uint64_t* acc_ts_index = nullptr;
    uint64_t* tr_ts_index = nullptr;
    bool acc_ts_stale = true, tr_ts_stale = true;
    uint32_t* sel_buf = nullptr;  // selection output for dumps / indexes (max rows)

    PulseScratch pulse;
    uint32_t pulse_row_bits = 1;  // bits of a transfer row (pulse.hpp PulsePack)
    FlowScratch flow;

    // The account_events groove (events.hpp): AccountEvents in timestamp order + their references.
    tb_account_event_t* ae_log = nullptr;
    AeRef* ae_ref = nullptr;
    // The log's length / last timestamp / order as of the last ae_settle; appends advance them on
    // device (ae_words[4..6]) and ae_bound, an upper bound of the length, on the host.
    uint64_t ae_cap = 0, ae_used = 0, ae_last_ts = 0, ae_bound = 0;
    bool ae_sorted = true, ae_pending = false;
    // Host-buffer create_transfers: its AccountEvents are launched after the results' download.
    bool ae_defer = false, ae_deferred = false;
    // A pulse's appends, queued later (ae_flush_graph): by the next call once its first kernels
    // are queued (the host's launches then overlap the GPU), or by whatever joins the side stream
    // or takes a staging buffer first.
    // The body buffer of the current host-buffer call (d_events).
    uint8_t* body_dst = nullptr;
    bool ae_graph_deferred = false;
    uint32_t ae_def_parity = 0, ae_def_epoch = 0;
    bool ae_def_pending = false;
    // The deferred appends are a small call's (not a pulse's): the pinned word h_pulse[4] says
    // which appends its staging needs once its snapshot (stage_out) has completed.
    bool ae_def_call = false;
    Call<tb_transfer_t> ae_call{};
    AeScratch ae{};
    uint64_t ae_touch_cap = 0;
    uint32_t* ae_list = nullptr;
    unsigned long long* ae_words = nullptr;  // bounds / counts
    // Small create_transfers calls hand their appends to a side stream (ae_transfers_async): a
    // staging buffer per parity, the side stream's own positions and grouping scratch. Every other
    // use of the log joins the side stream first (ae_join).
    hipStream_t ae_stream = nullptr;
    AeStage ae_stage[2] = {};
    uint32_t* ae_pos = nullptr;
    hipEvent_t ae_snap_ready[2] = {}, ae_done[2] = {};
    bool ae_done_recorded[2] = {};
    uint32_t ae_parity = 0;
    bool ae_async_pending = false;
    bool ae_async = true;  // tbg_debug_ae_sync(ctx, 1): every append on the call's stream
    bool ae_window_on = true;  // TBG_NO_AE_WINDOW=1: window calls take the general appends
    bool ae_async_ready = false;
    AeScratch ae_g{};
    // The call's stage_out took its staging and the side stream's appends were queued behind it,
    // before the host's synchronisation (valid unless a replay followed: then stage_out wrote no
    // created flags and the appends found nothing).
    bool ae_snap_early = false;
    unsigned long long* ae_g_words = nullptr;  // [0] created count; [8..] the graph's scan words
    unsigned int* ae_small_counts = nullptr;   // ae_small_emit: per workgroup, then done
    // ae_dense_* scratch (allocated at the first general call they take)
    uint4* ae_dense_touch = nullptr;
    uint4* ae_dense_ev = nullptr;
    uint32_t* ae_dense_partials = nullptr;
    unsigned int* ae_dense_counts = nullptr;
    unsigned long long* ae_dense_ts = nullptr;
    uint4* ae_dense_later = nullptr;
    AeDense ae_dense_job{};           // (ae_dense_prefix -> ae_dense)
    uint32_t ae_dense_prefixed = 0;   // the epoch whose prefix is queued
    uint32_t* ae_dense_pos = nullptr;
    unsigned int* ae_dense_claim = nullptr;
    unsigned long long* ae_small_ts = nullptr;
    // ae_wide_* scratch (grown to the largest wide window call): per slice, field and account
    u128* ae_wide_sums = nullptr;
    uint64_t ae_wide_sums_cap = 0;
    unsigned int* ae_wide_counts = nullptr;      // per slice; [ae_wide_slices_cap]: done
    unsigned long long* ae_wide_ts = nullptr;
    uint32_t ae_wide_slices_cap = 0;
    unsigned long long* flow_debug = nullptr;

    // Per-kernel timing (tbg_profile): HIP events recorded on the call's stream between launches.
    bool timing = false;
    bool timing_host = false;  // host phases only (tbg_profile(ctx, 2): no HIP events)
    // Span marks only (tbg_profile(ctx, 3)): each HIP event recorded between two launches idles
    // the GPU ~6 us (profiles/r06_lean/), so the per-kernel marks inflate a call's device time by
    // ~10 % on configs 3 / 4; these keep only the marks that bound the call's device spans.
    bool timing_lean = false;
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

// Every call on a ctx whose tables a failed compaction left undefined fails.
#define FAILED_GUARD(ctx)                                                        \
    do {                                                                         \
        if ((ctx)->failed) {                                                     \
            (ctx)->error = "tables undefined after a failed compaction";        \
            return TBG_EHIP;                                                     \
        }                                                                        \
    } while (0)

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

// Tile words for `tiles` tiles and this launch's ScanState (prims.hpp).
int scan_state(tbg_ctx* ctx, uint64_t tiles, ScanState* out) {
    if (tiles > 0xFFFFFFFFull) return TBG_EINVAL;
    if (!ctx->scan_ticket) HIP_TRY(ctx, hipMalloc(&ctx->scan_ticket, sizeof(unsigned int)));
    if (tiles > ctx->scan_tiles_cap) {
        if (ctx->scan_status) {
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
            HIP_TRY(ctx, hipFree(ctx->scan_status));
            ctx->scan_status = nullptr;
        }
        const uint64_t cap = std::max<uint64_t>(next_pow2(tiles), 1024);
        HIP_TRY(ctx, hipMalloc(&ctx->scan_status, cap * sizeof(unsigned long long)));
        // zero words carry sequence 0, which no launch uses: "not ready"
        HIP_TRY(ctx, hipMemsetAsync(ctx->scan_status, 0, cap * sizeof(unsigned long long), ctx->stream));
        HIP_TRY(ctx, hipMemsetAsync(ctx->scan_ticket, 0, sizeof(unsigned int), ctx->stream));
        ctx->scan_ticket_base = 0;
        ctx->scan_tiles_cap = cap;
    }
    ctx->scan_seq = ctx->scan_seq % ((1u << 30) - 1) + 1;
    *out = ScanState{ctx->scan_status, ctx->scan_ticket, ctx->scan_ticket_base, ctx->scan_seq};
    ctx->scan_ticket_base += uint32_t(tiles);
    return 0;
}

uint64_t scan_tiles(uint64_t n) { return n ? (n + kScanTile - 1) / kScanTile : 1; }

// One chained scan (prims.hpp): `n` items, the op's emits and total.
template <typename Op>
int launch_scan(tbg_ctx* ctx, uint64_t n, const Op& op) {
    const uint64_t tiles = scan_tiles(n);
    ScanState st;
    if (int rc = scan_state(ctx, tiles, &st)) return rc;
    hipLaunchKernelGGL(chained_scan<Op>, dim3(uint32_t(tiles)), dim3(kScanThreads), 0, ctx->stream,
                       n, op, st);
    return 0;
}

// Two independent chained scans in one launch (chained_scan2).
template <typename Op1, typename Op2>
int launch_scan2(tbg_ctx* ctx, uint64_t n1, const Op1& op1, uint64_t n2, const Op2& op2) {
    const uint64_t t1 = scan_tiles(n1), t2 = scan_tiles(n2);
    ScanState st;
    if (int rc = scan_state(ctx, t1 + t2, &st)) return rc;
    hipLaunchKernelGGL((chained_scan2<Op1, Op2>), dim3(uint32_t(t1 + t2)), dim3(kScanThreads), 0,
                       ctx->stream, n1, op1, n2, op2, uint32_t(t1), st);
    return 0;
}

// Order-preserving selection of indices [0, n) whose flag is nonzero (one launch).
int select_flagged(tbg_ctx* ctx, const uint8_t* flags, uint64_t n, uint32_t* out,
                   unsigned int* d_count) {
    return launch_scan(ctx, n, SelectFlags8{flags, out, d_count});
}

int stage_call_outputs(tbg_ctx* ctx, const tb_create_result_t* d_results, tb_create_result_t* dst,
                       uint32_t n, bool scalars, const AeSnapJob* snap = nullptr,
                       bool fixes = false, unsigned int seq = 0, uint32_t skip_epoch = 0,
                       bool clear = false);
// The scalars block to the host (a kernel writes the mapped pinned copy: no DMA hand-off).
int sync_scalars(tbg_ctx* ctx) {
    int rc = stage_call_outputs(ctx, nullptr, nullptr, 0, true);
    if (rc) return rc;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

// The marks tbg_profile(ctx, 3) records: the call's start, the host's waits, the end of a
// replayed call's work ("call"), the skipped spans ('-'), the AccountEvents and pulse spans, and
// the accounts' (their calls keep every mark).
bool lean_mark(const char* n) {
    return n[0] == '-' || !strcmp(n, "begin") || !strcmp(n, "host_sync") || !strcmp(n, "call") ||
           !strcmp(n, "account_events") || !strncmp(n, "pulse:", 6) || !strncmp(n, "acc_", 4);
}
void tmark(tbg_ctx* ctx, const char* name) {
    if (!ctx->timing || ctx->n_marks >= tbg_ctx::kMaxMarks) return;
    if (ctx->timing_lean && !lean_mark(name)) return;
    // (a skipped span right after "call" is empty: the next span starts at "call" instead of a
    // second event recorded back to back)
    if (ctx->timing_lean && name[0] == '-' && ctx->n_marks > 0 &&
        !strcmp(ctx->mark_names[ctx->n_marks - 1], "call"))
        return;
    if (!ctx->marks[ctx->n_marks]) (void)hipEventCreate(&ctx->marks[ctx->n_marks]);
    (void)hipEventRecord(ctx->marks[ctx->n_marks], ctx->stream);
    ctx->mark_names[ctx->n_marks++] = name;
}

// Host wall time of a phase of a host-buffer call (tbg_profile): accumulated like the marks.
void hprof(tbg_ctx* ctx, const char* name, double ms) {
    if (!ctx->timing_host) return;
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
double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

// After the stream is synchronised: accumulate the time between consecutive marks per name.
void tcollect(tbg_ctx* ctx) {
    if (!ctx->timing) return;
    for (int i = 1; i < ctx->n_marks; i++) {
        if (ctx->mark_names[i][0] == '-') continue;  // a span start only
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

// Sorted timestamps of live rows (creation order is timestamp order within each groove).
template <typename Row>
int rebuild_ts_index(tbg_ctx* ctx, const Row* rows, const uint8_t* live, uint64_t used,
                     uint64_t* index, uint64_t* count) {
    if (used == 0) {
        *count = 0;
        return 0;
    }
    unsigned int* d_count = &ctx->d_scalars->slow_count;  // scratch word (between calls)
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
    c.one_chain = ctx->call_one_chain ? 1 : 0;
    c.force_replay = ctx->force_replay || ctx->call_one_chain ? 1 : 0;
    c.bal_items = nullptr;
    c.key_bits = 0;
    c.pair_shift = 0;
    c.lean_lookup = 0;
    c.bucket_counts = nullptr;
    c.n_buckets = 0;
    c.chunk_info = nullptr;
    c.event_ts = nullptr;
    c.ev_slot = ctx->ev_slot;
    c.ev_dr = ctx->ev_dr;
    c.ev_cr = ctx->ev_cr;
    c.ev_amount = ctx->ev_amount;
    c.ev_prow = ctx->ev_prow;
    c.ev_info = ctx->ev_info;
    c.ev_slow = ctx->ev_slow;
    c.slow_list = ctx->slow_list;
    c.pnt_call = ctx->pnt_call;
    c.events_out = nullptr;
    c.ends_out = nullptr;
    c.ts_out = nullptr;
    c.fix_slots = ctx->fix_slots;
    c.chain_planes = nullptr;
    // (TBG_NO_PV_FAST: every post/void replays)
    c.pv_slots = ctx->knobs.no_pv_fast ? nullptr : ctx->pv_slots;
    c.pv_mask = ctx->pv_mask;
    c.pnt_force = ctx->pnt_sharded ? 1 : 0;
    c.finish_done = nullptr;
    c.finish_scalars = nullptr;
    c.finish_seq = nullptr;
    c.seq = 0;
    c.finish_always = 0;
    c.commit_done = nullptr;
    c.commit_scalars = nullptr;
    c.commit_seq = nullptr;
    c.commit_seq_val = 0;
    return c;
}

// zero_scalars: reset the per-call words of the scalars block (flags, slow_count, stats) here;
// create_transfers resets them in its first kernel (tr_chunk_info) instead.
int begin_call(tbg_ctx* ctx, bool zero_scalars = true) {
    if (zero_scalars) ctx->scalars_clean = false;  // (the call's kernels write its scalar words)
    if (ctx->timing && ctx->n_marks > 1) {  // the previous call's AccountEvents (queued after it)
        (void)hipStreamSynchronize(ctx->stream);
        tcollect(ctx);
    }
    ctx->n_marks = 0;
    if (zero_scalars)
        HIP_TRY(ctx, hipMemsetAsync(&ctx->d_scalars->flags, 0,
                                    sizeof(DevScalars) - offsetof(DevScalars, flags), ctx->stream));
    tmark(ctx, "begin");
    return 0;
}

int end_call(tbg_ctx* ctx, uint32_t n, bool already_synced = false) {
    if (!already_synced) {
        int rc = sync_scalars(ctx);
        if (rc) return rc;
    }
    tcollect(ctx);
    const DevScalars& s = *ctx->h_scalars;
    ctx->expiry_host = s.expiry_count;
    ctx->expiry_known = true;
    ctx->stats.events = n;
    ctx->stats.ae_window = 0;
    ctx->stats.ingest_finished = (s.flags & kFlagFinished) ? 1 : 0;
    ctx->stats.fast = s.stats[1];
    ctx->stats.replayed = s.stats[2];
    ctx->stats.static_fail = s.stats[3];
    if (s.flags & kFlagTableFull) {
        ctx->error = "table capacity exceeded";
        return TBG_ENOSPC;
    }
    if (s.flags & kFlagFlowStalled) {
        ctx->error = "flow replay stalled (watchdog)";
        return TBG_EHIP;
    }
    if (s.flags & kFlagUndoOverflow) {
        ctx->error = "linked chain longer than the undo log";
        return TBG_ENOSPC;
    }
    return 0;
}

void free_flow(FlowScratch& F) {
    void* ptrs[] = {F.head8, F.barrier8, F.heads, F.unit_of, F.barriers, F.vals, F.vals_sorted,
                    F.succ, F.indeg, F.indeg0, F.keys_sorted, F.steps, F.evs, F.queue,
                    F.outcome, F.recs, F.mailbox, F.owner_starts, F.mb_index, F.exp_flag,
                    F.hkeys, F.hcnt, F.hoff, F.loc, F.rank, F.big, F.chunk_seg, F.chunk_sum,
                    F.seg_done};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    F.head8 = F.barrier8 = F.outcome = nullptr;
    F.heads = F.unit_of = F.barriers = F.vals = F.vals_sorted = F.succ = F.indeg = F.indeg0 = nullptr;
    F.keys_sorted = nullptr;
    F.steps = nullptr;
    F.evs = nullptr;
    F.queue = nullptr;
    F.recs = nullptr;
    F.exp_flag = nullptr;
    F.mailbox = F.owner_starts = F.mb_index = nullptr;
    F.hkeys = nullptr;
    F.hcnt = F.hoff = F.loc = F.rank = nullptr;
    F.big = nullptr;
    F.chunk_seg = nullptr;
    F.chunk_sum = nullptr;
    F.seg_done = nullptr;
    F.cap = F.slots = 0;
}

int ensure_flow(tbg_ctx* ctx, uint64_t m) {
    FlowScratch& F = ctx->flow;
    bool ok = true;
    if (!F.dup_mark) {
        ok = dev_alloc(ctx, &F.dup_mark, ctx->opt.batch_events_max, true) &&
             dev_alloc(ctx, &F.counts, 12, true) && dev_alloc(ctx, &F.words, 4, true) &&
             dev_alloc(ctx, &F.lane_counts, 4, true) &&
             dev_alloc(ctx, &F.lane_undo, uint64_t(kFlowLanesMax) * kFlowUndoPerLane, false) &&
             dev_alloc(ctx, &F.engine, kFlowEngineWords, true) &&
             dev_alloc(ctx, &F.acc_free, ctx->opt.account_capacity, true) &&
             dev_alloc(ctx, &F.acc_pot, ctx->opt.account_capacity, true) &&
             dev_alloc(ctx, &F.doom_off, 1, true);
        if (!ok) return TBG_EHIP;
    }
    if (m <= F.cap) return 0;
    free_flow(F);
    // Sized once for the context's calls (up to 2^21 replayed events): a reallocation -- ~30
    // allocations, their clears and the frees' synchronisation -- costs ~50-100 us of host time
    // with the GPU idle, so growing with each call's replay list cost config 4's first calls that
    // much each.
    const uint64_t cap = std::max<uint64_t>(
        {next_pow2(m), 1u << 14, std::min<uint64_t>(next_pow2(ctx->opt.batch_events_max), 1u << 21)});
    const uint64_t kc = kFlowKeys * cap;
    const uint64_t slots = 2 * kc;  // grouping table load <= 0.5
    ok = dev_alloc(ctx, &F.head8, cap, false) && dev_alloc(ctx, &F.barrier8, cap, false) &&
         dev_alloc(ctx, &F.heads, cap, false) && dev_alloc(ctx, &F.unit_of, cap, false) &&
         dev_alloc(ctx, &F.barriers, cap, false) && dev_alloc(ctx, &F.indeg, cap, true) && dev_alloc(ctx, &F.indeg0, cap, false) &&
         dev_alloc(ctx, &F.vals, kc, false) && dev_alloc(ctx, &F.vals_sorted, kc, false) &&
         dev_alloc(ctx, &F.succ, kc, false) && dev_alloc(ctx, &F.keys_sorted, kc, false) &&
         dev_alloc(ctx, &F.steps, cap, false) && dev_alloc(ctx, &F.evs, cap, false) &&
         dev_alloc(ctx, &F.queue, cap, false) &&
         dev_alloc(ctx, &F.outcome, cap, false) && dev_alloc(ctx, &F.recs, cap, false) &&
         dev_alloc(ctx, &F.mailbox, cap, false) && dev_alloc(ctx, &F.mb_index, cap, false) &&
         dev_alloc(ctx, &F.exp_flag, cap, false) && dev_alloc(ctx, &F.owner_starts, kc, false) &&
         dev_alloc(ctx, &F.hkeys, slots, true) && dev_alloc(ctx, &F.hcnt, slots, true) &&
         dev_alloc(ctx, &F.hoff, slots, false) && dev_alloc(ctx, &F.loc, kc, false) &&
         dev_alloc(ctx, &F.rank, kc, false) && dev_alloc(ctx, &F.big, kc / kGroupSmall + 1, false) &&
         dev_alloc(ctx, &F.chunk_seg, kc / kGroupChunk + kc / kGroupSmall + 1, false) &&
         dev_alloc(ctx, &F.chunk_sum, 2 * (kc / kGroupChunk + kc / kGroupSmall + 1), false) &&
         dev_alloc(ctx, &F.seg_done, kc / kGroupSmall + 1, false);
    if (!ok) {
        free_flow(F);
        return TBG_EHIP;
    }
    F.cap = cap;
    F.slots = slots;
    return 0;
}

// The flow replay of a create_transfers call (flow.hpp): plan the units and group their keys
// (group.hpp), then run the account lanes (lanes.hpp) or the flow engine; pulse_next_timestamp is
// resolved afterwards in post/void calls.
int run_flow_replay(tbg_ctx* ctx, Call<tb_transfer_t>& c, uint32_t m, unsigned int call_flags) {
    int rc = ensure_flow(ctx, m);
    if (rc) return rc;
    FlowScratch& F = ctx->flow;
    FlowPlan P{};
    P.m = m;
    P.epoch = c.epoch;
    P.slow_list = c.slow_list;
    P.head8 = F.head8;
    P.heads = F.heads;
    P.counts = F.counts;
    P.unit_of = F.unit_of;
    P.barrier8 = F.barrier8;
    P.barriers = F.barriers;
    P.dup_mark = F.dup_mark;
    P.succ = F.succ;
    P.indeg = F.indeg;
    P.indeg0 = F.indeg0;
    P.queue = F.queue;
    const bool post_void = (call_flags & kFlagPostVoid) != 0;
    P.pnt_ops = post_void || c.pnt_force ? c.pnt_call : nullptr;
    P.lane_undo = F.lane_undo;
    P.steps = F.steps;
    P.evs = F.evs;
    P.engine = F.engine;
    P.exp_flag = F.exp_flag;
    P.exp_base = &F.words[1];
    P.lane_counts = F.lane_counts;
    // Additive accounts get no key (Replay::additive); TBG_NO_ADDITIVE keys every account.
    // (kFlagNoLanes: a replayed event the lanes would refuse -- the plan then keeps doomed debits
    // off their accounts' keys; config 4's first call, no post/void yet: 825 -> ~360 us)
    const bool lanes_possible =
        !(call_flags & (kFlagDuplicate | kFlagPostVoid | kFlagClosable | kFlagImported |
                        kFlagNoLanes)) &&
        !c.force_replay && !ctx->knobs.no_lanes;
    P.add_epoch = ctx->knobs.no_additive ? 0 : c.epoch;
    // Doomed debits (group.hpp): not with the account lanes (which decide limit events themselves).
    const bool doom = !lanes_possible && !ctx->knobs.no_doom;
    P.acc_pot = doom ? F.acc_pot : nullptr;
    P.doom_off = F.doom_off;

    GroupPlan G{};
    // The grouping table sized for this call (load <= 0.5 at kFlowKeys keys per event): a prefix
    // of the allocation, which group_small leaves clear after every call.
    const uint64_t slots = std::min<uint64_t>(F.slots, std::max<uint64_t>(next_pow2(2 * kFlowKeys * uint64_t(m)), 1u << 15));
    G.hmask = slots - 1;
    G.hkeys = F.hkeys;
    G.hcnt = F.hcnt;
    G.hoff = F.hoff;
    G.loc = F.loc;
    G.rank = F.rank;
    G.vals = F.vals;
    G.vals_sorted = F.vals_sorted;
    G.keys_sorted = F.keys_sorted;
    G.big = F.big;
    G.counts = F.counts + 4;
    G.chunk_seg = F.chunk_seg;
    G.chunk_sum = F.chunk_sum;
    G.seg_done = F.seg_done;
    G.unit_of = F.unit_of;
    G.succ = F.succ;
    G.indeg = F.indeg;
    G.lanes = lanes_possible;
    G.free_owners = !ctx->knobs.no_free_owners;
    G.stats = ctx->knobs.flow_debug;
    G.pairs = uint32_t(std::min<uint64_t>(uint64_t(kFlowKeys) * m, 0xFFFFFFFFull));
    G.epoch = c.epoch;
    G.owner_starts = F.owner_starts;
    G.lane_counts = F.lane_counts;
    G.recs = F.recs;
    G.acc_free = F.acc_free;

    LanePlan L{};
    L.m = m;
    L.keys_sorted = F.keys_sorted;
    L.n_pairs = F.counts + 4;
    L.steps = F.steps;
    L.slow_list = c.slow_list;
    L.recs = F.recs;
    L.mailbox = F.mailbox;
    L.mb_index = F.mb_index;
    L.outcome = F.outcome;
    L.owner_starts = F.owner_starts;
    L.counts = F.lane_counts;
    L.epoch = c.epoch;
    L.acc_free = F.acc_free;
    L.walk_seq = ctx->knobs.walk_seq;

    const dim3 block(kBlock);
    const uint64_t pairs = kFlowKeys * uint64_t(m);
    hipLaunchKernelGGL(flow_heads, dim3(grid_for(std::max<uint64_t>(m, kFlowEngineWords))), block,
                       0, ctx->stream, ctx->T, c, P);
    rc = launch_scan(ctx, m, SelectHeads{F.head8, F.heads, F.unit_of, &F.counts[0]});
    if (rc) return rc;
    if (doom)
        hipLaunchKernelGGL(flow_credit_pot, dim3(grid_for(m)), block, 0, ctx->stream, ctx->T, c, P,
                           call_flags);
    hipLaunchKernelGGL(plan_keys, dim3((m + kPlanKeysThreads - 1) / kPlanKeysThreads), dim3(kPlanKeysThreads), 0,
                       ctx->stream, ctx->T, c, P, G, L, call_flags);
    // the planned expires_at entries, and the slots' segments (one launch)
    rc = launch_scan2(ctx, m,
                      PlanExpiry{F.exp_flag, c.slow_list, ctx->T.expiry, ctx->T.expiry_capacity,
                                 c.row_base, &F.words[1],
                                 reinterpret_cast<unsigned long long*>(&ctx->T.scalars->expiry_count),
                                 &ctx->T.scalars->flags},
                      slots, ExclusiveSumU32{F.hcnt, F.hoff, &F.counts[4]});
    if (rc) return rc;
    hipLaunchKernelGGL(group_scatter, dim3(grid_for(pairs)), block, 0, ctx->stream, G, pairs);
    hipLaunchKernelGGL(group_small, dim3(grid_for(slots)), block, 0, ctx->stream, ctx->T, G,
                       slots);
    hipLaunchKernelGGL(group_sort, dim3(kGroupBigBlocks), dim3(kGroupBigThreads), 0, ctx->stream, G);
    hipLaunchKernelGGL(group_chunk, dim3(kGroupChunkBlocks), dim3(kGroupBigThreads), 0, ctx->stream,
                       ctx->T, G);
    // the initially ready units, and the barrier events (one launch)
    rc = launch_scan2(ctx, m, SelectReady{F.indeg, F.counts, F.queue, F.engine, &F.counts[2], F.indeg0}, m,
                      SelectFlags8{F.barrier8, F.barriers, &F.counts[1]});
    if (rc) return rc;
    // Calls of limit events only: the account lanes (lanes.hpp); the flow replay then skips.
    P.skip = nullptr;
    if (lanes_possible) {
        // One-lane walk (lanes_replay): LDS mailbox indexes. Wave walk (lanes_walk, the
        // default): a zeroed word per position (plan_keys).
        const bool one_lane = ctx->knobs.lanes_one_lane;
        if (one_lane) {
            rc = launch_scan(ctx, m, ExclusiveSumU32{F.mailbox, F.mb_index, nullptr});
            if (rc) return rc;
            hipLaunchKernelGGL(lanes_mailboxes, dim3(grid_for(m)), block, 0, ctx->stream, L);
        }
        tmark(ctx, "flow_plan");
        // Free owners (their verdicts: the grouping): their events' owner bits.
        if (!ctx->knobs.no_free_owners)
            hipLaunchKernelGGL(lanes_free, dim3(grid_for(m)), block, 0, ctx->stream, ctx->T, L);
        if (one_lane)
            hipLaunchKernelGGL(lanes_replay, dim3(1), dim3(kLanesMax), 0, ctx->stream, ctx->T, c, L);
        else {
            const bool dbg = ctx->knobs.flow_debug;
            if (dbg) {
                if (!ctx->flow_debug) HIP_TRY(ctx, hipMalloc(&ctx->flow_debug, kFlowDebugBytes));
                HIP_TRY(ctx, hipMemsetAsync(ctx->flow_debug, 0, kFlowDebugBytes, ctx->stream));
            }
            if (dbg)
                hipLaunchKernelGGL(lanes_walk<true>, dim3(kLanesMax / kWalkWaves),
                                   dim3(kWalkWaves * 64), 0, ctx->stream, ctx->T, c, L, F.mb_index,
                                   ctx->flow_debug);
            else
                hipLaunchKernelGGL(lanes_walk<false>, dim3(kLanesMax / kWalkWaves),
                                   dim3(kWalkWaves * 64), 0, ctx->stream, ctx->T, c, L, F.mb_index,
                                   nullptr);
            if (dbg) {
                unsigned long long d[16] = {};
                (void)hipMemcpyAsync(d, ctx->flow_debug, 128, hipMemcpyDeviceToHost, ctx->stream);
                (void)hipStreamSynchronize(ctx->stream);
                fprintf(stderr, "walk: m=%u walks=%llu windows=%llu events=%llu polls=%llu "
                        "poll_us=%.1f snapshot_hits=%llu longest_walk_us=%.1f refreshes=%llu "
                        "refresh_us=%.1f window_head_us=%.1f\n", m, d[6], d[0], d[1], d[2],
                        d[3] / 100.0, d[5], d[4] / 100.0, d[7], d[8] / 100.0, d[9] / 100.0);
                std::vector<unsigned long long> o(8 * 1000);
                (void)hipMemcpy(o.data(), ctx->flow_debug + 16, o.size() * 8, hipMemcpyDeviceToHost);
                std::vector<uint32_t> idx;
                for (uint32_t i = 0; i < 1000; i++)
                    if (o[8 * i]) idx.push_back(i);
                std::sort(idx.begin(), idx.end(),
                          [&](uint32_t a, uint32_t b) { return o[8 * a] > o[8 * b]; });
                for (size_t i = 0; i < idx.size() && i < 3; i++) {
                    const unsigned long long* w = &o[8 * idx[i]];
                    const unsigned long long lo24 = (1ull << 24) - 1;
                    fprintf(stderr, "  owner %u: events=%llu windows=%llu all_pass=%llu iters=%llu "
                            "polls=%llu poll_us=%.1f walk_us=%.1f refreshes=%llu refresh_us=%.1f "
                            "head_us=%.1f window_us=%.1f stepB_us=%.1f tail_us=%.1f\n",
                            idx[i], w[0], w[4] & lo24, w[6] & lo24, w[5] & lo24, w[1] & lo24,
                            w[2] / 100.0, w[3] / 100.0, w[7] >> 32, (w[7] & 0xFFFFFFFFull) / 100.0,
                            (w[4] >> 24) / 100.0, (w[1] >> 24) / 100.0, (w[5] >> 24) / 100.0,
                            (w[6] >> 24) / 100.0);
                }
            }
        }
        hipLaunchKernelGGL(lanes_finish, dim3(grid_for(m)), block, 0, ctx->stream, ctx->T, c, L);
        if (!ctx->knobs.no_free_owners)
            hipLaunchKernelGGL(lanes_free_sums, dim3(grid_for(pairs)), block, 0, ctx->stream,
                               ctx->T, L, pairs);
        tmark(ctx, "tr_lanes");
        P.skip = &F.lane_counts[2];
    }
    tmark(ctx, "flow_plan");
    const bool debug = ctx->knobs.flow_debug;
    if (debug) {
        if (!ctx->flow_debug) HIP_TRY(ctx, hipMalloc(&ctx->flow_debug, kFlowDebugBytes));
        HIP_TRY(ctx, hipMemsetAsync(ctx->flow_debug, 0, 128, ctx->stream));
        P.debug = ctx->flow_debug;
    }
    // Engine shape (flow.hpp; tbg_ctx::Knobs): lanes per wave x waves per workgroup x workgroups.
    // Default (config 4 sweeps, profiles/r02_shapes): 1 lane per wave, 4 waves x 256 workgroups
    // (1024 lanes) over the whole chip -- with the replay's per-event latency down to ~2.8 us,
    // lanes sharing a wave (divergent branches take turns) cost more than the extra lanes gain:
    // 8192 lanes (8 per wave) 5.9 ms per 1M events, 4096 (1 or 4 per wave) 5.3, 1024 (1 per wave)
    // 4.8-5.2, 512 5.2-5.6.
    P.lanes_per_wave = ctx->knobs.flow_lpw;
    const uint32_t waves = ctx->knobs.flow_waves;
    const uint32_t blocks = ctx->knobs.flow_blocks;
    P.xcd_stride = ctx->knobs.flow_xcd;
    P.backoff = ctx->knobs.flow_backoff;
    const uint32_t lanes = blocks * waves * P.lanes_per_wave;
    if (debug)
        hipLaunchKernelGGL(flow_replay<true>, dim3(blocks * P.xcd_stride), dim3(waves * 64), 0,
                           ctx->stream, ctx->T, c, P);
    else
        hipLaunchKernelGGL(flow_replay<false>, dim3(blocks * P.xcd_stride), dim3(waves * 64), 0,
                           ctx->stream, ctx->T, c, P);
    tmark(ctx, "tr_flow");
    if (debug) {
        unsigned int cnt[2] = {0, 0};
        unsigned long long d[12] = {};
        unsigned int cnt3[8] = {};
        (void)hipMemcpyAsync(cnt3, F.counts, 32, hipMemcpyDeviceToHost, ctx->stream);
        (void)hipMemcpyAsync(d, ctx->flow_debug, 96, hipMemcpyDeviceToHost, ctx->stream);
        cnt[0] = cnt3[0];
        cnt[1] = cnt3[1];
        (void)hipStreamSynchronize(ctx->stream);
        fprintf(stderr, "flow: initially ready %u grouped pairs %u listed segments %u longest id "
                "key %u longest account key %u\n", cnt3[2], cnt3[4], cnt3[5], cnt3[6], cnt3[7]);
        // wall_clock64 runs at 100 MHz on MI300-class parts
        fprintf(stderr, "flow: m=%u units=%u barriers=%u flags=%#x lanes=%u iterations=%llu "
                "events=%llu exec_us=%.1f engine_us=%.1f\n", m, cnt[0], cnt[1], call_flags, lanes,
                d[0], d[1], d[2] / 100.0, d[3] / 100.0);
        fprintf(stderr, "flow: continuations %llu stall: head %llu tail %llu done %llu pos %llu\n",
                d[4], d[8], d[9], d[10], d[11]);
        // The critical path: units in order are a topological order (edges go to later units).
        const uint32_t units = cnt3[0];
        std::vector<uint32_t> heads(units), succ(uint64_t(kFlowKeys) * m);
        (void)hipMemcpy(heads.data(), F.heads, units * 4ull, hipMemcpyDeviceToHost);
        (void)hipMemcpy(succ.data(), F.succ, succ.size() * 4, hipMemcpyDeviceToHost);
        std::vector<uint64_t> start(units, 0), depth(units, 0);
        std::vector<uint32_t> via(units, kNone32), via_key(units, 0);  // the edge that set start
        uint64_t longest = 0, longest_units = 0;
        uint32_t last = 0;
        for (uint32_t u = 0; u < units; u++) {
            const uint32_t b = heads[u], e = u + 1 < units ? heads[u + 1] : m;
            const uint64_t fin = start[u] + (e - b);
            const uint64_t dep = depth[u] + 1;
            if (fin > longest) {
                longest = fin;
                last = u;
            }
            longest_units = std::max(longest_units, dep);
            for (uint64_t i = uint64_t(kFlowKeys) * b; i < uint64_t(kFlowKeys) * e; i++) {
                const uint32_t v = succ[i];
                if (v == kNone32 || v >= units) continue;
                if (fin > start[v]) {
                    start[v] = fin;
                    via[v] = u;
                    via_key[v] = uint32_t(i % kFlowKeys);
                }
                depth[v] = std::max(depth[v], dep);
            }
        }
        // The path's edges by key kind: [0] id, [1] pending id, [2] debit account, [3] credit.
        unsigned kinds[kFlowKeys] = {};
        unsigned chain_units = 0, path_units = 0;
        for (uint32_t u = last; u != kNone32; u = via[u]) {
            path_units++;
            const uint32_t b = heads[u], e = u + 1 < units ? heads[u + 1] : m;
            chain_units += e - b > 1;
            if (via[u] != kNone32) kinds[via_key[u]]++;
        }
        fprintf(stderr, "flow: critical path %llu events, %llu units (%u on the path, %u chains; "
                "edges by key: id %u pending %u debit %u credit %u)\n",
                (unsigned long long)longest, (unsigned long long)longest_units, path_units,
                chain_units, kinds[0], kinds[1], kinds[2], kinds[3]);
    }
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

// pulse_next_timestamp of a call with post/void: its recorded updates in call order (kernels.hpp
// pnt_*). The scratch is the balance items' (consumed before the replay).
int pnt_resolve(tbg_ctx* ctx, const Call<tb_transfer_t>& c) {
    const uint32_t n = c.n;
    const uint32_t tiles = std::max<uint32_t>(1, (n + kPntTile - 1) / kPntTile);
    // (not bal_items: a sharded call without post/void resolves too, and its AccountEvents balance
    // window reads the pair items there afterwards)
    uint64_t* tile_min = ctx->pnt_tiles;
    hipLaunchKernelGGL(pnt_tile_min, dim3(tiles), dim3(kPntThreads), 0, ctx->stream, c.pnt_call, n,
                       tile_min);
    hipLaunchKernelGGL(pnt_tile_resolve, dim3(tiles), dim3(kPntThreads), 0, ctx->stream, ctx->T,
                       c.pnt_call, n, tile_min, ctx->pnt_fired, c.pnt_force);
    tmark(ctx, "pnt_resolve");
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

// The replay list (order-preserving), the replay, and the id slots of the replayed events.
template <typename Event>
int run_replay(tbg_ctx* ctx, Call<Event>& c, bool is_transfers, bool finalize_everything,
               bool selected = false) {
    // (selected: the list was selected before the host's synchronisation)
    int rc = selected ? 0 : select_flagged(ctx, ctx->ev_slow, c.n, ctx->slow_list,
                                          &ctx->d_scalars->slow_count);
    if (rc) return rc;
    if (!selected) tmark(ctx, "select_replay_list");
    const unsigned int call_flags = ctx->h_scalars->flags;
    const uint64_t m = ctx->h_scalars->stats[0];
    if constexpr (__is_same(Event, tb_transfer_t)) {
        if (!ctx->serial_replay && !c.one_chain && !(call_flags & kFlagImported) && m > 1 &&
            m < (1ull << kFlowUnitBits)) {
            rc = run_flow_replay(ctx, c, uint32_t(m), call_flags);
            if (rc) return rc;
            hipLaunchKernelGGL(finalize_slow<Event>, dim3(grid_for(c.n)), dim3(kBlock), 0,
                               ctx->stream, ctx->T, c, 1);
            tmark(ctx, "tr_finalize");
            HIP_TRY(ctx, hipGetLastError());
            return 0;
        }
    }
    hipLaunchKernelGGL(replay_kernel<Event>, dim3(1), dim3(64), 0, ctx->stream, ctx->T, c,
                       is_transfers ? 1 : 0);
    tmark(ctx, is_transfers ? "tr_replay" : "acc_replay");
    if (finalize_everything)
        hipLaunchKernelGGL(finalize_all<Event>, dim3(grid_for(c.n)), dim3(kBlock), 0, ctx->stream,
                           ctx->T, c, is_transfers ? 1 : 0);
    else
        hipLaunchKernelGGL(finalize_slow<Event>, dim3(grid_for(c.n)), dim3(kBlock), 0,
                           ctx->stream, ctx->T, c, is_transfers ? 1 : 0);
    tmark(ctx, is_transfers ? "tr_finalize" : "acc_finalize");
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

int ensure_pulse_scratch(tbg_ctx* ctx, uint64_t count) {
    PulseScratch& S = ctx->pulse;
    // keep: expiry_capacity entries, once (tbg_pulse swaps it with the index: it never shrinks)
    if (!S.keep && !dev_alloc(ctx, &S.keep, ctx->T.expiry_capacity, false)) return TBG_ENOMEM;
    if (S.counters && count <= S.capacity) return 0;
    for (void* p : {(void*)S.exp, (void*)S.ts, (void*)S.rows, (void*)S.exp_b, (void*)S.rows_b,
                    (void*)S.counters_base, (void*)S.run_len, (void*)S.expired, (void*)S.sel})
        if (p) (void)hipFree(p);
    uint64_t* keep = S.keep;
    S = PulseScratch();
    S.keep = keep;
    // (twice the index length: a growing index reallocates -- synchronously -- rarely; merged runs
    // sit at strides up to kPulseRun, so a level's runs may reach past the candidates by one stride)
    const uint64_t want = std::max<uint64_t>(2 * count, 1u << 18) + 2 * kPulseRun;
    const uint64_t cap = (want + kPulseRun - 1) / kPulseRun * kPulseRun;
    if (!(dev_alloc(ctx, &S.exp, cap, false) &&
          dev_alloc(ctx, &S.ts, cap, false) && dev_alloc(ctx, &S.rows, cap, false) &&
          dev_alloc(ctx, &S.exp_b, cap, false) && dev_alloc(ctx, &S.rows_b, cap, false) &&
          dev_alloc(ctx, &S.run_len, 2 * (cap / kPulseSortRun + 1), false) &&
          dev_alloc(ctx, &S.expired, 1, true) && dev_alloc(ctx, &S.counters_base, 16, false) &&
          dev_alloc(ctx, &S.sel, kPulseRun, false)))
        return TBG_ENOMEM;
    S.counters = S.counters_base;
    S.counters_next = S.counters_base + 8;
    S.capacity = cap;
    return 0;
}

template <typename Row>
int64_t dump_impl(tbg_ctx* ctx, const Row* rows, const uint8_t* live, uint64_t used, Row* out,
                  uint8_t* status_out) {
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

// ---- AccountEvents (events.hpp) ---------------------------------------------------------------

void free_ae_scratch(AeScratch& S) {
    GroupPlan& G = S.G;
    void* ptrs[] = {S.deltas, G.hkeys, G.hcnt, G.hoff, G.loc, G.rank, G.vals, G.vals_sorted, G.big,
                    G.counts, S.chunk_seg, S.chunk_tot};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    S = AeScratch{};
}

int alloc_ae_scratch(tbg_ctx* ctx, AeScratch& S, uint64_t cap) {
    const uint64_t slots = 2 * cap;  // grouping table load <= 0.5
    GroupPlan& G = S.G;
    if (!(dev_alloc(ctx, &S.deltas, cap, false) && dev_alloc(ctx, &G.hkeys, slots, true) &&
          dev_alloc(ctx, &G.hcnt, slots, true) && dev_alloc(ctx, &G.hoff, slots, false) &&
          dev_alloc(ctx, &G.loc, cap, false) && dev_alloc(ctx, &G.rank, cap, false) &&
          dev_alloc(ctx, &G.vals, cap, false) && dev_alloc(ctx, &G.vals_sorted, cap, false) &&
          dev_alloc(ctx, &G.big, cap / kGroupSmall + 1, false) && dev_alloc(ctx, &G.counts, 4, true) &&
          dev_alloc(ctx, &S.chunk_seg, cap / kAeChunk + cap / kGroupSmall + 1, false) &&
          dev_alloc(ctx, &S.chunk_tot, cap / kAeChunk + cap / kGroupSmall + 1, false)))
        return TBG_ENOMEM;
    G.hmask = slots - 1;
    return 0;
}

int ensure_ae_scratch(tbg_ctx* ctx, uint64_t touches) {
    if (touches <= ctx->ae_touch_cap) return 0;
    free_ae_scratch(ctx->ae);
    ctx->ae_touch_cap = 0;
    const uint64_t cap = std::max<uint64_t>(next_pow2(touches), 1u << 14);
    int rc = alloc_ae_scratch(ctx, ctx->ae, cap);
    if (rc) return rc;
    ctx->ae_touch_cap = cap;
    return 0;
}

// The call's stream waits for the side stream's appends (GPU-side; no host synchronisation).
int ae_flush_graph(tbg_ctx* ctx);
int ae_flush_all(tbg_ctx* ctx);

int ae_join(tbg_ctx* ctx) {
    if (int rc = ae_flush_all(ctx)) return rc;
    if (!ctx->ae_async_pending) return 0;
    if (hipEventQuery(ctx->ae_done[ctx->ae_parity ^ 1]) != hipSuccess)
        HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ae_done[ctx->ae_parity ^ 1], 0));
    ctx->ae_async_pending = false;
    return 0;
}

// The host's view of the log (ae_used / ae_last_ts / ae_sorted) after the appends in flight.
int ae_settle(tbg_ctx* ctx) {
    if (int rc = ae_join(ctx)) return rc;
    if (!ctx->ae_pending) return 0;
    unsigned long long st[4] = {0, 0, 0, 0};
    HIP_TRY(ctx, hipMemcpyAsync(st, ctx->ae_words + 4, 32, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    if (st[3]) {  // (an append found no room on device and wrote nothing: the bound was wrong)
        ctx->error = "account_events capacity exceeded (device check)";
        ctx->failed = true;
        return TBG_ENOSPC;
    }
    ctx->ae_used = ctx->ae_bound = st[0];
    ctx->ae_last_ts = st[1];
    ctx->ae_sorted = st[2] == 0;
    ctx->ae_pending = false;
    return 0;
}

// Sets the device's view of the log from the host's (open / restore / after a sort).
int ae_publish(tbg_ctx* ctx) {
    if (int rc = ae_join(ctx)) return rc;
    const unsigned long long st[3] = {ctx->ae_used, ctx->ae_last_ts, ctx->ae_sorted ? 0ull : 1ull};
    HIP_TRY(ctx, hipMemcpyAsync(ctx->ae_words + 4, st, 24, hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // (`st` is a stack value)
    ctx->ae_bound = ctx->ae_used;
    ctx->ae_pending = false;
    return 0;
}

// Appends the AccountEvents of up to `n_upper` events (the exact count at d_count, or n_upper
// itself when d_count is null): `collect` writes their event-level fields and groups both touches
// of each by account (events.hpp); the account halves follow from the final rows and the later
// touches' sums per account. No host synchronisation: the block's position in the log and the
// log's length advance on device (ae_tail); the host synchronises only when the upper bound of
// the length could pass the capacity.
template <typename Collect>
int ae_append(tbg_ctx* ctx, uint32_t n_upper, const unsigned int* d_count, Collect collect,
              const char* mark = "account_events") {
    if (n_upper == 0) return 0;
    if (int rc = ae_join(ctx)) return rc;
    if (ctx->ae_bound + n_upper > ctx->ae_cap) {
        int rc = ae_settle(ctx);
        if (rc) return rc;
        unsigned int m = n_upper;
        if (d_count) {
            HIP_TRY(ctx, hipMemcpyAsync(&m, d_count, 4, hipMemcpyDeviceToHost, ctx->stream));
            HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        }
        if (ctx->ae_used + m > ctx->ae_cap) {
            ctx->error = "account_events capacity exceeded";
            return TBG_ENOSPC;
        }
    }
    int rc = ensure_ae_scratch(ctx, 2 * uint64_t(n_upper));
    if (rc) return rc;
    AeScratch& S = ctx->ae;
    S.state = ctx->ae_words + 4;
    S.cap = ctx->ae_cap;
    const uint64_t slots = S.G.hmask + 1;
    tb_account_event_t* log = ctx->ae_log;  // (+ the device length, read by each kernel)
    tmark(ctx, "-account_events");
    collect(S, log, ctx->ae_ref);
    rc = launch_scan(ctx, slots, ExclusiveSumU32{S.G.hcnt, S.G.hoff, &S.G.counts[0]});
    if (rc) return rc;
    const uint64_t pairs = 2 * uint64_t(n_upper);
    hipLaunchKernelGGL(group_scatter, dim3(grid_for(pairs)), dim3(kBlock), 0, ctx->stream, S.G, pairs);
    hipLaunchKernelGGL(ae_group_small, dim3(grid_for(slots)), dim3(kBlock), 0, ctx->stream, ctx->T,
                       S, slots, log);
    hipLaunchKernelGGL(ae_group_sort, dim3(kGroupBigBlocks), dim3(kGroupBigThreads), 0, ctx->stream,
                       S);
    hipLaunchKernelGGL(ae_chunk_totals, dim3(kAeChunkBlocks), dim3(kGroupBigThreads), 0,
                       ctx->stream, S);
    hipLaunchKernelGGL(ae_chunk_emit, dim3(kAeChunkBlocks), dim3(kGroupBigThreads), 0, ctx->stream,
                       ctx->T, S, log);
    hipLaunchKernelGGL(ae_tail, dim3(1), dim3(64), 0, ctx->stream, log, d_count, n_upper, S.state);
    tmark(ctx, mark);
    HIP_TRY(ctx, hipGetLastError());
    ctx->ae_bound += n_upper;
    ctx->ae_pending = true;
    return 0;
}

// The side stream's appends of staging buffer p (ae_append's sequence over the staging, at its
// fixed upper bound kAeAsyncMax): number the created events, copy and group, place, emit. The two
// chained scans use their own status words and ticket (ae_g_words[7 ..]), which ae_scatter_tail
// clears for the next append.
// which: 0 both paths (ae_small_emit takes the staging unless an event needs the general appends,
// which then run; else they skip), 1 ae_small_emit only, 2 the general appends only (the host
// knows from the snapshot which one the staging needs).
int ae_launch_appends(tbg_ctx* ctx, uint32_t p, uint32_t epoch, bool pending, int which = 0) {
    hipStream_t st = ctx->ae_stream;
    // The one-pass appends first (ae_small_emit); they take the call unless the staging holds an
    // event they cannot, and then every kernel below skips it.
    const bool small = which != 2 && ctx->ae_window_on && ctx->T.acc_rows_used <= kAeWinRowsMax;
    const unsigned int* handled = ctx->ae_stage[p].words + 1;
    if (small) {
        AeSmall A{ctx->ae_stage[p], epoch, uint32_t(ctx->T.acc_rows_used), pending ? 1u : 0u,
                  ctx->ae_log, ctx->ae_ref, ctx->ae_words + 4, ctx->ae_small_counts,
                  ctx->ae_small_ts, ctx->ae_cap};
        hipLaunchKernelGGL(ae_small_emit, dim3(kAeSmallWgs), dim3(kAeSmallThreads), 0, st, A);
        if (which == 1) {
            HIP_TRY(ctx, hipGetLastError());
            return 0;
        }
    }
    AeScratch S = ctx->ae_g;
    S.state = ctx->ae_words + 4;
    S.cap = ctx->ae_cap;
    S.pos = nullptr;
    S.skip = small ? handled : nullptr;
    S.skip_if = epoch;
    AeScratch Se = S;  // the emit kernels: the block's base (kept by ae_scatter_tail), event-
    Se.state = ctx->ae_g_words + 2;  // numbered touches and the staged deltas
    Se.pos = ctx->ae_pos;
    Se.deltas = ctx->ae_stage[p].delta;
    unsigned int* d_count = reinterpret_cast<unsigned int*>(ctx->ae_g_words);
    unsigned long long* scan_words = ctx->ae_g_words + 8;
    unsigned int* ticket = reinterpret_cast<unsigned int*>(ctx->ae_g_words + 7);
    const uint64_t slots = S.G.hmask + 1;
    const uint32_t tiles1 = (kAeAsyncMax + kScanTile - 1) / kScanTile;
    const uint32_t tiles2 = uint32_t((slots + kScanTile - 1) / kScanTile);
    hipLaunchKernelGGL(chained_scan<PositionsOf8>, dim3(tiles1), dim3(kScanThreads), 0, st,
                       uint64_t(kAeAsyncMax), PositionsOf8{ctx->ae_stage[p].created, ctx->ae_pos, d_count},
                       ScanState{scan_words, ticket, 0, 1, S.skip, epoch});
    hipLaunchKernelGGL(ae_copy_group, dim3((kAeAsyncMax + kPlanThreads - 1) / kPlanThreads),
                       dim3(kPlanThreads), 0, st, ctx->ae_stage[p], ctx->ae_pos, d_count, S, ctx->ae_log,
                       ctx->ae_ref);
    hipLaunchKernelGGL(chained_scan<ExclusiveSumU32>, dim3(tiles2), dim3(kScanThreads), 0, st,
                       slots, ExclusiveSumU32{S.G.hcnt, S.G.hoff, &S.G.counts[0]},
                       ScanState{scan_words + tiles1, ticket, tiles1, 2, S.skip, epoch});
    const uint64_t pairs = 2 * uint64_t(kAeAsyncMax);
    hipLaunchKernelGGL(ae_scatter_tail, dim3(grid_for(pairs)), dim3(kBlock), 0, st, S.G, pairs,
                       ctx->ae_log, d_count, S.state, ctx->ae_g_words + 2, ctx->ae_g_words + 7,
                       1 + tiles1 + tiles2, S.skip, epoch);
    hipLaunchKernelGGL(ae_group_small, dim3(grid_for(slots)), dim3(kBlock), 0, st, ctx->T, Se, slots,
                       ctx->ae_log);
    hipLaunchKernelGGL(ae_group_big_serial, dim3(2 * kAeAsyncMax / (kGroupMid + 1) + 1),
                       dim3(kGroupBigThreads), 0, st, Se, ctx->ae_log);
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

int ensure_ae_async(tbg_ctx* ctx) {
    if (ctx->ae_async_ready) return 0;
    const uint64_t cap = 2 * uint64_t(kAeAsyncMax);
    for (int p = 0; p < 2; p++) {
        AeStage& st = ctx->ae_stage[p];
        if (!(dev_alloc(ctx, &st.rec, kAeAsyncMax, false) && dev_alloc(ctx, &st.ref, kAeAsyncMax, false) &&
              dev_alloc(ctx, &st.delta, 2 * kAeAsyncMax, false) &&
              dev_alloc(ctx, &st.created, kAeAsyncMax, true) && dev_alloc(ctx, &st.words, 4, true)))
            return TBG_ENOMEM;
    }
    if (!(dev_alloc(ctx, &ctx->ae_pos, kAeAsyncMax, false) && dev_alloc(ctx, &ctx->ae_g_words, 64, true) &&
          dev_alloc(ctx, &ctx->ae_small_counts, kAeSmallWgs + 1, true) &&
          dev_alloc(ctx, &ctx->ae_small_ts, 2 * kAeSmallWgs, false)))
        return TBG_ENOMEM;
    if (int rc = alloc_ae_scratch(ctx, ctx->ae_g, cap)) return rc;
    // (the scans' words: 8 + tiles of both scans)
    if ((cap * 2 + kScanTile - 1) / kScanTile + (kAeAsyncMax + kScanTile - 1) / kScanTile + 8 > 64)
        return TBG_EINVAL;
    HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->ae_stream, hipStreamNonBlocking));
    for (int p = 0; p < 2; p++) {
        HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->ae_snap_ready[p], hipEventDisableTiming));
        HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->ae_done[p], hipEventDisableTiming));
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // (the scratch's zeroing)
    ctx->ae_async_ready = true;
    return 0;
}

// Can call c's appends go to the side stream? (a small call; the log's capacity checked on the
// host's upper bound; not while kernels are being timed)
bool ae_async_ok(const tbg_ctx* ctx, uint32_t n) {
    return ctx->ae_log && ctx->ae_async && !ctx->timing && n <= kAeAsyncMax &&
           ctx->ae_bound + n <= ctx->ae_cap;
}

// The snapshot job of the next small call (buffer ctx->ae_parity), after the call's stream waited
// for that buffer's previous graph.
// The staging buffer of the next appends (ctx->ae_parity), once the call's stream waited for its
// previous appends.
int ae_flush_graph(tbg_ctx* ctx);
int ae_flush_all(tbg_ctx* ctx);

int ae_stage_acquire(tbg_ctx* ctx) {
    if (int rc = ae_flush_all(ctx)) return rc;
    if (int rc = ensure_ae_async(ctx)) return rc;
    const uint32_t p = ctx->ae_parity;
    // (a wait on an event that has already completed still puts a barrier packet on the call's
    // stream: skipped when the appends two calls back are done)
    if (ctx->ae_done_recorded[p] && (hipEventQuery(ctx->ae_done[p]) != hipSuccess))
        HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, ctx->ae_done[p], 0));
    return 0;
}

// (the snapshots: one wave a workgroup, 128 workgroups -- the event's dependent loads spread over
// more CUs than 32 workgroups of four waves)
constexpr uint32_t kSnapThreads = 64;

int ae_snap_job(tbg_ctx* ctx, const Call<tb_transfer_t>& c, AeSnapJob* J) {
    if (int rc = ae_stage_acquire(ctx)) return rc;
    *J = AeSnapJob{ctx->T, c, ctx->ae_stage[ctx->ae_parity], false};
    return 0;
}

// The side stream appends staging buffer p (at most n AccountEvents) once the call's stream
// reaches this point. The log's bound grows as the graph is queued: a call that fails later still
// leaves a graph that may append.
int ae_launch_graph(tbg_ctx* ctx, uint32_t n, uint32_t epoch, bool pending = false) {
    const uint32_t p = ctx->ae_parity;
    ctx->ae_bound += n;
    ctx->ae_pending = true;
    HIP_TRY(ctx, hipEventRecord(ctx->ae_snap_ready[p], ctx->stream));
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->ae_stream, ctx->ae_snap_ready[p], 0));
    if (int rc = ae_launch_appends(ctx, p, epoch, pending)) return rc;
    HIP_TRY(ctx, hipEventRecord(ctx->ae_done[p], ctx->ae_stream));
    ctx->ae_done_recorded[p] = true;
    ctx->ae_parity = p ^ 1;
    ctx->ae_async_pending = true;
    return 0;
}

// ae_launch_graph in two halves: the bound, the snapshot's event and the parity now; the side
// stream's launches at ae_flush_graph.
int ae_defer_graph(tbg_ctx* ctx, uint32_t n, uint32_t epoch, bool pending) {
    const uint32_t p = ctx->ae_parity;
    ctx->ae_bound += n;
    ctx->ae_pending = true;
    HIP_TRY(ctx, hipEventRecord(ctx->ae_snap_ready[p], ctx->stream));
    ctx->ae_graph_deferred = true;
    ctx->ae_def_parity = p;
    ctx->ae_def_epoch = epoch;
    ctx->ae_def_pending = pending;
    ctx->ae_def_call = false;
    ctx->ae_parity = p ^ 1;
    return 0;
}
int ae_flush_graph(tbg_ctx* ctx) {
    if (!ctx->ae_graph_deferred) return 0;
    ctx->ae_graph_deferred = false;
    const uint32_t p = ctx->ae_def_parity;
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->ae_stream, ctx->ae_snap_ready[p], 0));
    // (the pulse synchronised after its snapshot: the pinned word says which appends it needs; a
    // small call's snapshot has usually completed by the next call -- else every path is queued
    // and the ones the staging does not need skip on device)
    const bool small_ok = ctx->ae_window_on && ctx->T.acc_rows_used <= kAeWinRowsMax;
    int which = !small_ok ? 0 : ctx->h_pulse[3] == ctx->ae_def_epoch ? 2 : 1;
    if (ctx->ae_def_call) {
        const bool known = small_ok && hipEventQuery(ctx->ae_snap_ready[p]) == hipSuccess;
        which = !known ? 0 : __atomic_load_n(&ctx->h_pulse[4], __ATOMIC_ACQUIRE) == ctx->ae_def_epoch ? 2 : 1;
    }
    if (int rc = ae_launch_appends(ctx, p, ctx->ae_def_epoch, ctx->ae_def_pending, which)) return rc;
    HIP_TRY(ctx, hipEventRecord(ctx->ae_done[p], ctx->ae_stream));
    ctx->ae_done_recorded[p] = true;
    ctx->ae_async_pending = true;
    return 0;
}

// Every deferred side-stream job (a pulse's appends).
int ae_flush_all(tbg_ctx* ctx) { return ae_flush_graph(ctx); }

// AccountEvents of a small create_transfers call behind the next call. When no replay ran, the
// call's stage_out took the snapshot and the graph is already queued behind it; else the snapshot
// is taken now (the speculative graph found no created flags and appended nothing).
int ae_transfers_async(tbg_ctx* ctx, const Call<tb_transfer_t>& c) {
    if (!ctx->ae_snap_early) {
        AeSnapJob J;
        if (int rc = ae_snap_job(ctx, c, &J)) return rc;
        hipLaunchKernelGGL(ae_snapshot, dim3(kAeAsyncMax / kSnapThreads), dim3(kSnapThreads), 0, ctx->stream, J);
        HIP_TRY(ctx, hipGetLastError());
        if (int rc = ae_launch_graph(ctx, c.n, c.epoch)) return rc;
    }
    ctx->ae_snap_early = false;
    return 0;
}

// AccountEvents of a balance-window call in one pass (events.hpp, ae_window_emit), when the call
// qualifies: its window partials are still current (nothing ran since), no replay ran, and no
// flag says an event or a sum is outside what the window emit tracks. Returns 1 when not taken.
int ae_window_wide(tbg_ctx* ctx, const Call<tb_transfer_t>& c);
int ae_window(tbg_ctx* ctx, const Call<tb_transfer_t>& c) {
    const DevScalars& h = *ctx->h_scalars;
    constexpr unsigned int kNot = kFlagChain | kFlagPostVoid | kFlagImported | kFlagAeSlow;
    if (ctx->win.epoch != c.epoch || ctx->epoch != c.epoch || (h.flags & kNot) || h.stats[0] ||
        ctx->T.acc_rows_used > kAeWinRowsMax || !ctx->ae_window_on)
        return 1;
    if (int rc = ae_join(ctx)) return rc;
    if (ctx->ae_bound + c.n > ctx->ae_cap) {
        if (int rc = ae_settle(ctx)) return rc;
        if (ctx->ae_used + c.n > ctx->ae_cap) return 1;  // (the general path counts exactly)
    }
    if (h.flags & (kFlagWideItems | kFlagWideSums)) return ae_window_wide(ctx, c);
    AeWindow W{};
    W.items = ctx->bal_items;
    W.results = c.results;
    W.acc_rows = ctx->T.acc_rows;
    W.n = c.n;
    W.ps = ctx->win.ps;
    W.rows = uint32_t(ctx->T.acc_rows_used);
    W.nwg = ctx->win.nwg;
    W.wkeys = ctx->win.wkeys;
    W.row_base = c.row_base;
    W.suffix = ctx->window_partials;
    W.slice_count = ctx->window_counts;
    W.slice_ts = ctx->window_ts;
    W.done = ctx->window_counts + kWindowGridMax;
    W.log = ctx->ae_log;
    W.refs = ctx->ae_ref;
    W.state = ctx->ae_words + 4;
    W.cap = ctx->ae_cap;
    tmark(ctx, "-account_events");
    hipLaunchKernelGGL(ae_window_suffix, dim3(std::max<uint32_t>(1, (2 * W.rows + kBlock - 1) / kBlock)), dim3(kBlock), 0,
                       ctx->stream, W);
    hipLaunchKernelGGL(ae_window_emit, dim3(W.nwg), dim3(kAeWinThreads), 0, ctx->stream, W);
    tmark(ctx, "account_events");
    HIP_TRY(ctx, hipGetLastError());
    ctx->win.epoch = 0;  // (the partials are suffix sums now)
    ctx->stats.ae_window = 1;
    ctx->ae_bound += c.n;
    ctx->ae_pending = true;
    return 0;
}

// AccountEvents of a balance-window call whose amounts or sums are too wide for ae_window_emit's
// u32 later-sums (events.hpp, ae_wide_*): per-slice sums, their suffix over the slices, and the
// emit's rounds from the last one back with the account state in HBM. ae_window checked the rest.
int ae_window_wide(tbg_ctx* ctx, const Call<tb_transfer_t>& c) {
    const uint32_t rows = uint32_t(ctx->T.acc_rows_used);
    const uint32_t per = ae_wide_per(c.n);
    const uint32_t slices = (c.n + per - 1) / per;
    // (sized once for the context's largest call and the window's row limit: no reallocation)
    const uint64_t bmax = std::max<uint64_t>(ctx->opt.batch_events_max, c.n);
    const uint32_t slices_max = std::max<uint32_t>(
        slices, uint32_t((bmax + ae_wide_per(uint32_t(bmax)) - 1) / ae_wide_per(uint32_t(bmax))));
    const uint32_t slices_alloc = std::max<uint32_t>(slices_max, kAeWideGrid);
    const uint64_t words = 2 * uint64_t(slices) * std::max<uint32_t>(rows, 1);
    if (words > ctx->ae_wide_sums_cap) {
        const uint64_t alloc_words = std::max<uint64_t>(words, 2 * uint64_t(slices_alloc) * kAeWinRowsMax);
        if (ctx->ae_wide_sums) HIP_TRY(ctx, hipFree(ctx->ae_wide_sums));
        ctx->ae_wide_sums = nullptr;
        ctx->ae_wide_sums_cap = 0;
        if (!dev_alloc(ctx, &ctx->ae_wide_sums, alloc_words, false)) return TBG_ENOMEM;
        ctx->ae_wide_sums_cap = alloc_words;
    }
    if (slices > ctx->ae_wide_slices_cap) {
        for (void* q : {(void*)ctx->ae_wide_counts, (void*)ctx->ae_wide_ts})
            if (q) HIP_TRY(ctx, hipFree(q));
        ctx->ae_wide_counts = nullptr;
        ctx->ae_wide_ts = nullptr;
        ctx->ae_wide_slices_cap = 0;
        if (!(dev_alloc(ctx, &ctx->ae_wide_counts, slices_alloc + 1, true) &&
              dev_alloc(ctx, &ctx->ae_wide_ts, 2 * uint64_t(slices_alloc), false)))
            return TBG_ENOMEM;
        ctx->ae_wide_slices_cap = slices_alloc;
    }
    AeWide A{};
    A.items = ctx->bal_items;
    A.amounts = c.ev_amount;
    A.results = c.results;
    A.acc_rows = ctx->T.acc_rows;
    A.n = c.n;
    A.ps = ctx->win.ps;
    A.rows = rows;
    A.slices = slices;
    A.per = per;
    A.row_base = c.row_base;
    A.sums = ctx->ae_wide_sums;
    A.slice_count = ctx->ae_wide_counts;
    A.slice_ts = ctx->ae_wide_ts;
    A.done = ctx->ae_wide_counts + ctx->ae_wide_slices_cap;
    A.log = ctx->ae_log;
    A.refs = ctx->ae_ref;
    A.state = ctx->ae_words + 4;
    A.cap = ctx->ae_cap;
    tmark(ctx, "-account_events");
    hipLaunchKernelGGL(ae_wide_partials, dim3(2 * slices), dim3(kAeWideThreads), 0, ctx->stream, A);
    hipLaunchKernelGGL(ae_wide_suffix, dim3(std::max<uint32_t>(1, (2 * rows + kBlock - 1) / kBlock)),
                       dim3(kBlock), 0, ctx->stream, A);
    hipLaunchKernelGGL(ae_wide_emit, dim3(slices), dim3(kAeWideThreads), 0, ctx->stream, A);
    tmark(ctx, "account_events");
    HIP_TRY(ctx, hipGetLastError());
    ctx->win.epoch = 0;
    ctx->stats.ae_window = 3;
    ctx->ae_bound += c.n;
    ctx->ae_pending = true;
    return 0;
}

// AccountEvents of a general call in one pass over dense key spaces (events.hpp, ae_dense_*):
// staged, summed per slice, suffix-summed; the call is refused (1: the general appends take it)
// when an event flips `closed` or moves 2^19 or more, or a later-delta sum leaves the i32 range.
constexpr uint32_t kAeDenseMax = 1u << 18;  // events per call
// Its first half (stage, partials, suffix, the refusal word to pinned memory), launched before the
// host's next synchronisation: by create_transfers after a replay, right before end_call's sync, so
// the refusal is known without a synchronisation of its own. 1: not eligible.
int ae_dense_prefix(tbg_ctx* ctx, const Call<tb_transfer_t>& c) {
    if (!ctx->ae_window_on || ctx->T.acc_rows_used > kAeWinRowsMax || c.n > kAeDenseMax ||
        c.n > ctx->opt.batch_events_max)
        return 1;
    if (!ctx->ae_dense_touch) {
        const uint64_t cap = std::min<uint64_t>(kAeDenseMax, ctx->opt.batch_events_max);
        const uint64_t slices = (cap + kAeDenseSlice - 1) / kAeDenseSlice;
        if (!(dev_alloc(ctx, &ctx->ae_dense_touch, cap, false) &&
              dev_alloc(ctx, &ctx->ae_dense_ev, 5 * cap, false) &&
              dev_alloc(ctx, &ctx->ae_dense_partials, 2 * slices * 2 * kAeWinRowsMax, false) &&
              dev_alloc(ctx, &ctx->ae_dense_counts, slices + 1, true) &&
              dev_alloc(ctx, &ctx->ae_dense_ts, 2, false) &&
              dev_alloc(ctx, &ctx->ae_dense_later, 2 * cap, false) &&
              dev_alloc(ctx, &ctx->ae_dense_pos, cap, false) &&
              dev_alloc(ctx, &ctx->ae_dense_claim, 4, true)))
            return TBG_ENOMEM;
        // (ae_dense_records' min / max words; a kernel on the stream: a synchronous copy waited for
        // every stream, ~10 ms inside config 4's first dense call)
        hipLaunchKernelGGL(ae_dense_ts_init, dim3(1), dim3(64), 0, ctx->stream, ctx->ae_dense_ts);
    }
    if (int rc = ae_join(ctx)) return rc;
    if (ctx->ae_bound + c.n > ctx->ae_cap) {
        if (int rc = ae_settle(ctx)) return rc;
        if (ctx->ae_used + c.n > ctx->ae_cap) return 1;  // (the general path counts exactly)
    }
    AeDense& A = ctx->ae_dense_job;
    A = AeDense{};
    A.T = ctx->T;
    A.c = c;
    A.rows = uint32_t(ctx->T.acc_rows_used);
    A.slices = (c.n + kAeDenseSlice - 1) / kAeDenseSlice;
    A.touch = reinterpret_cast<AeTouch*>(ctx->ae_dense_touch);
    A.ev = ctx->ae_dense_ev;
    A.partials = ctx->ae_dense_partials;
    A.slice_count = ctx->ae_dense_counts;
    A.done = ctx->ae_dense_counts + (std::min<uint64_t>(kAeDenseMax, ctx->opt.batch_events_max) +
                                     kAeDenseSlice - 1) / kAeDenseSlice;
    A.slice_ts = ctx->ae_dense_ts;
    A.later = ctx->ae_dense_later;
    A.pos = ctx->ae_dense_pos;
    // (the refusal word is written straight to pinned memory: no report kernel)
    A.fail = reinterpret_cast<unsigned int*>(ctx->dh_pulse + 2);
    A.claim = ctx->ae_dense_claim;
    static_assert(__BYTE_ORDER__ == __ORDER_LITTLE_ENDIAN__, "the word's low half");
    A.epoch = c.epoch;
    A.log = ctx->ae_log;
    A.refs = ctx->ae_ref;
    A.state = ctx->ae_words + 4;
    A.cap = ctx->ae_cap;
    tmark(ctx, "-account_events");
    hipLaunchKernelGGL(ae_dense_stage, dim3(grid_for(c.n)), dim3(kBlock), 0, ctx->stream, A);
    hipLaunchKernelGGL(ae_dense_partials, dim3(2 * A.slices), dim3(kAeWinThreads), 0, ctx->stream, A);
    hipLaunchKernelGGL(ae_dense_suffix, dim3(std::max<uint32_t>(1, (4 * A.rows + 63) / 64)),
                       dim3(kAeSufThreads), 0, ctx->stream, A);
    tmark(ctx, "account_events");
    HIP_TRY(ctx, hipGetLastError());
    ctx->ae_dense_prefixed = c.epoch;
    return 0;
}

int ae_dense(tbg_ctx* ctx, const Call<tb_transfer_t>& c) {
    if (ctx->ae_dense_prefixed != c.epoch) {
        const int rc = ae_dense_prefix(ctx, c);
        if (rc) return rc;
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    ctx->ae_dense_prefixed = 0;
    if (uint32_t(ctx->h_pulse[2]) == c.epoch) return 1;  // (ae_dense_stage / _suffix wrote it)
    const AeDense& A = ctx->ae_dense_job;
    tmark(ctx, "-account_events");
    hipLaunchKernelGGL(ae_dense_later, dim3(A.slices), dim3(kAeDenseEmitThreads), 0, ctx->stream, A);
    hipLaunchKernelGGL(ae_dense_records, dim3((c.n + kAeDenseRecThreads - 1) / kAeDenseRecThreads),
                       dim3(kAeDenseRecThreads), 0, ctx->stream, A);
    tmark(ctx, "account_events");
    HIP_TRY(ctx, hipGetLastError());
    ctx->stats.ae_window = 2;
    ctx->ae_bound += c.n;
    ctx->ae_pending = true;
    return 0;
}

// AccountEvents of a create_transfers call: its created events in call order.
int ae_transfers(tbg_ctx* ctx, const Call<tb_transfer_t>& c) {
    if (ctx->ae_snap_early) {  // (stage_out took the snapshot and its graph is queued)
        ctx->ae_snap_early = false;
        return 0;
    }
    const int wrc = ae_window(ctx, c);
    if (wrc <= 0) return wrc;
    if (ae_async_ok(ctx, c.n)) return ae_transfers_async(ctx, c);
    const int drc = ae_dense(ctx, c);
    if (drc <= 0) return drc;
    ctx->ae_snap_early = false;
    unsigned int* d_count = reinterpret_cast<unsigned int*>(ctx->ae_words);
    int rc = launch_scan(ctx, c.n, SelectCreated{c.results, ctx->ae_list, d_count});
    if (rc) return rc;
    const uint32_t* list = ctx->ae_list;
    return ae_append(ctx, c.n, d_count, [&](const AeScratch& S, tb_account_event_t* log,
                                           AeRef* refs) {
        hipLaunchKernelGGL(ae_collect_transfers, dim3((c.n + kPlanThreads - 1) / kPlanThreads),
                           dim3(kPlanThreads), 0, ctx->stream, ctx->T, c, list, d_count, S, log,
                           refs);
    });
}

// AccountEvents of a pulse: the expired rows in expiry order.
// (m: the count, or its upper bound when d_count holds it on device)
int ae_expiry(tbg_ctx* ctx, const uint64_t* rows, uint64_t m, uint64_t timestamp,
              const uint64_t* d_stamps = nullptr, const unsigned int* d_count = nullptr) {
    return ae_append(ctx, uint32_t(m), d_count, [&](const AeScratch& S, tb_account_event_t* log,
                                                    AeRef* refs) {
        hipLaunchKernelGGL(ae_collect_expiry, dim3((uint32_t(m) + kPlanThreads - 1) / kPlanThreads),
                           dim3(kPlanThreads), 0, ctx->stream, ctx->T, rows, uint32_t(m), d_count,
                           timestamp, d_stamps, S, log, refs);
    }, "pulse:account_events");
}


// Restores timestamp order of the log (stable) when an append broke it.
int ae_sort_log(tbg_ctx* ctx) {
    int rc = ae_settle(ctx);
    if (rc) return rc;
    if (ctx->ae_sorted) return 0;
    if (ctx->ae_used < 2) {
        ctx->ae_sorted = true;
        return ae_publish(ctx);
    }
    const uint64_t n = ctx->ae_used;
    uint64_t *keys = nullptr, *keys2 = nullptr, *starts = nullptr;
    uint32_t *idx = nullptr, *idx2 = nullptr, *list = nullptr;
    uint8_t* run_first = nullptr;
    tb_account_event_t* log2 = nullptr;
    AeRef* ref2 = nullptr;
    if (!(dev_alloc(ctx, &keys, n, false) && dev_alloc(ctx, &keys2, n, false) &&
          dev_alloc(ctx, &idx, n, false) && dev_alloc(ctx, &idx2, n, false) &&
          dev_alloc(ctx, &run_first, n, false) && dev_alloc(ctx, &list, n, false) &&
          dev_alloc(ctx, &starts, n + 1, false) &&
          dev_alloc(ctx, &log2, n, false) && dev_alloc(ctx, &ref2, n, false)))
        rc = TBG_ENOMEM;
    if (!rc) {
        // the natural runs (each appended block is in order), merged pairwise
        hipLaunchKernelGGL(ae_sort_keys, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream,
                           ctx->ae_log, n, keys, idx, run_first);
        unsigned int* d_count = &ctx->d_scalars->slow_count;  // scratch word (between calls)
        rc = select_flagged(ctx, run_first, n, list, d_count);
        unsigned int runs = 0;
        if (!rc && (hipMemcpyAsync(&runs, d_count, 4, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
                    hipStreamSynchronize(ctx->stream) != hipSuccess))
            rc = TBG_EHIP;
        std::vector<uint32_t> first(runs);
        if (!rc && runs && hipMemcpy(first.data(), list, runs * 4ull, hipMemcpyDeviceToHost) != hipSuccess)
            rc = TBG_EHIP;
        std::vector<uint64_t> st(first.begin(), first.end());
        st.push_back(n);
        while (!rc && runs > 1) {
            if (hipMemcpy(starts, st.data(), st.size() * 8, hipMemcpyHostToDevice) != hipSuccess) {
                rc = TBG_EHIP;
                break;
            }
            const uint64_t lanes = (n + kMergePer - 1) / kMergePer;
            hipLaunchKernelGGL(ae_merge_pass, dim3(grid_for(lanes)), dim3(kBlock), 0, ctx->stream,
                               keys, idx, starts, runs, n, keys2, idx2);
            if (hipStreamSynchronize(ctx->stream) != hipSuccess) rc = TBG_EHIP;
            std::swap(keys, keys2);
            std::swap(idx, idx2);
            std::vector<uint64_t> next;
            for (uint32_t r = 0; r < runs; r += 2) next.push_back(st[r]);
            next.push_back(n);
            st.swap(next);
            runs = (runs + 1) / 2;
        }
        if (!rc) {
            hipLaunchKernelGGL(ae_permute, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream,
                               ctx->ae_log, ctx->ae_ref, idx, n, log2, ref2);
            if (hipMemcpyAsync(ctx->ae_log, log2, n * sizeof(tb_account_event_t),
                               hipMemcpyDeviceToDevice, ctx->stream) != hipSuccess ||
                hipMemcpyAsync(ctx->ae_ref, ref2, n * sizeof(AeRef), hipMemcpyDeviceToDevice,
                               ctx->stream) != hipSuccess ||
                hipStreamSynchronize(ctx->stream) != hipSuccess)
                rc = TBG_EHIP;
        }
    }
    for (void* p : {(void*)run_first, (void*)list, (void*)starts})
        if (p) (void)hipFree(p);
    for (void* p : {(void*)keys, (void*)keys2, (void*)idx, (void*)idx2, (void*)log2, (void*)ref2})
        if (p) (void)hipFree(p);
    if (rc) return rc;
    ctx->ae_sorted = true;
    return ae_publish(ctx);
}

// The GPU's address of host range [p, p + bytes) if it lies in a registered range, else null.
template <typename T>
T* mapped(const tbg_ctx* ctx, T* p, uint64_t bytes) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    for (const auto& r : ctx->registered)
        if (a >= r.host && a + bytes <= r.host + r.size) return reinterpret_cast<T*>(r.dev + (a - r.host));
    return nullptr;
}
bool is_registered(const tbg_ctx* ctx, const void* p, uint64_t bytes) {
    return mapped(ctx, p, bytes) != nullptr;
}

// Process-wide registrations of host ranges (tbg_register_host): one hipHostRegister per range
// start, counted over the ctxs using it. A range that HIP reports as already registered by
// someone else (not through this registry) is used but never unregistered here.
struct HostPin {
    uint64_t size;
    uintptr_t dev;
    uint32_t users;
    bool owned;
};
std::mutex& host_pins_mu() {
    static std::mutex m;
    return m;
}
std::map<uintptr_t, HostPin>& host_pins() {
    static std::map<uintptr_t, HostPin> m;
    return m;
}

bool host_pin_acquire(tbg_ctx* ctx, void* ptr, uint64_t size, uintptr_t* dev_out) {
    std::lock_guard<std::mutex> g(host_pins_mu());
    auto& pins = host_pins();
    const uintptr_t a = reinterpret_cast<uintptr_t>(ptr);
    auto it = pins.find(a);
    if (it != pins.end()) {
        if (size > it->second.size) {
            ctx->error = "tbg_register_host: range overlaps a smaller registration at the same start";
            return false;
        }
        it->second.users++;
        *dev_out = it->second.dev;
        return true;
    }
    const hipError_t e = hipHostRegister(ptr, size, hipHostRegisterMapped);
    const bool owned = e == hipSuccess;
    if (!owned) {
        (void)hipGetLastError();  // (clears the error for later calls)
        if (e != hipErrorHostMemoryAlreadyRegistered) return hip_ok(ctx, e, "hipHostRegister");
    }
    void* dev = nullptr;
    if (hipHostGetDevicePointer(&dev, ptr, 0) != hipSuccess || !dev) {
        (void)hipGetLastError();
        if (owned) (void)hipHostUnregister(ptr);
        ctx->error = "hipHostGetDevicePointer";
        return false;
    }
    pins[a] = HostPin{size, reinterpret_cast<uintptr_t>(dev), 1, owned};
    *dev_out = reinterpret_cast<uintptr_t>(dev);
    return true;
}

void host_pin_release(void* ptr) {
    std::lock_guard<std::mutex> g(host_pins_mu());
    auto& pins = host_pins();
    auto it = pins.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == pins.end() || --it->second.users) return;
    if (it->second.owned) (void)hipHostUnregister(ptr);
    pins.erase(it);
}

// A host-buffer call's inputs into HBM: the batch ends / timestamps from the pinned staging and,
// when the body lies in a registered range, the body itself -- one kernel on the call's stream
// (hostio.hpp); an unregistered body takes hipMemcpyAsync.
int ae_flush_all(tbg_ctx* ctx);

// Chooses the host-buffer call's body buffer (ctx->body_dst).
int body_buffer(tbg_ctx* ctx) {
    ctx->body_dst = ctx->d_events;
    return 0;
}

int stage_call_inputs(tbg_ctx* ctx, const void* events, uint64_t bytes, uint32_t nb,
                      bool reset_scalars, bool ingest_reads_host = false) {
    const uint4* src = mapped(ctx, static_cast<const uint4*>(events), bytes);
    ctx->events_host = nullptr;
    ctx->batches_host = false;
    // A small create_transfers call's registered body is read by tr_ingest itself across PCIe
    // (it leaves the HBM copy for the later kernels): with AccountEvents this measured 70-72 us a
    // commit against 70-77 with stage_in copying the body first.
    if (src && ingest_reads_host) {
        ctx->events_host = reinterpret_cast<const tb_transfer_t*>(src);
        src = nullptr;
        bytes = 0;
        // ... and so are the batch bounds, when the call's scalar words are already clear (the
        // last call's end cleared them): no stage_in launch at all.
        if (!reset_scalars || ctx->scalars_clean) {
            ctx->batches_host = true;
            return 0;
        }
    }
    if (!src && bytes)
        HIP_TRY(ctx, hipMemcpyAsync(ctx->body_dst, events, bytes, hipMemcpyHostToDevice, ctx->stream));
    StageIn s{src, reinterpret_cast<uint4*>(ctx->body_dst), bytes / 16, ctx->dh_batch_ends,
              ctx->d_batch_ends, ctx->dh_batch_ts, ctx->d_batch_ts, nb,
              reset_scalars ? ctx->d_scalars : nullptr};
    const uint64_t per_block = uint64_t(kStageThreads) * kStageWords;
    const uint32_t grid = src ? uint32_t(std::min<uint64_t>(kStageInGridMax, std::max<uint64_t>(1, (s.words + per_block - 1) / per_block))) : 1;
    hipLaunchKernelGGL(stage_in, dim3(grid), dim3(kStageThreads), 0, ctx->stream, s);
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}


// Results (n > 0) and / or the scalars block to mapped host memory, as one kernel on the stream.
// Waits for stage_out's sequence word (every kernel before it has finished: the scalars and
// results it wrote are visible). The stream is queried now and then, so that a fault or a hang
// surfaces as the runtime reports it.
// The wait is bounded (TBG_CALL_TIMEOUT_MS, default 60 s): a kernel that hangs instead of faulting
// ends the call with TBG_EHIP and leaves the ctx failed (its tables are undefined).
int spin_wait(tbg_ctx* ctx, unsigned int seq) {
    const double deadline = now_ms() + ctx->call_timeout_ms;
    // (seq or any later number: the stream writes them in order, and a call's early signal may
    // already be overwritten by its stage_out's)
    auto reached = [&] {
        return int32_t(__atomic_load_n(ctx->h_seq, __ATOMIC_ACQUIRE) - seq) >= 0;
    };
    for (uint64_t spins = 1;; spins++) {
        if (reached()) return 0;
        if ((spins & 4095) == 0) {
            const hipError_t q = hipStreamQuery(ctx->stream);
            if (q == hipSuccess) {
                if (reached()) return 0;
                return hip_ok(ctx, hipStreamSynchronize(ctx->stream), "sync") ? 0 : TBG_EHIP;
            }
            if (q != hipErrorNotReady) return hip_ok(ctx, q, "sync") ? 0 : TBG_EHIP;
            if (now_ms() > deadline) {
                char buf[160];
                snprintf(buf, sizeof(buf), "sync: the call did not finish within %.0f ms "
                         "(a kernel hangs; the ctx is unusable)", ctx->call_timeout_ms);
                ctx->error = buf;
                ctx->failed = true;
                return TBG_EHIP;
            }
        }
        __builtin_ia32_pause();
    }
}

int stage_call_outputs(tbg_ctx* ctx, const tb_create_result_t* d_results, tb_create_result_t* dst,
                       uint32_t n, bool scalars, const AeSnapJob* snap, bool fixes,
                       unsigned int seq, uint32_t skip_epoch, bool clear) {
    StageOut s{reinterpret_cast<const uint4*>(d_results), reinterpret_cast<uint4*>(dst), n,
               scalars ? reinterpret_cast<const unsigned long long*>(ctx->d_scalars) : nullptr,
               reinterpret_cast<unsigned long long*>(ctx->dh_scalars),
               uint32_t(sizeof(DevScalars) / 8), fixes ? ctx->fix_slots : nullptr,
               ctx->T.tr.slots, ctx->d_scalars, seq ? ctx->d_stage_done : nullptr,
               seq ? ctx->dh_seq : nullptr, seq, clear && seq && scalars,
               skip_epoch ? ctx->d_stage_done + 2 : nullptr, skip_epoch, snap != nullptr, {}};
    if (snap) s.snap = *snap;
    if (!dst || !n) s.src = nullptr;
    // (with a snapshot: one 64-lane wave a workgroup, kAeAsyncMax lanes at least -- an event's
    // dependent loads spread over more CUs, as ae_snapshot's)
    const uint32_t threads = snap ? kSnapThreads : kStageThreads;
    uint32_t grid = std::max<uint32_t>(1, std::min<uint32_t>((n + threads - 1) / threads, 1024));
    // (with a snapshot, 32 workgroups copy and count and the rest only snapshot: fewer
    // system-scope releases and same-address adds before the sequence word -- SM per-commit
    // 62.3-64.1 -> 60.8-63.2 us, profiles/r05_stage_copy/)
    if (snap) s.copy_wgs = std::min<uint32_t>(grid, 32);
    if (snap) grid = std::max<uint32_t>(grid, kAeAsyncMax / kSnapThreads);
    hipLaunchKernelGGL(stage_out, dim3(grid), dim3(threads), 0, ctx->stream, s);
    HIP_TRY(ctx, hipGetLastError());
    return 0;
}

int upload_batches(tbg_ctx* ctx, uint32_t n, const uint32_t* batch_lens, const uint64_t* batch_ts,
                   uint32_t nb, const void* events, uint64_t event_bytes, bool reset_scalars,
                   bool ingest_reads_host = false) {
    if (nb == 0 || nb > ctx->opt.batch_count_max) return TBG_EINVAL;
    // (the pinned staging is free: the previous call's copies completed before it returned)
    uint64_t total = 0;
    for (uint32_t b = 0; b < nb; b++) {
        total += batch_lens[b];
        ctx->h_batch_ends[b] = uint32_t(total);
        ctx->h_batch_ts[b] = batch_ts[b];
    }
    if (total != n) return TBG_EINVAL;
    return stage_call_inputs(ctx, events, uint64_t(n) * event_bytes, nb, reset_scalars,
                             ingest_reads_host);
}

int64_t lookup_impl(tbg_ctx* ctx, const tb_uint128_t* ids, uint32_t n, void* out, bool accounts) {
    if (!ctx) return TBG_EINVAL;
    FAILED_GUARD(ctx);
    if (n == 0) return 0;
    if (n > ctx->opt.batch_events_max) return TBG_EINVAL;
    // Scratch: ids and output rows in d_events; rows in bal_items; found flags in ev_slow.
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_events, ids, size_t(n) * 16, hipMemcpyHostToDevice,
                                ctx->stream));
    const tb_uint128_t* d_ids = reinterpret_cast<const tb_uint128_t*>(ctx->d_events);
    uint64_t* d_rows = ctx->bal_items;
    if (accounts)
        hipLaunchKernelGGL(lookup_accounts_kernel, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream,
                           ctx->T, d_ids, n, d_rows, ctx->ev_slow);
    else
        hipLaunchKernelGGL(lookup_transfers_kernel, dim3(grid_for(n)), dim3(kBlock), 0,
                           ctx->stream, ctx->T, d_ids, n, d_rows, ctx->ev_slow);
    HIP_TRY(ctx, hipGetLastError());
    unsigned int* d_count = &ctx->d_scalars->slow_count;
    int rc = select_flagged(ctx, ctx->ev_slow, n, ctx->slow_list, d_count);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->h_scalars->slow_count, d_count, 4, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint32_t found = ctx->h_scalars->slow_count;
    if (found == 0) return 0;
    void* d_out = ctx->d_events + size_t(n) * 16;  // after the ids (144 B per event allocated)
    if (accounts)
        hipLaunchKernelGGL(gather_rows<tb_account_t>, dim3(grid_for(found)), dim3(kBlock), 0,
                           ctx->stream, ctx->T.acc_rows, d_rows, ctx->slow_list, found,
                           static_cast<tb_account_t*>(d_out));
    else
        hipLaunchKernelGGL(gather_rows<tb_transfer_t>, dim3(grid_for(found)), dim3(kBlock), 0,
                           ctx->stream, ctx->T.tr_rows, d_rows, ctx->slow_list, found,
                           static_cast<tb_transfer_t*>(d_out));
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemcpyAsync(out, d_out, size_t(found) * 128, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return found;
}

}  // namespace

extern "C" {

tbg_ctx* tbg_open(const tbg_options* options) {
    if (!options || options->account_capacity == 0 || options->transfer_capacity == 0 ||
        options->batch_events_max == 0 || options->batch_count_max == 0 ||
        options->pulse_batch_max == 0 || options->pulse_batch_max > kPulseRun)
        return nullptr;
    // Slots and rows are addressed with 32-bit indexes in per-event scratch.
    if (options->account_capacity >= (1ull << 31) || options->transfer_capacity >= (1ull << 31))
        return nullptr;
    tbg_ctx* ctx = new tbg_ctx();
    ctx->opt = *options;
    ctx->pulse_row_bits = options->transfer_capacity > 1
                              ? uint32_t(64 - __builtin_clzll(options->transfer_capacity - 1)) : 1u;
    bool ok = hip_ok(ctx, hipSetDevice(int(options->device)), "hipSetDevice") &&
              hip_ok(ctx, hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking),
                     "hipStreamCreate");
    const uint64_t acc_cap = options->account_capacity, tr_cap = options->transfer_capacity;
    const uint64_t ev_max = options->batch_events_max;
    // Slot tables hold at least 4 probe groups (hash_id / probe_next step 16 slots at a time).
    const uint64_t acc_slots = std::max<uint64_t>(next_pow2(acc_cap * 2), 64);
    // 4 id slots per transfer of capacity: ids claim in blocks of 16 (group-16 homes), and a
    // block whose home group is taken probes on; at group load <= 1/4 most blocks claim at home.
    const uint64_t tr_slots = std::max<uint64_t>(next_pow2(tr_cap * 4), 64);
    // 4 index entries per account (entry indexes are u32: at most 2^31 entries).
    const uint64_t acc_entries =
        std::min<uint64_t>(std::max<uint64_t>(next_pow2(acc_cap * 4), 64), 1ull << 31);
    Tables& T = ctx->T;
    ctx->idx_dirty_cap = uint32_t(std::min<uint64_t>(2 * ev_max + 4096, 1u << 30));
    ok = ok && dev_alloc(ctx, &ctx->idx_dirty, ctx->idx_dirty_cap, false) &&
         dev_alloc(ctx, &ctx->idx_counters, 2, true);
    ok = ok && dev_alloc(ctx, &T.acc_index.entries, acc_entries, true) &&
         dev_alloc(ctx, &T.acc_entry_of, acc_cap, false) &&
         hip_ok(ctx, hipMemsetAsync(T.acc_entry_of, 0xFF, acc_cap * sizeof(uint32_t), ctx->stream), "memset");
    ok = ok && dev_alloc(ctx, &T.acc.slots, acc_slots, true) &&
         dev_alloc(ctx, &T.acc_rows, acc_cap, true) && dev_alloc(ctx, &T.acc_live, acc_cap, true) &&
         dev_alloc(ctx, &T.acc_hot, acc_cap, true) &&
         dev_alloc(ctx, &T.acc_closable, acc_cap, true) &&
         dev_alloc(ctx, &T.tr.slots, tr_slots, true) && dev_alloc(ctx, &T.tr_rows, tr_cap, false) &&
         dev_alloc(ctx, &T.tr_live, tr_cap, true) && dev_alloc(ctx, &T.tr_status, tr_cap, true) &&
         dev_alloc(ctx, &T.expiry, tr_cap, false) && dev_alloc(ctx, &ctx->d_scalars, 1, true);
    const uint64_t undo_cap = 3 * std::min<uint64_t>(ev_max, 65536);
    ok = ok && dev_alloc(ctx, &T.undo, undo_cap, false);
    // (144 B per event: tbg_lookup_* place n ids and up to n 128-B rows side by side)
    ok = ok && dev_alloc(ctx, &ctx->d_events, ev_max * 144, false) &&
         dev_alloc(ctx, &ctx->d_results, ev_max, false) &&
         dev_alloc(ctx, &ctx->d_batch_ends, options->batch_count_max, false) &&
         dev_alloc(ctx, &ctx->d_batch_ts, options->batch_count_max, false) &&
         dev_alloc(ctx, &ctx->ev_slot, ev_max, false) && dev_alloc(ctx, &ctx->ev_dr, ev_max, false) &&
         dev_alloc(ctx, &ctx->ev_cr, ev_max, false) && dev_alloc(ctx, &ctx->ev_amount, ev_max, false) &&
         dev_alloc(ctx, &ctx->ev_prow, ev_max, false) &&
         dev_alloc(ctx, &ctx->ev_info, ev_max, false) && dev_alloc(ctx, &ctx->ev_slow, ev_max, false) &&
         dev_alloc(ctx, &ctx->slow_list, ev_max, false) &&
         dev_alloc(ctx, &ctx->fix_slots, ev_max, false) &&
         dev_alloc(ctx, &ctx->chain_planes, (uint64_t(ev_max) + 63) / 64 * kPlWords, false) &&
         dev_alloc(ctx, &ctx->pnt_call, ev_max, false) && dev_alloc(ctx, &ctx->pnt_fired, 4, true) &&
         dev_alloc(ctx, &ctx->pnt_tiles, (uint64_t(ev_max) + kPntTile - 1) / kPntTile + 1, false) &&
         dev_alloc(ctx, &ctx->d_stamps, ev_max + 1, false) &&
         dev_alloc(ctx, &ctx->pv_slots, next_pow2(2 * uint64_t(ev_max)), true);
    ctx->pv_mask = next_pow2(2 * uint64_t(ev_max)) - 1;
    // (2 * ev_max items, at least ev_max u64 of lookup scratch)
    ok = ok && dev_alloc(ctx, &ctx->bal_items, 2 * ev_max, false) &&
         dev_alloc(ctx, &ctx->chunk_info, (ev_max + 63) / 64 + 1, false);
    if (ev_max >= kSortThreshold) {
        ctx->bucket_slices_max = (2 * ev_max + kSliceItems - 1) / kSliceItems + kBucketsMax;
        ok = ok && dev_alloc(ctx, &ctx->bal_items_sorted, 2 * ev_max, false) &&
             dev_alloc(ctx, &ctx->bucket_words, 4 * (kBucketsMax + 1), true) &&
             dev_alloc(ctx, &ctx->bucket_partials, ctx->bucket_slices_max * kBucketKeys, false) &&
             dev_alloc(ctx, &ctx->window_partials, uint64_t(kWindowGridMax) * kWindowKeys, false) &&
             dev_alloc(ctx, &ctx->window_carry, kWindowKeys, true) &&
             dev_alloc(ctx, &ctx->window_counts, kWindowGridMax + 1, true) &&
             dev_alloc(ctx, &ctx->window_ts, 2 * kWindowGridMax, false);
    }
    ok = ok && dev_alloc(ctx, &ctx->acc_ts_index, acc_cap, false) &&
         dev_alloc(ctx, &ctx->tr_ts_index, tr_cap, false) &&
         dev_alloc(ctx, &ctx->sel_buf, std::max(acc_cap, tr_cap), false);
    if (options->account_events_capacity) {
        ctx->ae_cap = options->account_events_capacity;
        ok = ok && dev_alloc(ctx, &ctx->ae_log, ctx->ae_cap, false) &&
             dev_alloc(ctx, &ctx->ae_ref, ctx->ae_cap, false) &&
             dev_alloc(ctx, &ctx->ae_list, std::max<uint64_t>(ev_max, options->pulse_batch_max), false) &&
             dev_alloc(ctx, &ctx->ae_words, 8, true);
    }
    ok = ok && hip_ok(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->h_scalars),
                                         sizeof(DevScalars), kCoherentHost), "hipHostMalloc");
    ok = ok && hip_ok(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->h_pulse), 64, kCoherentHost), "hipHostMalloc") &&
         hip_ok(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->dh_pulse), ctx->h_pulse, 0),
                "hipHostGetDevicePointer");
    if (ok) std::memset(ctx->h_pulse, 0, 64);
    ok = ok && hip_ok(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->h_seq), 64, kCoherentHost), "hipHostMalloc") &&
         hip_ok(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->dh_seq), ctx->h_seq, 0),
                "hipHostGetDevicePointer") &&
         // stage_out's and tr_ingest's finished workgroups, the epoch of the call tr_ingest ended
         dev_alloc(ctx, &ctx->d_stage_done, 4, true);
    if (ok) *ctx->h_seq = 0;
    ctx->spin_sync = getenv("TBG_NO_SPIN_SYNC") == nullptr;
    {
        tbg_ctx::Knobs& k = ctx->knobs;
        auto on = [](const char* name) { return getenv(name) != nullptr; };
        k.no_pv_fast = on("TBG_NO_PV_FAST");
        k.no_lanes = on("TBG_NO_LANES");
        k.no_additive = on("TBG_NO_ADDITIVE");
        k.no_doom = on("TBG_NO_DOOM");
        k.no_free_owners = on("TBG_NO_FREE_OWNERS");
        k.flow_debug = on("TBG_FLOW_DEBUG");
        k.walk_seq = on("TBG_WALK_SEQ");
        k.lanes_one_lane = on("TBG_LANES_ONE_LANE");
        k.no_window = on("TBG_NO_WINDOW");
        k.no_lean_lookup = on("TBG_NO_LEAN_LOOKUP");
        k.no_ingest_finish = on("TBG_NO_INGEST_FINISH");
        // Engine shape (flow.hpp): lanes per wave x waves per workgroup x workgroups; TBG_FLOW_XCD=8
        // packs the running workgroups onto one XCD.
        auto env_u = [](const char* name, uint32_t def, uint32_t lo, uint32_t hi) {
            const char* e = getenv(name);
            const uint32_t v = e ? uint32_t(atoi(e)) : def;
            return std::max(lo, std::min(hi, v));
        };
        k.flow_lpw = env_u("TBG_FLOW_LPW", kFlowLanesPerWave, 1, 64);
        k.flow_waves = env_u("TBG_FLOW_WAVES", kFlowWaves, 1, kFlowReplayThreads / 64);
        k.flow_blocks = env_u("TBG_FLOW_BLOCKS", kFlowBlocks, 1, kFlowLanesMax / (k.flow_waves * k.flow_lpw));
        k.flow_xcd = env_u("TBG_FLOW_XCD", 1, 1, 8);
        k.flow_backoff = env_u("TBG_FLOW_BACKOFF", 1, 0, 1);
    }
    if (const char* e = getenv("TBG_CALL_TIMEOUT_MS")) ctx->call_timeout_ms = std::max(1.0, atof(e));
    ok = ok && hip_ok(ctx, hipEventCreateWithFlags(&ctx->results_ready, hipEventDisableTiming),
                      "hipEventCreate");
    ok = ok && hip_ok(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->h_batch_ends),
                                         size_t(options->batch_count_max) * 4), "hipHostMalloc") &&
         hip_ok(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->h_batch_ts),
                                   size_t(options->batch_count_max) * 8), "hipHostMalloc");
    ok = ok && hip_ok(ctx, hipHostMalloc(reinterpret_cast<void**>(&ctx->h_results),
                                         size_t(std::max<uint64_t>(ev_max, 1)) *
                                             sizeof(tb_create_result_t), kCoherentHost),
                      "hipHostMalloc");
    ok = ok && hip_ok(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->dh_scalars),
                                                   ctx->h_scalars, 0), "hipHostGetDevicePointer") &&
         hip_ok(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->dh_results),
                                             ctx->h_results, 0), "hipHostGetDevicePointer") &&
         hip_ok(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->dh_batch_ends),
                                             ctx->h_batch_ends, 0), "hipHostGetDevicePointer") &&
         hip_ok(ctx, hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->dh_batch_ts),
                                             ctx->h_batch_ts, 0), "hipHostGetDevicePointer");
    if (!ok) {
        fprintf(stderr, "tbg_open: %s\n", ctx->error.c_str());
        tbg_close(ctx);
        return nullptr;
    }
    T.acc.mask = acc_slots - 1;
    T.acc_index.mask = acc_entries - 1;
    T.tr.mask = tr_slots - 1;
    T.expiry_capacity = tr_cap;
    T.undo_capacity = undo_cap;
    T.scalars = ctx->d_scalars;
    ctx->ae_window_on = getenv("TBG_NO_AE_WINDOW") == nullptr;
    // (TBG_AE_SIDE_SNAP=1: a small call's snapshot on a stream of its own, the next call's ingest
    // waiting for it: 83-96 us a commit against 69-74 on the call's stream -- the two cross-stream
    // event waits on the critical path cost more than the 11 us snapshot they hide)
    ctx->body_dst = nullptr;
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
    // (the side stream's staging and scratch now, not in the first small call)
    if (ctx->ae_log && ctx->ae_async && ensure_ae_async(ctx) != 0) {
        fprintf(stderr, "tbg_open: %s\n", ctx->error.c_str());
        tbg_close(ctx);
        return nullptr;
    }
    // (and the pulse's scratch: a first pulse that allocates waits on every stream)
    if (ensure_pulse_scratch(ctx, 0) != 0) {
        fprintf(stderr, "tbg_open: pulse scratch\n");
        tbg_close(ctx);
        return nullptr;
    }
    return ctx;
}

void tbg_close(tbg_ctx* ctx) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return;
    if (ctx->ae_stream) (void)hipStreamSynchronize(ctx->ae_stream);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    for (int p = 0; p < 2; p++) {
        if (ctx->ae_snap_ready[p]) (void)hipEventDestroy(ctx->ae_snap_ready[p]);
        if (ctx->ae_done[p]) (void)hipEventDestroy(ctx->ae_done[p]);
        for (void* q : {(void*)ctx->ae_stage[p].rec, (void*)ctx->ae_stage[p].ref,
                        (void*)ctx->ae_stage[p].delta, (void*)ctx->ae_stage[p].created,
                        (void*)ctx->ae_stage[p].words})
            if (q) (void)hipFree(q);
    }
    if (ctx->ae_pos) (void)hipFree(ctx->ae_pos);
    if (ctx->ae_g_words) (void)hipFree(ctx->ae_g_words);
    for (void* q : {(void*)ctx->ae_small_counts, (void*)ctx->ae_small_ts, (void*)ctx->ae_dense_touch,
                    (void*)ctx->ae_dense_ev, (void*)ctx->ae_dense_partials,
                    (void*)ctx->ae_dense_counts, (void*)ctx->ae_dense_ts,
                    (void*)ctx->ae_dense_claim, (void*)ctx->ae_dense_later, (void*)ctx->ae_dense_pos, (void*)ctx->ae_wide_sums,
                    (void*)ctx->ae_wide_counts, (void*)ctx->ae_wide_ts})
        if (q) (void)hipFree(q);
    free_ae_scratch(ctx->ae_g);
    if (ctx->ae_stream) (void)hipStreamDestroy(ctx->ae_stream);
    void* ptrs[] = {ctx->idx_dirty, ctx->idx_counters, ctx->T.acc_index.entries, ctx->T.acc_entry_of, ctx->T.acc.slots, ctx->T.acc_rows, ctx->T.acc_live, ctx->T.acc_hot,
                    ctx->T.acc_closable, ctx->T.tr.slots, ctx->T.tr_rows, ctx->T.tr_live,
                    ctx->T.tr_status, ctx->T.expiry, ctx->d_scalars, ctx->T.undo, ctx->d_events,
                    ctx->d_results, ctx->d_batch_ends, ctx->d_batch_ts, ctx->ev_slot, ctx->ev_dr,
                    ctx->ev_cr, ctx->ev_amount, ctx->ev_prow, ctx->ev_info, ctx->ev_slow, ctx->slow_list,
                    ctx->fix_slots, ctx->chain_planes, ctx->d_stage_done,
                    ctx->pnt_call, ctx->pnt_fired, ctx->pnt_tiles, ctx->d_stamps, ctx->pv_slots,
                    ctx->bal_items, ctx->chunk_info, ctx->bal_items_sorted, ctx->bucket_words, ctx->bucket_partials,
                    ctx->window_partials, ctx->window_carry, ctx->window_counts, ctx->window_ts,
                    ctx->acc_ts_index, ctx->tr_ts_index, ctx->sel_buf,
                    ctx->pulse.keep, ctx->pulse.exp, ctx->pulse.ts, ctx->pulse.rows,
                    ctx->pulse.exp_b, ctx->pulse.rows_b, ctx->pulse.counters,
                    ctx->pulse.run_len, ctx->pulse.expired,
                    ctx->flow.dup_mark, ctx->flow.counts, ctx->flow.words, ctx->flow.lane_counts,
                    ctx->scan_status, ctx->scan_ticket,
                    ctx->flow.lane_undo, ctx->flow.engine, ctx->flow.acc_free,
                    ctx->flow.acc_pot, ctx->flow.doom_off,
                    ctx->ae_log, ctx->ae_ref, ctx->ae_list, ctx->ae_words};
    free_ae_scratch(ctx->ae);
    free_flow(ctx->flow);
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    for (hipEvent_t e : ctx->marks)
        if (e) (void)hipEventDestroy(e);
    if (ctx->h_scalars) (void)hipHostFree(ctx->h_scalars);
    if (ctx->h_seq) (void)hipHostFree(ctx->h_seq);
    if (ctx->h_pulse) (void)hipHostFree(ctx->h_pulse);
    if (ctx->h_results) (void)hipHostFree(ctx->h_results);
    if (ctx->h_batch_ends) (void)hipHostFree(ctx->h_batch_ends);
    if (ctx->h_batch_ts) (void)hipHostFree(ctx->h_batch_ts);
    for (const auto& r : ctx->registered) host_pin_release(reinterpret_cast<void*>(r.host));
    if (ctx->results_ready) (void)hipEventDestroy(ctx->results_ready);
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    delete ctx;
}

const char* tbg_last_error(const tbg_ctx* ctx) {
    TBG_DEVICE_SCOPE(ctx); return ctx ? ctx->error.c_str() : "null ctx"; }

}  // extern "C"

namespace {

#ifndef TBG_SMALL_INGEST_THREADS
#define TBG_SMALL_INGEST_THREADS 128
#endif
int create_transfers_impl(tbg_ctx* ctx, const tb_transfer_t* d_events, uint32_t n,
                          const uint32_t* d_batch_ends, const uint64_t* d_batch_ts,
                          uint32_t n_batches, tb_create_result_t* d_results, void* stream,
                          const uint64_t* d_event_ts) {
    if (!ctx || n > ctx->opt.batch_events_max || n_batches > ctx->opt.batch_count_max)
        return TBG_EINVAL;
    FAILED_GUARD(ctx);
    if (ctx->T.tr_rows_used + n > ctx->opt.transfer_capacity) {
        ctx->error = "transfer capacity exceeded";
        return TBG_ENOSPC;
    }
    if (n == 0) return 0;
    hipStream_t saved = ctx->stream;
    if (stream) ctx->stream = static_cast<hipStream_t>(stream);
    ctx->expiry_known = false;  // (end_call learns it again)
    int rc = begin_call(ctx, false);
    Call<tb_transfer_t> c = make_call(ctx, d_events, n, d_batch_ends, d_batch_ts, n_batches,
                                      d_results, ctx->T.tr_rows_used);
    c.event_ts = d_event_ts;
    const dim3 grid(std::min(grid_for(n), kMaxGrid)), block(kBlock);  // grid-stride kernels
    // tr_ingest: 12,288 workgroups (48 per CU) beat the grid-stride default of 4,096 by 3 % on
    // config 2 (0.707 vs 0.728 ms per 10M events); 32,768 and more lose 40 %.
    uint32_t ig = std::min(grid_for(n), kIngestGrid);
    const bool use_sort = n >= kSortThreshold && ctx->bal_items_sorted;
    // Balance items pack (amount << key_bits) | field key into a u64; the all-ones key is the
    // "no item" sentinel, so key_bits covers 4 * accounts + 1 values.
    const uint32_t key_end = uint32_t(4 * ctx->T.acc_rows_used);
    uint32_t key_bits = 1;
    while ((1ull << key_bits) <= key_end) key_bits++;
    // Key spaces of <= 2^14 accounts take the balance window (pair items, LDS counters; config
    // 2); up to 262,144 accounts the bucketed path, whose LDS sums need amounts < 2^48 (key_bits
    // >= 16); larger ones per-workgroup LDS hash tables (bal_hash_apply), or u128 atomics when
    // the key space is sparse.
    uint32_t pair_shift = 1;
    while ((1ull << pair_shift) < ctx->T.acc_rows_used) pair_shift++;
    const bool use_window = use_sort && ctx->window_partials && pair_shift <= kWindowShiftMax &&
                            !ctx->knobs.no_window;
    const bool use_buckets = use_sort && !use_window && key_end <= kBucketsMax * kBucketKeys;
    // Sparse key spaces (many more account fields than balance items, e.g. 125M accounts under
    // 1M-event calls): u128 atomics per item instead of the sort; collisions are rare.
    const bool use_atomic = use_sort && !use_window && !use_buckets &&
                            uint64_t(key_end) > kAtomicKeysPerItem * 2 * uint64_t(n);
    // Sparse key spaces: tr_ingest applies each FAST event's deltas with u128 atomics itself (as
    // in small calls; a demotion subtracts them) -- no items written, read back and applied by a
    // second kernel.
    const bool ingest_atomics = use_atomic;
    if (use_buckets && key_bits < 16) key_bits = 16;
    BucketPlan plan{};
    c.lean_lookup = ingest_atomics && !ctx->knobs.no_lean_lookup;
    if (use_sort && !ingest_atomics) {
        c.bal_items = ctx->bal_items;
        c.key_bits = key_bits;
        if (use_window) c.pair_shift = pair_shift;
    }
    if (use_buckets && !rc) {
        plan.counts = ctx->bucket_words;
        plan.cursor = plan.counts + kBucketsMax;
        plan.offset = plan.cursor + kBucketsMax;
        plan.slice_base = plan.offset + kBucketsMax + 1;
        plan.n_buckets = std::max<uint32_t>(1, (key_end + kBucketKeys - 1) / kBucketKeys);
        c.bucket_counts = plan.counts;
        c.n_buckets = plan.n_buckets;
        rc = hip_ok(ctx, hipMemsetAsync(plan.counts, 0, kBucketsMax * sizeof(unsigned int),
                                        ctx->stream), "memset") ? 0 : TBG_EHIP;
    }
    if (!rc && n_batches > kChunkBatchMask) rc = TBG_EINVAL;
    // Small calls whose scalar words the host-buffer staging already reset: each ingest wave
    // finds its chunk's batch bounds itself (no tr_chunk_info launch).
    const bool inline_chunks = (ctx->scalars_reset || ctx->scalars_clean) && n <= kInlineChunkMax;
    ctx->scalars_reset = false;
    ctx->scalars_clean = false;
    // The call's outputs for the host: a host-buffer call's results go to mapped host memory (the
    // registered destination, or the pinned staging); a spinning host waits for a sequence word.
    tb_create_result_t* dst = nullptr;
    if (ctx->early_dst) {
        dst = mapped(ctx, ctx->early_dst, uint64_t(n) * 16);
        if (!dst) dst = ctx->dh_results;
    }
    // (timed calls wait as untimed ones do: a stream synchronisation's slower wake-up, ~70 us, was
    // counted into the next mark's span -- the flow plan's -- with the GPU idle; end_call still
    // synchronises the stream before the marks are read)
    const bool spin = ctx->spin_sync;
    // A large call after a replayed one is expected to replay too: tr_commit's last workgroup
    // publishes the scalars block (the replay count is final there) under a sequence word of its
    // own, and the host launches the plan while the balance kernels and stage_out run -- the
    // launch latency that idled the GPU before the plan's first kernel. (The earlier number: the
    // host's wait accepts any later one.)
    const unsigned int early_seq =
        spin && !inline_chunks && n > kInlineChunkMax && ctx->replay_hint && !ae_async_ok(ctx, n)
            ? (++ctx->seq ? ctx->seq : ++ctx->seq) : 0u;
    const unsigned int seq = spin ? (++ctx->seq ? ctx->seq : ++ctx->seq) : 0u;
    if (early_seq) {
        c.commit_done = ctx->d_stage_done + 3;
        c.commit_scalars = reinterpret_cast<unsigned long long*>(ctx->dh_scalars);
        c.commit_seq = ctx->dh_seq;
        c.commit_seq_val = early_seq;
    }
    // A small device-buffer call without balance items may end in its last tr_ingest workgroup
    // (Call::finish_done); tr_commit and stage_out are queued all the same and return at once then
    // (device per-commit 27.7 -> 24.5 us, r05_g / r05_i). Host-buffer calls keep stage_out: with
    // the results' PCIe writes in tr_ingest's workgroups a commit took 71-77 us against 64-68
    // (r05_i A/B).
    const bool finish = inline_chunks && !use_sort && !dst && !ctx->knobs.no_ingest_finish;
    // A spinning host launches tr_commit and stage_out only when the ingest did not end the call:
    // queued behind it and returning at once, the two launches were ~9.5 of the ~25 us a small
    // device call took on the GPU (profiles/r06_pc/). (A call whose stage_out carries an
    // AccountEvents snapshot keeps them queued.)
    const bool finish_first = finish && spin && !ae_async_ok(ctx, n);
    if (!rc && inline_chunks) {
        c.chunk_info = nullptr;
        if (finish) {
            c.finish_done = ctx->d_stage_done + 1;
            c.finish_scalars = reinterpret_cast<unsigned long long*>(ctx->dh_scalars);
            c.finish_seq = seq ? ctx->dh_seq : nullptr;
            c.seq = seq;
            c.finish_always = finish_first ? 1u : 0u;
        }
        Call<tb_transfer_t> ci = c;
        if (ctx->events_host) {
            ci.events = ctx->events_host;
            ci.events_out = const_cast<tb_transfer_t*>(c.events);
        }
        if (ctx->batches_host) {
            ci.batch_ends = ctx->dh_batch_ends;
            ci.batch_ts = ctx->dh_batch_ts;
            ci.ends_out = const_cast<uint32_t*>(c.batch_ends);
            ci.ts_out = const_cast<uint64_t*>(c.batch_ts);
        }
        // (small calls: one 64-event chunk a wave, two waves a workgroup -- the chunks' dependent
        // round trips on twice as many CUs: per-commit p50 24.6-26.0 -> 23.3-25.1 us with 128 lanes,
        // 23.6-24.7 with 64, profiles/r06_si/)
        const uint32_t sthreads = TBG_SMALL_INGEST_THREADS;
        hipLaunchKernelGGL(tr_ingest, dim3((n + sthreads - 1) / sthreads), dim3(sthreads), 0,
                           ctx->stream, ctx->T, ci);
        tmark(ctx, "tr_ingest");
        if (!finish_first) {
            hipLaunchKernelGGL(tr_commit, grid, block, 0, ctx->stream, ctx->T, c);
            tmark(ctx, "tr_commit");
        }
        rc = hip_ok(ctx, hipGetLastError(), "launch") ? 0 : TBG_EHIP;
        if (!rc) rc = ae_flush_all(ctx);  // (deferred appends, while this call runs)
    } else if (!rc) {
        c.chunk_info = ctx->chunk_info;
        hipLaunchKernelGGL(tr_chunk_info, dim3(grid_for((n + 63) / 64)), block, 0, ctx->stream, c,
                           ctx->chunk_info, ctx->d_scalars);
        hipLaunchKernelGGL(tr_ingest, dim3(ig), block, 0, ctx->stream, ctx->T, c);
        tmark(ctx, "tr_ingest");
        // (large calls: chains resolved from bit planes -- a launch that returns at once when the
        // call has no chain to confirm -- only while the calls have chains: the planes' launch
        // alone costs ~5 us a call, and tr_commit is exact either way: without planes it walks
        // the chains)
        if (ctx->chain_hint) {
            c.chain_planes = ctx->chain_planes;
            hipLaunchKernelGGL(tr_chain_planes, grid, block, 0, ctx->stream, ctx->T, c);
        }
        hipLaunchKernelGGL(tr_commit, grid, block, 0, ctx->stream, ctx->T, c);
        tmark(ctx, "tr_commit");
        rc = hip_ok(ctx, hipGetLastError(), "launch") ? 0 : TBG_EHIP;
        if (!rc) rc = ae_flush_all(ctx);
    }
    const int items = int(2 * uint64_t(n));
    const BalTarget target{ctx->T.acc_rows, ctx->T.acc_index, ctx->T.acc_entry_of};
    if (!rc && use_window) {
        // Balance deltas: pair items summed per workgroup in LDS counters, partials applied.
        // (even: a call with wide items pairs the workgroups, one per posted field and slice)
        const uint32_t nwg =
            std::max<uint32_t>(2, std::min<uint32_t>(kWindowGridMax, n / 8192)) & ~1u;
        const uint32_t wkeys = std::min<uint32_t>(kWindowKeys, 4u << pair_shift);
        hipLaunchKernelGGL(bal_window_accumulate, dim3(nwg), dim3(kWindowThreads), 0, ctx->stream,
                           target, ctx->bal_items, c.ev_amount, n, pair_shift, wkeys,
                           ctx->window_partials,
                           ctx->window_carry, ctx->window_counts, &ctx->d_scalars->flags);
        tmark(ctx, "bal_window");
        hipLaunchKernelGGL(bal_window_apply, dim3((wkeys + 63) / 64), dim3(kApplyThreads), 0,
                           ctx->stream, target,
                           ctx->window_partials, nwg, pair_shift, wkeys, ctx->T.acc_rows_used,
                           ctx->window_carry, &ctx->d_scalars->flags);
        ctx->win.epoch = c.epoch;
        ctx->win.nwg = nwg;
        ctx->win.ps = pair_shift;
        ctx->win.wkeys = wkeys;
        tmark(ctx, "bal_apply");
        rc = hip_ok(ctx, hipGetLastError(), "launch") ? 0 : TBG_EHIP;
    } else if (!rc && use_buckets) {
        // Balance deltas: bucket the packed items by key range, sum each slice in LDS, apply.
        hipLaunchKernelGGL(bal_bucket_plan, dim3(1), dim3(64), 0, ctx->stream, plan);
        hipLaunchKernelGGL(bal_bucket_scatter, dim3(uint32_t((items + kScatterTile - 1) / kScatterTile)),
                           block, 0, ctx->stream, plan, ctx->bal_items, uint64_t(items), key_bits,
                           key_end, ctx->bal_items_sorted);
        tmark(ctx, "bal_scatter");
        const uint32_t slices = uint32_t((uint64_t(items) + kSliceItems - 1) / kSliceItems) +
                                plan.n_buckets;
        hipLaunchKernelGGL(bal_bucket_accumulate, dim3(slices), block, 0, ctx->stream, plan,
                           ctx->bal_items_sorted, key_bits, ctx->bucket_partials);
        tmark(ctx, "bal_accumulate");
        hipLaunchKernelGGL(bal_bucket_apply, dim3(grid_for(key_end)), block, 0, ctx->stream,
                           target, plan, ctx->bucket_partials, key_end);
        tmark(ctx, "bal_apply");
        rc = hip_ok(ctx, hipGetLastError(), "launch") ? 0 : TBG_EHIP;
    } else if (!rc && use_sort && !ingest_atomics) {
        // Balance deltas: items summed per account field in per-workgroup LDS hash tables.
        const uint64_t blocks = (uint64_t(items) + kHashSliceItems - 1) / kHashSliceItems;
        hipLaunchKernelGGL(bal_hash_apply, dim3(uint32_t(blocks)), dim3(kHashThreads), 0,
                           ctx->stream, target, ctx->bal_items, uint64_t(items), key_bits, key_end);
        tmark(ctx, "bal_hash");
        rc = hip_ok(ctx, hipGetLastError(), "launch") ? 0 : TBG_EHIP;
    }
    // A large call that follows a replayed one selects its replay list before the host's
    // synchronisation (a call without replayed events ignores the list): after it the host goes
    // straight to the plan.
    const bool pre_selected = !rc && n > kInlineChunkMax && ctx->replay_hint;
    if (pre_selected)
        rc = select_flagged(ctx, ctx->ev_slow, c.n, ctx->slow_list, &ctx->d_scalars->slow_count);
    // A host-buffer call's results are queued for download here, so that one host
    // synchronisation covers them when the call needs no replay (else they are downloaded again).
    // One host synchronisation: does the call need the ordered replay (and, with imported events,
    // the accounts' timestamp index)? One kernel writes the scalars and, for a host-buffer call,
    // its results to mapped host memory (the registered destination, or the pinned staging).
    if (!rc && finish_first) {
        ctx->ae_snap_early = false;
        tmark(ctx, "host_sync");
        rc = spin_wait(ctx, seq);
        if (!rc && !(ctx->h_scalars->flags & kFlagFinished)) {
            // (the ingest raised a commit flag: the call's tr_commit and stage_out, now)
            const unsigned int seq2 = ++ctx->seq ? ctx->seq : ++ctx->seq;
            hipLaunchKernelGGL(tr_commit, grid, block, 0, ctx->stream, ctx->T, c);
            tmark(ctx, "tr_commit");
            rc = hip_ok(ctx, hipGetLastError(), "launch") ? 0 : TBG_EHIP;
            if (!rc) rc = stage_call_outputs(ctx, d_results, nullptr, 0, true, nullptr, true, seq2,
                                             0u, !c.pnt_force);
            tmark(ctx, "host_sync");
            if (!rc) rc = spin_wait(ctx, seq2);
        }
    } else if (!rc) {
        const bool snap = ae_async_ok(ctx, n);
        // A small call's AccountEvents snapshot is taken by stage_out's workgroups once they are
        // counted (the host's wait ends at the sequence word): final unless a replay follows, then
        // it stages nothing. Its appends are queued on the side stream now, so that the host's
        // launch calls overlap the call's kernels.
        // (the appends themselves are queued at the next call's start, ae_flush_all, when the
        // snapshot has told the host which of them the staging needs: one launch instead of the
        // general path's seven that skip)
        AeSnapJob J;
        if (snap) {
            rc = ae_snap_job(ctx, c, &J);
            J.speculative = true;
            ctx->h_pulse[4] = 0;
            J.host_general = ctx->dh_pulse + 4;
        }
        if (!rc)
            rc = stage_call_outputs(ctx, d_results, dst, dst ? n : 0, true, snap ? &J : nullptr,
                                    true, seq, finish ? c.epoch : 0u, !c.pnt_force);
        if (!rc && snap) {
            rc = ae_defer_graph(ctx, n, c.epoch, false);
            ctx->ae_def_call = true;
        }
        ctx->ae_snap_early = snap && !rc;
        // (the mark before the wait: recorded after it, on an idle GPU, its host cost delayed the
        // replay's first launch and was counted into the flow plan's span)
        tmark(ctx, "host_sync");
        if (!rc) rc = spin ? spin_wait(ctx, early_seq ? early_seq : seq)
                           : (hip_ok(ctx, hipStreamSynchronize(ctx->stream), "sync") ? 0 : TBG_EHIP);
        // (no replay after all: the call's end is stage_out's sequence word)
        if (!rc && early_seq && ctx->h_scalars->stats[0] == 0) rc = spin_wait(ctx, seq);
    }
    const bool replay = !rc && ctx->h_scalars->stats[0] > 0;
    if (!rc && n > kInlineChunkMax) {
        ctx->chain_hint = (ctx->h_scalars->flags & kFlagChain) != 0;
        ctx->replay_hint = replay;
    }
    if (replay) ctx->ae_snap_early = false;
    ctx->early_done = !rc && ctx->early_dst && !replay;  // (only the replay rewrites results)
    if (replay && (ctx->h_scalars->flags & kFlagImported)) rc = check_imported_indexes(ctx, true);
    if (replay && !rc) rc = run_replay(ctx, c, true, false, pre_selected);
    const bool pnt = !rc && ((ctx->h_scalars->flags & kFlagPostVoid) || c.pnt_force);
    if (pnt) rc = pnt_resolve(ctx, c);
    // (lean marks: the end of the work queued after the host's wait)
    if (!rc && ctx->timing_lean && (replay || pnt)) tmark(ctx, "call");
    if (!rc) {
        ctx->pnt_last = c;
        ctx->pnt_last_valid = c.pnt_force != 0;
    }
    // (a replayed call's one-pass AccountEvents start now: end_call's synchronisation then covers
    // their refusal word)
    if (!rc && replay && ctx->ae_log && !ae_async_ok(ctx, n)) {
        const int prc = ae_dense_prefix(ctx, c);
        if (prc < 0) rc = prc;
    }
    if (!rc) rc = end_call(ctx, n, !replay);
    if (!rc && ctx->ae_log && ctx->ae_defer) {
        ctx->ae_call = c;  // launched by tbg_create_transfers once the results' copy is queued
        ctx->ae_deferred = true;
    } else if (!rc && ctx->ae_log) {
        const double ta = ctx->timing_host ? now_ms() : 0;
        rc = ae_transfers(ctx, c);
        hprof(ctx, "host:account_events", now_ms() - ta);
    }
    if (!rc && (ctx->h_scalars->flags & (kFlagFinished | kFlagStageCleared))) {
        ctx->scalars_clean = true;  // (tr_ingest's or stage_out's last workgroup cleared them)
    } else if (!rc) {
        hipLaunchKernelGGL(tr_reset_scalars, dim3(1), dim3(64), 0, ctx->stream, ctx->d_scalars);
        ctx->scalars_clean = hip_ok(ctx, hipGetLastError(), "reset");
    }
    ctx->stream = saved;
    ctx->T.tr_rows_used += n;  // rows are consumed whether or not the events created objects
    ctx->tr_ts_stale = true;
    return rc;
}

// Results of a host-buffer call: DMA straight into a registered destination, else into the
// pinned staging rows and one host copy (a pageable destination would take the driver's slower
// staged path). A create_transfers call's deferred AccountEvents are launched behind the copy:
// the host waits for the results only, and the next call's work queues behind the appends on the
// same stream. `early`: the results were already downloaded before the call's synchronisation.
int download_results(tbg_ctx* ctx, tb_create_result_t* results, uint32_t n, bool early = false) {
    tb_create_result_t* dst = mapped(ctx, results, uint64_t(n) * 16);
    const bool direct = dst != nullptr;
    if (!early) {
        int rc = stage_call_outputs(ctx, ctx->d_results, direct ? dst : ctx->dh_results, n, false);
        if (rc) return rc;
        HIP_TRY(ctx, hipEventRecord(ctx->results_ready, ctx->stream));
    }
    int rc = 0;
    if (ctx->ae_deferred) {
        ctx->ae_deferred = false;
        const double ta = ctx->timing_host ? now_ms() : 0;
        rc = ae_transfers(ctx, ctx->ae_call);
        hprof(ctx, "host:account_events", now_ms() - ta);
    }
    if (!early) HIP_TRY(ctx, hipEventSynchronize(ctx->results_ready));
    if (!direct) std::memcpy(results, ctx->h_results, size_t(n) * 16);
    return rc;
}

}  // namespace

extern "C" {

int tbg_create_transfers_device(tbg_ctx* ctx, const tb_transfer_t* d_events, uint32_t n,
                                const uint32_t* d_batch_ends, const uint64_t* d_batch_ts,
                                uint32_t n_batches, tb_create_result_t* d_results, void* stream) {
    TBG_DEVICE_SCOPE(ctx);
    return create_transfers_impl(ctx, d_events, n, d_batch_ends, d_batch_ts, n_batches, d_results,
                                 stream, nullptr);
}

int tbg_create_transfers_stamped_device(tbg_ctx* ctx, const tb_transfer_t* d_events, uint32_t n,
                                        const uint64_t* d_event_timestamps,
                                        tb_create_result_t* d_results, void* stream) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || n > ctx->opt.batch_events_max || !d_event_timestamps) return TBG_EINVAL;
    if (n == 0) return 0;
    // One batch: its end, and its timestamp = the last event's (imported events' must_not_advance
    // bound; the router sends no imported event on this path).
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : ctx->stream;
    const uint32_t end = n;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_batch_ends, &end, 4, hipMemcpyHostToDevice, st));
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_batch_ts, d_event_timestamps + (n - 1), 8,
                                hipMemcpyDeviceToDevice, st));
    HIP_TRY(ctx, hipStreamSynchronize(st));  // (`end` is a stack value)
    return create_transfers_impl(ctx, d_events, n, ctx->d_batch_ends, ctx->d_batch_ts, 1,
                                 d_results, stream, d_event_timestamps);
}

}  // extern "C"

namespace {

int create_accounts_impl(tbg_ctx* ctx, const tb_account_t* d_events, uint32_t n,
                         const uint32_t* d_batch_ends, const uint64_t* d_batch_ts,
                         uint32_t n_batches, tb_create_result_t* d_results, void* stream,
                         const uint64_t* d_event_ts) {
    if (!ctx || n > ctx->opt.batch_events_max || n_batches > ctx->opt.batch_count_max)
        return TBG_EINVAL;
    FAILED_GUARD(ctx);
    if (ctx->T.acc_rows_used + n > ctx->opt.account_capacity) {
        ctx->error = "account capacity exceeded";
        return TBG_ENOSPC;
    }
    if (n == 0) return 0;
    hipStream_t saved = ctx->stream;
    if (stream) ctx->stream = static_cast<hipStream_t>(stream);
    int rc = begin_call(ctx);
    Call<tb_account_t> c = make_call(ctx, d_events, n, d_batch_ends, d_batch_ts, n_batches,
                                     d_results, ctx->T.acc_rows_used);
    c.event_ts = d_event_ts;
    const dim3 grid(grid_for(n)), block(kBlock);
    if (!rc) {
        hipLaunchKernelGGL(acc_prepare, grid, block, 0, ctx->stream, ctx->T, c);
        tmark(ctx, "acc_prepare");
        rc = sync_scalars(ctx);
    }
    if (!rc && (ctx->h_scalars->flags & kFlagImported)) rc = check_imported_indexes(ctx, false);
    if (!rc) {
        hipLaunchKernelGGL(acc_classify, grid, block, 0, ctx->stream, ctx->T, c);
        tmark(ctx, "acc_classify");
        rc = hip_ok(ctx, hipGetLastError(), "launch") ? 0 : TBG_EHIP;
    }
    if (!rc) rc = run_replay(ctx, c, false, true);
    if (!rc) {
        const IndexBuild ib{ctx->idx_dirty, ctx->idx_counters, ctx->idx_dirty_cap};
        rc = hip_ok(ctx, hipMemsetAsync(ctx->idx_counters, 0, 2 * sizeof(unsigned int),
                                        ctx->stream), "memset") ? 0 : TBG_EHIP;
        if (!rc) {
            hipLaunchKernelGGL(acc_index_insert_rows, grid, block, 0, ctx->stream, ctx->T,
                               ctx->T.acc_rows_used, n, ib);
            hipLaunchKernelGGL(acc_index_repair, dim3(1024), block, 0, ctx->stream, ctx->T, ib);
            tmark(ctx, "acc_index_build");
            rc = hip_ok(ctx, hipGetLastError(), "launch") ? 0 : TBG_EHIP;
        }
    }
    if (!rc) rc = end_call(ctx, n);
    ctx->stream = saved;
    ctx->T.acc_rows_used += n;
    ctx->acc_ts_stale = true;
    return rc;
}

// Validates a stamped call's per-event timestamps (nonzero, increasing); its batch timestamp
// (0: the last event's) in *bts.
int stamps_ok(const uint64_t* ts, uint32_t n, uint64_t batch_timestamp, uint64_t* bts) {
    if (!ts) return TBG_EINVAL;
    for (uint32_t i = 0; i < n; i++)
        if (ts[i] == 0 || (i && ts[i] <= ts[i - 1])) return TBG_EINVAL;
    *bts = batch_timestamp ? batch_timestamp : ts[n - 1];
    return 0;
}

// A host stamped call's inputs: the body and one batch (its end, its timestamp) through the
// host-buffer staging, the per-event timestamps to d_stamps.
int upload_stamped(tbg_ctx* ctx, const void* events, uint32_t n, const uint64_t* ts, uint64_t bts) {
    int rc = body_buffer(ctx);
    if (rc) return rc;
    const uint32_t len = n;
    rc = upload_batches(ctx, n, &len, &bts, 1, events, 128, false);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_stamps, ts, size_t(n) * 8, hipMemcpyHostToDevice,
                                ctx->stream));
    return 0;
}

}  // namespace

extern "C" {

int tbg_create_accounts_device(tbg_ctx* ctx, const tb_account_t* d_events, uint32_t n,
                               const uint32_t* d_batch_ends, const uint64_t* d_batch_ts,
                               uint32_t n_batches, tb_create_result_t* d_results, void* stream) {
    TBG_DEVICE_SCOPE(ctx);
    return create_accounts_impl(ctx, d_events, n, d_batch_ends, d_batch_ts, n_batches, d_results,
                                stream, nullptr);
}

int tbg_create_transfers_stamped(tbg_ctx* ctx, const tb_transfer_t* events, uint32_t n,
                                 const uint64_t* event_timestamps, uint64_t batch_timestamp,
                                 uint32_t options, tb_create_result_t* results) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || n > ctx->opt.batch_events_max || (options & ~TBG_ONE_CHAIN)) return TBG_EINVAL;
    if (n == 0) return 0;
    FAILED_GUARD(ctx);
    uint64_t bts = 0;
    int rc = stamps_ok(event_timestamps, n, batch_timestamp, &bts);
    if (!rc) rc = upload_stamped(ctx, events, n, event_timestamps, bts);
    ctx->call_one_chain = (options & TBG_ONE_CHAIN) != 0;
    if (!rc)
        rc = create_transfers_impl(ctx, reinterpret_cast<const tb_transfer_t*>(ctx->body_dst), n,
                                   ctx->d_batch_ends, ctx->d_batch_ts, 1, ctx->d_results, nullptr,
                                   ctx->d_stamps);
    ctx->call_one_chain = false;
    if (!rc) rc = download_results(ctx, results, n);
    return rc;
}

int tbg_create_accounts_stamped(tbg_ctx* ctx, const tb_account_t* events, uint32_t n,
                                const uint64_t* event_timestamps, uint64_t batch_timestamp,
                                uint32_t options, tb_create_result_t* results) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || n > ctx->opt.batch_events_max || (options & ~TBG_ONE_CHAIN)) return TBG_EINVAL;
    if (n == 0) return 0;
    FAILED_GUARD(ctx);
    uint64_t bts = 0;
    int rc = stamps_ok(event_timestamps, n, batch_timestamp, &bts);
    if (!rc) rc = upload_stamped(ctx, events, n, event_timestamps, bts);
    ctx->call_one_chain = (options & TBG_ONE_CHAIN) != 0;
    if (!rc)
        rc = create_accounts_impl(ctx, reinterpret_cast<const tb_account_t*>(ctx->body_dst), n,
                                  ctx->d_batch_ends, ctx->d_batch_ts, 1, ctx->d_results, nullptr,
                                  ctx->d_stamps);
    ctx->call_one_chain = false;
    if (!rc) rc = download_results(ctx, results, n);
    return rc;
}

int tbg_create_transfers(tbg_ctx* ctx, const tb_transfer_t* events, uint32_t n,
                         const uint32_t* batch_lens, const uint64_t* batch_ts, uint32_t nb,
                         tb_create_result_t* results) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || n > ctx->opt.batch_events_max) return TBG_EINVAL;
    if (n == 0) return 0;
    const double t0 = ctx->timing_host ? now_ms() : 0;
    // The body's buffer: d_events, unless a deferred snapshot still reads it (then a small call
    // takes the second buffer, a larger one queues that snapshot first).
    int rc = body_buffer(ctx);
    if (rc) return rc;
    // (stage_in resets the call's scalar words: no tr_chunk_info launch for a small call)
    rc = upload_batches(ctx, n, batch_lens, batch_ts, nb, events, 128, n <= kInlineChunkMax,
                        n <= kInlineChunkMax);
    if (rc) return rc;
    ctx->scalars_reset = n <= kInlineChunkMax;
    const double t1 = ctx->timing_host ? now_ms() : 0;
    ctx->ae_defer = true;
    // (the results go to the host with the call's end unless the last large call replayed: a
    // replay rewrites them, and the early copy -- ~70 us of PCIe writes for 131k results -- is then
    // made for nothing; they are downloaded after the call instead)
    ctx->early_dst = n > kInlineChunkMax && ctx->replay_hint ? nullptr : results;
    rc = tbg_create_transfers_device(ctx, reinterpret_cast<const tb_transfer_t*>(ctx->body_dst), n,
                                     ctx->d_batch_ends, ctx->d_batch_ts, nb, ctx->d_results,
                                     nullptr);
    ctx->ae_defer = false;
    ctx->early_dst = nullptr;
    ctx->scalars_reset = false;
    ctx->events_host = nullptr;
    ctx->batches_host = false;
    if (rc) {
        ctx->ae_deferred = false;
        return rc;
    }
    const double t2 = ctx->timing_host ? now_ms() : 0;
    rc = download_results(ctx, results, n, ctx->early_done);
    if (rc) return rc;
    if (ctx->timing_host) {
        hprof(ctx, "host:upload", t1 - t0);
        hprof(ctx, "host:call", t2 - t1);
        hprof(ctx, "host:download", now_ms() - t2);
    }
    return 0;
}

int tbg_create_accounts(tbg_ctx* ctx, const tb_account_t* events, uint32_t n,
                        const uint32_t* batch_lens, const uint64_t* batch_ts, uint32_t nb,
                        tb_create_result_t* results) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || n > ctx->opt.batch_events_max) return TBG_EINVAL;
    if (n == 0) return 0;
    int rc = body_buffer(ctx);
    if (rc) return rc;
    rc = upload_batches(ctx, n, batch_lens, batch_ts, nb, events, 128, false);
    if (rc) return rc;
    rc = tbg_create_accounts_device(ctx, reinterpret_cast<const tb_account_t*>(ctx->body_dst), n,
                                    ctx->d_batch_ends, ctx->d_batch_ts, nb, ctx->d_results, nullptr);
    if (rc) return rc;
    rc = download_results(ctx, results, n);
    if (rc) return rc;
    return 0;
}

}  // extern "C"

namespace {

// The expired-eligible entries of the expires_at index: candidates (rows, expires_at) at
// S.rows / S.exp, sorted into (expires_at, timestamp) order when `sort`; the entries still pending
// at S.keep. Row order is timestamp order, so a stable sort by row followed by a stable sort by
// expires_at yields the index order (scan_lookup.zig:150-175).
struct PulseGather {
    uint64_t cands = 0, kept = 0, next_unexpired = ~0ull;
};
// The expired candidates, their first min(candidates, k) in (expires_at, timestamp) order at
// S.exp / S.rows (pulse.hpp: LDS-sorted runs, pairwise merges keeping the first k); the entries still
// pending at S.keep; the counters on device. `out`: the counters on the host too (one sync).
int pulse_select(tbg_ctx* ctx, uint64_t timestamp, uint32_t k, PulseGather* out,
                 bool settle = false, unsigned long long* report = nullptr, bool fused = false) {
    int rc = 0;
    // The index length: known on the host since the last call or pulse (else one synchronisation).
    if (!ctx->expiry_known) {
        rc = sync_scalars(ctx);
        if (rc) return rc;
        ctx->expiry_host = ctx->h_scalars->expiry_count;
        ctx->expiry_known = true;
    }
    const uint64_t count = std::min<uint64_t>(ctx->expiry_host, ctx->T.expiry_capacity);
    rc = ensure_pulse_scratch(ctx, count);
    if (rc) return rc;
    PulseScratch& S = ctx->pulse;
    if (!S.counters_clean)
        hipLaunchKernelGGL(pulse_reset_counters, dim3(1), dim3(64), 0, ctx->stream, S.counters);
    S.counters_clean = false;
    if (count) {
        hipLaunchKernelGGL(pulse_collect, dim3(uint32_t((count + kPulseCollectTile - 1) / kPulseCollectTile)),
                           dim3(kPulseCollectThreads), 0, ctx->stream,
                           ctx->T, timestamp, count, S.keep, &S.counters[0], S.exp, S.ts, S.rows,
                           &S.counters[1], &S.counters[2], &S.counters[4]);
        // Sorted runs of kPulseSortRun, then pairwise merges (each keeping the first k): run r of
        // a level at r * stride, the stride doubling up to kPulseRun.
        const uint32_t runs = uint32_t((count + kPulseSortRun - 1) / kPulseSortRun);
        const uint64_t lens = S.capacity / kPulseSortRun + 1;
        const uint32_t row_bits = ctx->pulse_row_bits;
        PulseRuns A{S.exp, S.rows, S.run_len, kPulseSortRun};
        PulseRuns B{S.exp_b, S.rows_b, S.run_len + lens, kPulseSortRun};
        hipLaunchKernelGGL(pulse_sort_chunks, dim3(runs), dim3(kPulseSortThreads), 0, ctx->stream, A,
                           S.counters, k, timestamp, row_bits);
        const PulseRuns first = A, second = B;
        uint32_t live = runs, levels = 0;
        bool swapped = false;
        while (live > 1) {
            const uint32_t next = (live + 1) / 2;
            B.stride = std::min<uint32_t>(2 * A.stride, kPulseRun);
            hipLaunchKernelGGL(pulse_merge, dim3(next * kPulseSegs), dim3(kPulseSegThreads), 0, ctx->stream, A,
                               live, k, B, S.counters, timestamp, row_bits, levels);
            std::swap(A, B);
            swapped = !swapped;
            live = next;
            levels++;
        }
        S.first = first;
        S.second = second;
        if (fused) {
            // (pulse_apply_root reads the result where the levels that ran left it)
        } else if (levels)  // (moves the result where the host reads it; settles a pulse)
            hipLaunchKernelGGL(pulse_final_copy, dim3(1), dim3(kPulseThreads), 0, ctx->stream, first,
                               second, S.counters, levels, ctx->T, S.expired, k, uint32_t(settle),
                               report);
        else if (settle)
            hipLaunchKernelGGL(pulse_settle, dim3(1), dim3(64), 0, ctx->stream, ctx->T, S.exp,
                               S.counters, S.expired, k, report);
        if (swapped && !fused) {  // (the result is in the second buffers: they become the first)
            std::swap(S.exp, S.exp_b);
            std::swap(S.rows, S.rows_b);
        }
    } else if (fused) {
        S.first = PulseRuns{S.exp, S.rows, S.run_len, kPulseSortRun};
        S.second = S.first;
    } else if (settle) {
        hipLaunchKernelGGL(pulse_settle, dim3(1), dim3(64), 0, ctx->stream, ctx->T, S.exp, S.counters,
                           S.expired, k, report);
    }
    HIP_TRY(ctx, hipGetLastError());
    if (out) {
        unsigned long long h[3];
        HIP_TRY(ctx, hipMemcpyAsync(h, S.counters, sizeof(h), hipMemcpyDeviceToHost, ctx->stream));
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        out->kept = h[0];
        out->cands = h[1];
        out->next_unexpired = h[2];
    }
    return 0;
}

// Expire the first `expired` candidates (S.rows, in order), keep the still-pending entries, set
// pulse_next_timestamp.
int pulse_finish(tbg_ctx* ctx, uint64_t expired, uint64_t kept, uint64_t pulse_next) {
    PulseScratch& S = ctx->pulse;
    if (expired)
        hipLaunchKernelGGL(pulse_apply, dim3(grid_for(expired)), dim3(kBlock), 0, ctx->stream,
                           ctx->T, S.rows, expired, nullptr);
    HIP_TRY(ctx, hipGetLastError());
    // The index keeps the entries still pending (the ones just expired are dropped next time).
    if (kept)
        HIP_TRY(ctx, hipMemcpyAsync(ctx->T.expiry, S.keep, kept * 8, hipMemcpyDeviceToDevice,
                                    ctx->stream));
    unsigned long long kept_ull = kept, next_ull = pulse_next;
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->d_scalars->expiry_count, &kept_ull, 8, hipMemcpyHostToDevice,
                                ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->d_scalars->pulse_next_timestamp, &next_ull, 8,
                                hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    ctx->expiry_host = kept;
    ctx->expiry_known = true;
    return 0;
}

// The first n sorted candidates' keys to the host.
int pulse_keys(tbg_ctx* ctx, uint64_t n, std::vector<uint64_t>* exp, std::vector<uint64_t>* ts) {
    PulseScratch& S = ctx->pulse;
    exp->resize(n);
    ts->resize(n);
    if (!n) return 0;
    hipLaunchKernelGGL(pulse_key_timestamps, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream,
                       ctx->T, S.rows, n, S.ts);
    HIP_TRY(ctx, hipMemcpyAsync(exp->data(), S.exp, n * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(ts->data(), S.ts, n * 8, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

}  // namespace

extern "C" {


int tbg_register_host(tbg_ctx* ctx, void* ptr, uint64_t size) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || !ptr || size == 0) return TBG_EINVAL;
    if (is_registered(ctx, ptr, size)) return 0;
    // Several ctxs of one process (shards, state machines) may register the same message pool:
    // registrations are counted process-wide and the last user unregisters (host_pin_release).
    uintptr_t dev = 0;
    if (!host_pin_acquire(ctx, ptr, size, &dev)) return TBG_EHIP;
    ctx->registered.push_back({reinterpret_cast<uintptr_t>(ptr), size, dev});
    return 0;
}

int tbg_unregister_host(tbg_ctx* ctx, void* ptr) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    for (size_t i = 0; i < ctx->registered.size(); i++) {
        if (ctx->registered[i].host != reinterpret_cast<uintptr_t>(ptr)) continue;
        if (int rc = ae_join(ctx)) return rc;
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        host_pin_release(ptr);
        ctx->registered.erase(ctx->registered.begin() + long(i));
        return 0;
    }
    return TBG_EINVAL;
}

int tbg_synchronize(tbg_ctx* ctx) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    // (the side stream's AccountEvents appends too: the call's stream waits for them first)
    if (int rc = ae_join(ctx)) return rc;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

int64_t tbg_pulse(tbg_ctx* ctx, uint64_t timestamp) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    FAILED_GUARD(ctx);
    const uint32_t k = uint32_t(ctx->opt.pulse_batch_max);
    // The scan stops with buffer_finished after batch_max values (:4969-4999): the first batch_max
    // candidates in index order expire; everything after the host's first sync stays on device.
    tmark(ctx, "-pulse");
    static const bool htrace = getenv("TBG_PULSE_HOST_TRACE") != nullptr;
    double ht[8] = {htrace ? now_ms() : 0};
    // The expiries' AccountEvents: decided (and their staging acquired) before the pulse's
    // launches, so no host work sits between pulse_apply and the snapshot.
    const uint64_t count0 = ctx->expiry_known ? std::min<uint64_t>(ctx->expiry_host, ctx->T.expiry_capacity)
                                              : ctx->T.expiry_capacity;
    const uint32_t upper0 = uint32_t(std::min<uint64_t>(count0, k));
    bool ae_async = ctx->ae_log && upper0 && ae_async_ok(ctx, upper0) ;
    uint32_t ae_epoch = 0;
    int rc = 0;
    if (htrace) ht[1] = now_ms();
    rc = pulse_select(ctx, timestamp, k, nullptr, false, nullptr, true);
    if (rc) return rc;
    if (htrace) ht[2] = now_ms();
    // (after the selection's launches: deferred side-stream work -- a call's snapshot, which reads
    // the rows pulse_apply writes, and appends -- is queued while the selection runs; then this
    // pulse's staging buffer)
    rc = ae_flush_all(ctx);
    if (rc) return rc;
    if (ae_async) {
        rc = ae_stage_acquire(ctx);
        if (rc) return rc;
        ae_epoch = ++ctx->epoch;
    }
    tmark(ctx, "pulse:select");
    PulseScratch& S = ctx->pulse;
    const uint64_t count = std::min<uint64_t>(ctx->expiry_host, ctx->T.expiry_capacity);
    const uint32_t upper = uint32_t(std::min<uint64_t>(count, k));
    // The index keeps the entries still pending: pulse_collect wrote them to S.keep, which becomes
    // the index (the old one the next pulse's scratch; both hold expiry_capacity).
    if (count) std::swap(ctx->T.expiry, S.keep);
    // Expire, settle, report; the counters' other set cleared for the next pulse.
    hipLaunchKernelGGL(pulse_apply_root, dim3(upper ? grid_for(upper) : 1), dim3(kBlock), 0,
                       ctx->stream, S.first, S.second, S.counters, S.counters_next, ctx->T, k,
                       S.sel, S.expired, ctx->dh_pulse);
    HIP_TRY(ctx, hipGetLastError());
    std::swap(S.counters, S.counters_next);
    tmark(ctx, "pulse:apply");
    ctx->expiry_known = false;
    // The expiries' AccountEvents behind the next call (the side stream: the snapshot here, the
    // appends queued by the next call once its own kernels are queued), or here.
    if (ae_async && upper) {
        ctx->h_pulse[3] = 0;
        AeExpirySnap J{ctx->T, S.sel, S.expired, timestamp, ctx->ae_stage[ctx->ae_parity], ae_epoch,
                       ctx->dh_pulse + 3};
        hipLaunchKernelGGL(ae_expiry_snapshot, dim3(kAeAsyncMax / kSnapThreads), dim3(kSnapThreads), 0, ctx->stream, J);
        HIP_TRY(ctx, hipGetLastError());
    } else if (ctx->ae_log && upper) {
        ae_async = false;
        rc = ae_expiry(ctx, S.sel, upper, timestamp, nullptr, S.expired);
    } else {
        ae_async = false;
    }
    if (rc) return rc;
    // The count expired and the index's new length came to mapped pinned memory with the
    // settlement (pulse_apply_root: no copy-engine hand-off), which also cleared the counters the
    // next pulse takes; one synchronisation.
    S.counters_clean = true;
    if (htrace) ht[3] = now_ms();
    if (ae_async) ae_defer_graph(ctx, upper, ae_epoch, true);
    // (the host spins on a pinned word, as a call's end does: a stream synchronisation's wake-up
    // is the slower path)
    if (ctx->spin_sync) {
        const unsigned int seq = ++ctx->seq ? ctx->seq : ++ctx->seq;
        hipLaunchKernelGGL(host_signal, dim3(1), dim3(64), 0, ctx->stream, ctx->dh_seq, seq);
        HIP_TRY(ctx, hipGetLastError());
        rc = spin_wait(ctx, seq);
        if (rc) return rc;
    } else {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    }
    if (htrace) {
        ht[4] = now_ms();
        fprintf(stderr, "pulse host us: prep %.1f select %.1f rest %.1f sync %.1f\n",
                (ht[1] - ht[0]) * 1e3, (ht[2] - ht[1]) * 1e3, (ht[3] - ht[2]) * 1e3,
                (ht[4] - ht[3]) * 1e3);
    }
    tmark(ctx, "pulse:report");
    if (ctx->timing) (void)hipStreamSynchronize(ctx->stream);  // (the marks complete)
    tcollect(ctx);
    ctx->expiry_host = ctx->h_pulse[1];
    ctx->expiry_known = true;
    return int64_t(ctx->h_pulse[0]);
}

int64_t tbg_pulse_candidates(tbg_ctx* ctx, uint64_t timestamp, uint64_t* expires_at,
                             uint64_t* timestamps, uint32_t max) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    PulseGather G;
    int rc = pulse_select(ctx, timestamp, std::min<uint32_t>(max, kPulseRun), &G);
    if (rc) return rc;
    std::vector<uint64_t> e, t;
    rc = pulse_keys(ctx, std::min<uint64_t>({G.cands, max, kPulseRun}), &e, &t);
    if (rc) return rc;
    for (size_t i = 0; i < e.size(); i++) {
        if (expires_at) expires_at[i] = e[i];
        if (timestamps) timestamps[i] = t[i];
    }
    return int64_t(G.cands);
}

int64_t tbg_pulse_cut(tbg_ctx* ctx, uint64_t timestamp, uint64_t cut_expires_at,
                      uint64_t cut_timestamp, uint64_t pulse_next_timestamp,
                      const uint64_t* event_timestamps) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    PulseGather G;
    int rc = pulse_select(ctx, timestamp, uint32_t(ctx->opt.pulse_batch_max), &G);
    if (rc) return rc;
    // The cut is at most the global batch_max-th key: this shard expires at most that many.
    std::vector<uint64_t> e, t;
    rc = pulse_keys(ctx, std::min<uint64_t>(G.cands, ctx->opt.pulse_batch_max), &e, &t);
    if (rc) return rc;
    uint64_t expired = 0;
    while (expired < e.size() && (e[expired] < cut_expires_at ||
                                  (e[expired] == cut_expires_at && t[expired] <= cut_timestamp)))
        expired++;
    // 0: this shard's own next expiry (every candidate at or before the cut expires), as tbg_pulse.
    uint64_t pulse_next = pulse_next_timestamp;
    if (pulse_next == 0) {
        pulse_next = G.next_unexpired == ~0ull ? TB_TIMESTAMP_MAX : G.next_unexpired;
        if (expired < e.size()) pulse_next = std::min(pulse_next, e[expired]);
    }
    // The AccountEvents' stamps: the expiries' positions across all shards.
    uint64_t* d_stamps = nullptr;
    if (event_timestamps && expired && ctx->ae_log) {
        d_stamps = ctx->pulse.exp_b;  // (free after pulse_gather's sort)
        HIP_TRY(ctx, hipMemcpyAsync(d_stamps, event_timestamps, expired * 8, hipMemcpyHostToDevice,
                                    ctx->stream));
    }
    rc = pulse_finish(ctx, expired, G.kept, pulse_next);
    if (!rc && ctx->ae_log) rc = ae_expiry(ctx, ctx->pulse.rows, expired, timestamp, d_stamps);
    if (!rc && d_stamps) HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // (host stamps)
    return rc ? rc : int64_t(expired);
}

int tbg_raise_key_max(tbg_ctx* ctx, uint64_t accounts_key_max, uint64_t transfers_key_max) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    int rc = sync_scalars(ctx);
    if (rc) return rc;
    unsigned long long a = std::max<unsigned long long>(ctx->h_scalars->accounts_key_max,
                                                        accounts_key_max);
    unsigned long long t = std::max<unsigned long long>(ctx->h_scalars->transfers_key_max,
                                                        transfers_key_max);
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->d_scalars->accounts_key_max, &a, 8, hipMemcpyHostToDevice,
                                ctx->stream));
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->d_scalars->transfers_key_max, &t, 8, hipMemcpyHostToDevice,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return 0;
}

int64_t tbg_forget_orphans(tbg_ctx* ctx, const tb_uint128_t* ids, uint32_t n) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || n > ctx->opt.batch_events_max || (n && !ids)) return TBG_EINVAL;
    FAILED_GUARD(ctx);
    if (n == 0) return 0;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_events, ids, size_t(n) * 16, hipMemcpyHostToDevice,
                                ctx->stream));
    unsigned int* d_count = &ctx->d_scalars->slow_count;  // scratch word (between calls)
    HIP_TRY(ctx, hipMemsetAsync(d_count, 0, 4, ctx->stream));
    hipLaunchKernelGGL(forget_orphans_kernel, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream,
                       ctx->T, reinterpret_cast<const tb_uint128_t*>(ctx->d_events), n, d_count);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->h_scalars->slow_count, d_count, 4, hipMemcpyDeviceToHost,
                                ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return ctx->h_scalars->slow_count;
}

int64_t tbg_timestamps_exist(tbg_ctx* ctx, int transfers, const uint64_t* timestamps, uint32_t n,
                             uint8_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || n > ctx->opt.batch_events_max || (n && (!timestamps || !out))) return TBG_EINVAL;
    FAILED_GUARD(ctx);
    if (n == 0) return 0;
    // (check_imported_indexes rebuilds the index an imported call of the *other* groove reads)
    int rc = check_imported_indexes(ctx, transfers == 0);
    if (rc) return rc;
    uint64_t* d_ts = reinterpret_cast<uint64_t*>(ctx->d_events);
    uint8_t* d_out = reinterpret_cast<uint8_t*>(d_ts + n);
    HIP_TRY(ctx, hipMemcpyAsync(d_ts, timestamps, size_t(n) * 8, hipMemcpyHostToDevice,
                                ctx->stream));
    const uint64_t* index = transfers ? ctx->tr_ts_index : ctx->acc_ts_index;
    const uint64_t count = transfers ? ctx->T.tr_ts_count : ctx->T.acc_ts_count;
    hipLaunchKernelGGL(timestamps_exist_kernel, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream,
                       index, count, d_ts, n, d_out);
    HIP_TRY(ctx, hipGetLastError());
    HIP_TRY(ctx, hipMemcpyAsync(out, d_out, n, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    int64_t found = 0;
    for (uint32_t i = 0; i < n; i++) found += out[i];
    return found;
}

int tbg_key_max(tbg_ctx* ctx, uint64_t* accounts_key_max, uint64_t* transfers_key_max) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    FAILED_GUARD(ctx);
    int rc = sync_scalars(ctx);
    if (rc) return rc;
    if (accounts_key_max) *accounts_key_max = ctx->h_scalars->accounts_key_max;
    if (transfers_key_max) *transfers_key_max = ctx->h_scalars->transfers_key_max;
    return 0;
}

uint64_t tbg_pulse_next_timestamp(tbg_ctx* ctx) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || sync_scalars(ctx)) return 0;
    return ctx->h_scalars->pulse_next_timestamp;
}

int tbg_set_pnt_sharded(tbg_ctx* ctx, int on) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    ctx->pnt_sharded = on != 0;
    ctx->pnt_last_valid = false;
    return 0;
}

int64_t tbg_pnt_ops(tbg_ctx* ctx, uint64_t* timestamps, uint64_t* ops, uint64_t max,
                    uint64_t* start) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    FAILED_GUARD(ctx);
    if (!ctx->pnt_last_valid) {  // (no sharded call since: nothing recorded)
        if (start) *start = tbg_pulse_next_timestamp(ctx);
        return 0;
    }
    const Call<tb_transfer_t>& c = ctx->pnt_last;
    hipLaunchKernelGGL(pnt_flags, dim3(grid_for(c.n)), dim3(kBlock), 0, ctx->stream, c.pnt_call,
                       c.n, ctx->ev_slow);
    unsigned int* d_count = &ctx->d_scalars->slow_count;  // scratch word (between calls)
    int rc = select_flagged(ctx, ctx->ev_slow, c.n, ctx->slow_list, d_count);
    if (rc) return rc;
    hipLaunchKernelGGL(pnt_gather, dim3(grid_for(c.n)), dim3(kBlock), 0, ctx->stream, c,
                       ctx->slow_list, d_count, ctx->bal_items);
    HIP_TRY(ctx, hipGetLastError());
    rc = sync_scalars(ctx);
    if (rc) return rc;
    const uint64_t m = ctx->h_scalars->slow_count;
    unsigned long long st = 0;
    HIP_TRY(ctx, hipMemcpy(&st, ctx->pnt_fired + 2, 8, hipMemcpyDeviceToHost));
    if (start) *start = st;
    if (m && (timestamps || ops)) {
        std::vector<uint64_t> pairs(2 * m);
        HIP_TRY(ctx, hipMemcpy(pairs.data(), ctx->bal_items, 16 * m, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < std::min(m, max); i++) {
            if (timestamps) timestamps[i] = pairs[2 * i];
            if (ops) ops[i] = pairs[2 * i + 1];
        }
    }
    return int64_t(m);
}

int tbg_set_pulse_next_timestamp(tbg_ctx* ctx, uint64_t value) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    FAILED_GUARD(ctx);
    const unsigned long long v = value;
    HIP_TRY(ctx, hipMemcpyAsync(&ctx->d_scalars->pulse_next_timestamp, &v, 8,
                                hipMemcpyHostToDevice, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));  // (`v` is a stack value)
    return 0;
}

int64_t tbg_lookup_accounts(tbg_ctx* ctx, const tb_uint128_t* ids, uint32_t n, tb_account_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    return lookup_impl(ctx, ids, n, out, true);
}

int64_t tbg_lookup_transfers(tbg_ctx* ctx, const tb_uint128_t* ids, uint32_t n,
                             tb_transfer_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    return lookup_impl(ctx, ids, n, out, false);
}

int64_t tbg_dump_accounts(tbg_ctx* ctx, tb_account_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    return dump_impl(ctx, ctx->T.acc_rows, ctx->T.acc_live, ctx->T.acc_rows_used, out, nullptr);
}

int64_t tbg_dump_transfers(tbg_ctx* ctx, tb_transfer_t* out, uint8_t* pending_status) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    return dump_impl(ctx, ctx->T.tr_rows, ctx->T.tr_live, ctx->T.tr_rows_used, out,
                     pending_status);
}

// Rows an occupied id slot references: created transfers and orphaned ids (tombstones and empty
// slots reference none).
__global__ void mark_slot_rows(const unsigned long long* slots, uint64_t n_slots, uint8_t* flags,
                               uint64_t used) {
    const uint64_t s = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x;
    if (s >= n_slots) return;
    const uint64_t w = slots[s];
    if (w == kEmpty || w == kTomb) return;
    const uint64_t r = (w & kRefMask) - 1;
    if (r < used) flags[r] = 1;
}
__global__ void gather_transfer_ids(const tb_transfer_t* rows, const uint32_t* sel, uint32_t n,
                                    tb_uint128_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = rows[sel[i]].id;
}

int64_t tbg_dump_transfer_ids(tbg_ctx* ctx, tb_uint128_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    const uint64_t used = ctx->T.tr_rows_used;
    if (used == 0) return 0;
    uint8_t* flags = nullptr;
    if (!dev_alloc(ctx, &flags, used, true)) return TBG_ENOMEM;
    const uint64_t n_slots = ctx->T.tr.mask + 1;
    hipLaunchKernelGGL(mark_slot_rows, dim3(grid_for(n_slots)), dim3(kBlock), 0, ctx->stream,
                       ctx->T.tr.slots, n_slots, flags, used);
    unsigned int* d_count = &ctx->d_scalars->slow_count;
    int64_t result = select_flagged(ctx, flags, used, ctx->sel_buf, d_count);
    if (result == 0 && !hip_ok(ctx, hipMemcpyAsync(&ctx->h_scalars->slow_count, d_count, 4,
                                                   hipMemcpyDeviceToHost, ctx->stream), "count"))
        result = TBG_EHIP;
    if (result == 0 && !hip_ok(ctx, hipStreamSynchronize(ctx->stream), "sync")) result = TBG_EHIP;
    const uint64_t count = result == 0 ? ctx->h_scalars->slow_count : 0;
    if (result == 0 && out && count) {
        tb_uint128_t* d_out = nullptr;
        if (!dev_alloc(ctx, &d_out, count, false)) {
            result = TBG_ENOMEM;
        } else {
            hipLaunchKernelGGL(gather_transfer_ids, dim3(grid_for(count)), dim3(kBlock), 0,
                               ctx->stream, ctx->T.tr_rows, ctx->sel_buf, uint32_t(count), d_out);
            if (!hip_ok(ctx, hipMemcpyAsync(out, d_out, count * sizeof(tb_uint128_t),
                                            hipMemcpyDeviceToHost, ctx->stream), "ids copy"))
                result = TBG_EHIP;
            (void)hipStreamSynchronize(ctx->stream);
            (void)hipFree(d_out);
        }
    }
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipFree(flags);
    return result < 0 ? result : int64_t(count);
}

int tbg_debug_set_account_balances(tbg_ctx* ctx, tb_uint128_t id, tb_uint128_t debits_pending,
                                   tb_uint128_t debits_posted, tb_uint128_t credits_pending,
                                   tb_uint128_t credits_posted) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    if (int rc = ae_flush_all(ctx)) return rc;  // (a deferred snapshot reads the rows)
    int* d_rc = reinterpret_cast<int*>(&ctx->d_scalars->slow_count);
    hipLaunchKernelGGL(set_balances_kernel, dim3(1), dim3(1), 0, ctx->stream, ctx->T, id,
                       debits_pending, debits_posted, credits_pending, credits_posted, d_rc);
    HIP_TRY(ctx, hipGetLastError());
    int rc = 0;
    HIP_TRY(ctx, hipMemcpyAsync(&rc, d_rc, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return rc;
}

int64_t tbg_dump_account_events(tbg_ctx* ctx, tb_account_event_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    if (int rc = ae_settle(ctx)) return rc;
    if (!out || ctx->ae_used == 0) return int64_t(ctx->ae_used);
    int rc = ae_sort_log(ctx);
    if (rc) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(out, ctx->ae_log, ctx->ae_used * sizeof(tb_account_event_t),
                                hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    return int64_t(ctx->ae_used);
}

int64_t tbg_get_change_events(tbg_ctx* ctx, const tb_change_events_filter_t* filter,
                              uint32_t limit_max, tb_change_event_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || !filter) return TBG_EINVAL;
    // get_scan_from_change_events_filter (:2396-2434): an invalid filter yields no results.
    bool reserved_zero = true;
    for (int i = 0; i < 44; i++) reserved_zero &= filter->reserved[i] == 0;
    const uint64_t tmin = filter->timestamp_min, tmax = filter->timestamp_max;
    const bool valid = (tmin == 0 || (tmin >= TB_TIMESTAMP_MIN && tmin <= TB_TIMESTAMP_MAX)) &&
                       (tmax == 0 || (tmax >= TB_TIMESTAMP_MIN && tmax <= TB_TIMESTAMP_MAX)) &&
                       (tmax == 0 || tmin <= tmax) && filter->limit != 0 && reserved_zero;
    if (int rc = ae_settle(ctx)) return rc;
    if (!valid || ctx->ae_used == 0) return 0;
    int rc = ae_sort_log(ctx);
    if (rc) return rc;
    const uint64_t lo = tmin == 0 ? TB_TIMESTAMP_MIN : tmin;
    const uint64_t hi = tmax == 0 ? TB_TIMESTAMP_MAX : tmax;
    hipLaunchKernelGGL(ae_bounds, dim3(1), dim3(64), 0, ctx->stream, ctx->ae_log, ctx->ae_used, lo,
                       hi, ctx->ae_words);
    unsigned long long b[2] = {0, 0};
    HIP_TRY(ctx, hipMemcpyAsync(b, ctx->ae_words, 16, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t limit = std::min<uint64_t>(filter->limit, limit_max);
    const uint32_t count = uint32_t(std::min<uint64_t>(limit, b[1] - b[0]));
    if (count == 0 || !out) return count;
    tb_change_event_t* d_out = nullptr;
    if (!dev_alloc(ctx, &d_out, count, false)) return TBG_ENOMEM;
    hipLaunchKernelGGL(ae_change_events, dim3(grid_for(count)), dim3(kBlock), 0, ctx->stream,
                       ctx->T, ctx->ae_log, ctx->ae_ref, b[0], count, d_out);
    int64_t result = count;
    if (!hip_ok(ctx, hipMemcpyAsync(out, d_out, size_t(count) * sizeof(tb_change_event_t),
                                    hipMemcpyDeviceToHost, ctx->stream), "change events copy") ||
        !hip_ok(ctx, hipStreamSynchronize(ctx->stream), "sync"))
        result = TBG_EHIP;
    (void)hipFree(d_out);
    return result;
}

int tbg_last_stats(tbg_ctx* ctx, tbg_stats* out) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || !out) return TBG_EINVAL;
    *out = ctx->stats;
    return 0;
}

}  // extern "C"

namespace {

__device__ __host__ inline uint8_t sum_overflows_bits(uint32_t bits, const tb_uint128_t& a,
                                                      const tb_uint128_t& b) {
    return bits == 64 ? uint8_t(sum_overflows<uint64_t>(a.lo, b.lo))
                      : uint8_t(sum_overflows<u128>(U(a), U(b)));
}

__global__ void sum_overflows_kernel(uint32_t bits, const tb_uint128_t* a, const tb_uint128_t* b,
                                     uint32_t n, uint8_t* out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = sum_overflows_bits(bits, a[i], b[i]);
}

}  // namespace

extern "C" {

int tbg_sum_overflows(tbg_ctx* ctx, uint32_t bits, const tb_uint128_t* a, const tb_uint128_t* b,
                      uint32_t n, uint8_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    if ((bits != 64 && bits != 128) || (n && (!a || !b || !out))) return TBG_EINVAL;
    if (!ctx) {
        for (uint32_t i = 0; i < n; i++) out[i] = sum_overflows_bits(bits, a[i], b[i]);
        return 0;
    }
    if (n == 0) return 0;
    tb_uint128_t* d = nullptr;
    uint8_t* d_out = nullptr;
    int rc = dev_alloc(ctx, &d, 2 * uint64_t(n), false) && dev_alloc(ctx, &d_out, n, false)
                 ? 0 : TBG_ENOMEM;
    if (!rc && !(hip_ok(ctx, hipMemcpyAsync(d, a, n * 16ull, hipMemcpyHostToDevice, ctx->stream),
                        "copy") &&
                 hip_ok(ctx, hipMemcpyAsync(d + n, b, n * 16ull, hipMemcpyHostToDevice,
                                            ctx->stream), "copy")))
        rc = TBG_EHIP;
    if (!rc) {
        hipLaunchKernelGGL(sum_overflows_kernel, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream,
                           bits, d, d + n, n, d_out);
        if (!hip_ok(ctx, hipGetLastError(), "launch") ||
            !hip_ok(ctx, hipMemcpyAsync(out, d_out, n, hipMemcpyDeviceToHost, ctx->stream), "copy") ||
            !hip_ok(ctx, hipStreamSynchronize(ctx->stream), "sync"))
            rc = TBG_EHIP;
    }
    if (d) (void)hipFree(d);
    if (d_out) (void)hipFree(d_out);
    return rc;
}

int tbg_debug_force_replay(tbg_ctx* ctx, int enable) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    ctx->force_replay = enable != 0;
    return 0;
}

int tbg_debug_serial_replay(tbg_ctx* ctx, int enable) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    ctx->serial_replay = enable != 0;
    return 0;
}

int tbg_debug_ae_sync(tbg_ctx* ctx, int enable) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    ctx->ae_async = enable == 0;
    return 0;
}

int tbg_profile(tbg_ctx* ctx, int enable) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return TBG_EINVAL;
    ctx->timing = enable == 1 || enable == 3;
    ctx->timing_lean = enable == 3;
    ctx->timing_host = enable != 0;
    ctx->prof_names.clear();
    ctx->prof_ms.clear();
    ctx->prof_count.clear();
    return 0;
}

int tbg_profile_read(tbg_ctx* ctx, uint32_t index, char* name, uint32_t name_len,
                     double* total_ms, uint64_t* launches) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx) return 0;
    if (index == 0 && ctx->timing && ctx->n_marks > 1) {  // marks still pending (AccountEvents)
        (void)hipStreamSynchronize(ctx->stream);
        tcollect(ctx);
    }
    if (index >= ctx->prof_names.size()) return 0;
    if (name && name_len) snprintf(name, name_len, "%s", ctx->prof_names[index].c_str());
    if (total_ms) *total_ms = ctx->prof_ms[index];
    if (launches) *launches = ctx->prof_count[index];
    return 1;
}

}  // extern "C"

// ---- Durability (durability.hpp) ----------------------------------------------------------------

namespace {

// Checkpoint image: a header, the persistent tables in a fixed order, then a footer holding a
// checksum of the header and of every section (tbg_checkpoint); tbg_open_checkpoint installs
// nothing unless every checksum matches.
struct CkptHeader {
    char magic[8];
    uint32_t version, epoch;
    tbg_options opt;
    uint64_t acc_rows_used, tr_rows_used, ae_used, ae_last_ts;
    uint64_t acc_slots, tr_slots, acc_entries;
    uint32_t ae_sorted, pad;
    DevScalars scalars;
};
constexpr char kCkptMagic[8] = {'T', 'B', 'G', 'C', 'K', 'P', 'T', '2'};
constexpr uint32_t kCkptVersion = 3;  // (3: DevScalars::fixed)
constexpr uint32_t kCkptSections = 12;
struct CkptFooter {
    char magic[8];
    uint64_t header_checksum;
    uint64_t section_checksum[kCkptSections];
};
constexpr size_t kStageBytes = size_t(64) << 20;

// A streaming 64-bit checksum of a byte sequence (8 bytes per step, a multiply-rotate mix; the
// tail bytes as one short word); the sequence's length is folded in by ck_finish.
struct Checksum {
    uint64_t h = 0x243F6A8885A308D3ull, len = 0;
    void add(const uint8_t* p, size_t n) {
        size_t i = 0;
        for (; i + 8 <= n; i += 8) {
            uint64_t w;
            memcpy(&w, p + i, 8);
            h = ((h << 29) | (h >> 35)) ^ w;
            h *= 0x9E3779B97F4A7C15ull;
        }
        if (i < n) {  // (only at a section's end: staged chunks are multiples of 8 bytes)
            uint64_t w = 0;
            memcpy(&w, p + i, n - i);
            h = ((h << 29) | (h >> 35)) ^ w;
            h *= 0x9E3779B97F4A7C15ull;
        }
        len += n;
    }
    uint64_t finish() const {
        uint64_t x = h ^ len;
        x ^= x >> 33;
        x *= 0xFF51AFD7ED558CCDull;
        x ^= x >> 33;
        return x;
    }
};

// Device <-> file through one pinned staging buffer; each section's checksum as it passes.
struct Stager {
    tbg_ctx* ctx;
    FILE* f;
    uint8_t* host = nullptr;
    bool ok = true;
    Stager(tbg_ctx* c, FILE* file) : ctx(c), f(file) {
        ok = hip_ok(ctx, hipHostMalloc(reinterpret_cast<void**>(&host), kStageBytes), "stage");
    }
    ~Stager() {
        if (host) (void)hipHostFree(host);
    }
    bool write(const void* dev, uint64_t bytes, uint64_t* checksum) {
        const uint8_t* d = static_cast<const uint8_t*>(dev);
        Checksum ck;
        for (uint64_t off = 0; ok && off < bytes; off += kStageBytes) {
            const size_t n = size_t(std::min<uint64_t>(kStageBytes, bytes - off));
            ok = hip_ok(ctx, hipMemcpyAsync(host, d + off, n, hipMemcpyDeviceToHost, ctx->stream),
                        "checkpoint copy") &&
                 hip_ok(ctx, hipStreamSynchronize(ctx->stream), "checkpoint sync") &&
                 fwrite(host, 1, n, f) == n;
            if (ok) ck.add(host, n);
            if (!ok && ctx->error.empty()) ctx->error = "checkpoint write";
        }
        *checksum = ck.finish();
        return ok;
    }
    bool read(void* dev, uint64_t bytes, uint64_t* checksum) {
        uint8_t* d = static_cast<uint8_t*>(dev);
        Checksum ck;
        for (uint64_t off = 0; ok && off < bytes; off += kStageBytes) {
            const size_t n = size_t(std::min<uint64_t>(kStageBytes, bytes - off));
            ok = fread(host, 1, n, f) == n &&
                 hip_ok(ctx, hipMemcpyAsync(d + off, host, n, hipMemcpyHostToDevice, ctx->stream),
                        "restore copy");
            if (ok) ck.add(host, n);
            ok = ok && hip_ok(ctx, hipStreamSynchronize(ctx->stream), "restore sync");
            if (!ok && ctx->error.empty()) ctx->error = "checkpoint image truncated";
        }
        *checksum = ck.finish();
        return ok;
    }
};

uint64_t header_checksum(const CkptHeader& h) {
    Checksum ck;
    ck.add(reinterpret_cast<const uint8_t*>(&h), sizeof(h));
    return ck.finish();
}

// fsync of the directory holding `path` (a rename is durable once its directory is).
bool fsync_parent(const std::string& path) {
    const size_t slash = path.find_last_of('/');
    const std::string dir = slash == std::string::npos ? "." : (slash == 0 ? "/" : path.substr(0, slash));
    const int fd = open(dir.c_str(), O_RDONLY | O_DIRECTORY);
    if (fd < 0) return false;
    const bool ok = fsync(fd) == 0;
    close(fd);
    return ok;
}

uint64_t acc_slot_count(const tbg_ctx* ctx) { return ctx->T.acc.mask + 1; }
uint64_t tr_slot_count(const tbg_ctx* ctx) { return ctx->T.tr.mask + 1; }
uint64_t acc_entry_count(const tbg_ctx* ctx) { return ctx->T.acc_index.mask + 1; }

// The persistent tables, in image order: (device pointer, bytes).
std::vector<std::pair<void*, uint64_t>> ckpt_sections(tbg_ctx* ctx, uint64_t acc_used,
                                                      uint64_t tr_used, uint64_t expiry_count,
                                                      uint64_t ae_used) {
    Tables& T = ctx->T;
    return {
        {T.acc.slots, acc_slot_count(ctx) * 8},
        {T.acc_index.entries, acc_entry_count(ctx) * sizeof(AccEntry)},
        {T.acc_entry_of, acc_used * 4},
        {T.acc_rows, acc_used * sizeof(tb_account_t)},
        {T.acc_live, acc_used},
        {T.tr.slots, tr_slot_count(ctx) * 8},
        {T.tr_rows, tr_used * sizeof(tb_transfer_t)},
        {T.tr_live, tr_used},
        {T.tr_status, tr_used},
        {T.expiry, expiry_count * 8},
        {ctx->ae_log, ae_used * sizeof(tb_account_event_t)},
        {ctx->ae_ref, ae_used * sizeof(AeRef)},
    };
}

}  // namespace

extern "C" {

int64_t tbg_compact(tbg_ctx* ctx) {
    TBG_DEVICE_SCOPE(ctx);
    if (ctx) ctx->expiry_known = false;  // (compaction renumbers and drops index entries)
    if (!ctx) return TBG_EINVAL;
    FAILED_GUARD(ctx);
    Tables& T = ctx->T;
    const uint64_t used = T.tr_rows_used;
    if (used == 0) return 0;
    if (int rc = ae_join(ctx)) return rc;  // (the side stream's appends read transfer rows)
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_scalars, ctx->d_scalars, sizeof(DevScalars),
                                hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    const uint64_t expiry_count = ctx->h_scalars->expiry_count;
    const uint64_t chunk = std::min<uint64_t>(used, uint64_t(1) << 22);
    uint32_t *keep32 = nullptr, *new_row = nullptr, *sel = nullptr;
    tb_transfer_t* c_rows = nullptr;
    uint8_t *c_live = nullptr, *c_status = nullptr, *x_flags = nullptr;
    uint64_t* x_out = nullptr;
    unsigned int* d_words = nullptr;
    int64_t rc = 0;
    const uint64_t xn = std::max<uint64_t>(expiry_count, 1);
    if (!(dev_alloc(ctx, &keep32, used + 1, true) && dev_alloc(ctx, &new_row, used + 1, false) &&
          dev_alloc(ctx, &c_rows, chunk, false) && dev_alloc(ctx, &c_live, chunk, false) &&
          dev_alloc(ctx, &c_status, chunk, false) && dev_alloc(ctx, &x_flags, xn, false) &&
          dev_alloc(ctx, &sel, xn, false) && dev_alloc(ctx, &x_out, xn, false) &&
          dev_alloc(ctx, &d_words, 2, true)))
        rc = TBG_ENOMEM;
    uint32_t kept = 0;
    if (!rc) {
        hipLaunchKernelGGL(cmp_mark, dim3(grid_for(tr_slot_count(ctx))), dim3(kBlock), 0,
                           ctx->stream, T.tr, used, keep32);
        // (keep32[used] = 0: new_row[used] is the kept count; one chained scan, prims.hpp)
        rc = launch_scan(ctx, used + 1, ExclusiveSumU32{keep32, new_row, nullptr});
        if (!rc && !(hip_ok(ctx, hipMemcpyAsync(&kept, new_row + used, 4, hipMemcpyDeviceToHost,
                                                ctx->stream), "kept") &&
                     hip_ok(ctx, hipStreamSynchronize(ctx->stream), "sync")))
            rc = TBG_EHIP;
    }
    // From the first row move on, a failure leaves the tables undefined (ctx->failed).
    const bool mutating = !rc;
    // Rows move down in place, one chunk at a time: chunk [a, b)'s kept rows go to
    // [new_row[a], new_row[b]), which ends at or before b and starts after every earlier chunk's.
    for (uint64_t a = 0; !rc && a < used; a += chunk) {
        const uint64_t b = std::min(used, a + chunk);
        uint32_t bounds[2] = {0, 0};
        if (!(hip_ok(ctx, hipMemcpyAsync(&bounds[0], new_row + a, 4, hipMemcpyDeviceToHost,
                                         ctx->stream), "bounds") &&
              hip_ok(ctx, hipMemcpyAsync(&bounds[1], new_row + b, 4, hipMemcpyDeviceToHost,
                                         ctx->stream), "bounds") &&
              hip_ok(ctx, hipStreamSynchronize(ctx->stream), "sync"))) {
            rc = TBG_EHIP;
            break;
        }
        const uint64_t cnt = bounds[1] - bounds[0];
        if (cnt == 0 || (cnt == b - a && bounds[0] == a)) continue;  // nothing kept / nothing moves
        hipLaunchKernelGGL(cmp_gather, dim3(grid_for(b - a)), dim3(kBlock), 0, ctx->stream,
                           T.tr_rows, T.tr_live, T.tr_status, keep32, new_row, a, b, bounds[0],
                           c_rows, c_live, c_status);
        if (!(hip_ok(ctx, hipMemcpyAsync(T.tr_rows + bounds[0], c_rows, cnt * sizeof(tb_transfer_t),
                                         hipMemcpyDeviceToDevice, ctx->stream), "move rows") &&
              hip_ok(ctx, hipMemcpyAsync(T.tr_live + bounds[0], c_live, cnt,
                                         hipMemcpyDeviceToDevice, ctx->stream), "move live") &&
              hip_ok(ctx, hipMemcpyAsync(T.tr_status + bounds[0], c_status, cnt,
                                         hipMemcpyDeviceToDevice, ctx->stream), "move status")))
            rc = TBG_EHIP;
    }
    if (!rc) {
        // Fresh rows read as dead with TransferPending none.
        if (!(hip_ok(ctx, hipMemsetAsync(T.tr_live + kept, 0, used - kept, ctx->stream), "clear") &&
              hip_ok(ctx, hipMemsetAsync(T.tr_status + kept, 0, used - kept, ctx->stream), "clear") &&
              hip_ok(ctx, hipMemsetAsync(T.tr.slots, 0, tr_slot_count(ctx) * 8, ctx->stream),
                     "clear slots")))
            rc = TBG_EHIP;
    }
    if (!rc && kept) {
        hipLaunchKernelGGL(cmp_insert, dim3(grid_for(kept)), dim3(kBlock), 0, ctx->stream, T.tr,
                           T.tr_rows, T.tr_live, uint64_t(kept), d_words);
    }
    uint64_t x_kept = 0;
    if (!rc && expiry_count) {
        hipLaunchKernelGGL(cmp_expiry_flags, dim3(grid_for(expiry_count)), dim3(kBlock), 0,
                           ctx->stream, T.expiry, expiry_count, used, keep32, x_flags);
        rc = select_flagged(ctx, x_flags, expiry_count, sel, d_words + 1);
        unsigned int xk = 0;
        if (!rc && !(hip_ok(ctx, hipMemcpyAsync(&xk, d_words + 1, 4, hipMemcpyDeviceToHost,
                                                ctx->stream), "expiry count") &&
                     hip_ok(ctx, hipStreamSynchronize(ctx->stream), "sync")))
            rc = TBG_EHIP;
        x_kept = xk;
        if (!rc && x_kept) {
            hipLaunchKernelGGL(cmp_expiry_gather, dim3(grid_for(x_kept)), dim3(kBlock), 0,
                               ctx->stream, T.expiry, sel, x_kept, new_row, x_out);
            if (!hip_ok(ctx, hipMemcpyAsync(T.expiry, x_out, x_kept * 8, hipMemcpyDeviceToDevice,
                                            ctx->stream), "expiry"))
                rc = TBG_EHIP;
        }
    }
    if (!rc) rc = ae_settle(ctx);
    if (!rc && ctx->ae_used)
        hipLaunchKernelGGL(cmp_ae_refs, dim3(grid_for(ctx->ae_used)), dim3(kBlock), 0, ctx->stream,
                           ctx->ae_ref, ctx->ae_used, new_row);
    unsigned int failed = 0;
    if (!rc) {
        const unsigned long long xc = x_kept;
        if (!(hip_ok(ctx, hipGetLastError(), "compact launch") &&
              hip_ok(ctx, hipMemcpyAsync(&ctx->d_scalars->expiry_count, &xc, 8,
                                         hipMemcpyHostToDevice, ctx->stream), "expiry count") &&
              hip_ok(ctx, hipMemcpyAsync(&failed, d_words, 4, hipMemcpyDeviceToHost, ctx->stream),
                     "insert") &&
              hip_ok(ctx, hipStreamSynchronize(ctx->stream), "compact sync")))
            rc = TBG_EHIP;
    }
    if (!rc && failed) {
        ctx->error = "id index full during compaction";
        rc = TBG_ENOSPC;
    }
    if (!rc) {
        T.tr_rows_used = kept;
        ctx->tr_ts_stale = true;
        rc = int64_t(used - kept);
    } else if (mutating) {
        ctx->failed = true;
        ctx->error = "compaction failed after moving rows (" + ctx->error + "): tables undefined";
    }
    for (void* p : {(void*)keep32, (void*)new_row, (void*)sel, (void*)c_rows, (void*)c_live,
                    (void*)c_status, (void*)x_flags, (void*)x_out, (void*)d_words})
        if (p) (void)hipFree(p);
    return rc;
}

int tbg_checkpoint(tbg_ctx* ctx, const char* path) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || !path) return TBG_EINVAL;
    FAILED_GUARD(ctx);  // (never persist undefined tables)
    if (int rc = ae_join(ctx)) return rc;
    HIP_TRY(ctx, hipMemcpyAsync(ctx->h_scalars, ctx->d_scalars, sizeof(DevScalars),
                                hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    int rc = ae_sort_log(ctx);
    if (rc) return rc;
    CkptHeader h{};
    memcpy(h.magic, kCkptMagic, 8);
    h.version = kCkptVersion;
    h.epoch = ctx->epoch;
    h.opt = ctx->opt;
    h.acc_rows_used = ctx->T.acc_rows_used;
    h.tr_rows_used = ctx->T.tr_rows_used;
    h.ae_used = ctx->ae_used;
    h.ae_last_ts = ctx->ae_last_ts;
    h.acc_slots = acc_slot_count(ctx);
    h.tr_slots = tr_slot_count(ctx);
    h.acc_entries = acc_entry_count(ctx);
    h.ae_sorted = 1;
    h.scalars = *ctx->h_scalars;
    // (per-call words are not state)
    memset(&h.scalars.flags, 0, sizeof(DevScalars) - offsetof(DevScalars, flags));
    const std::string tmp = std::string(path) + ".tmp";
    FILE* f = fopen(tmp.c_str(), "wb");
    if (!f) {
        ctx->error = "checkpoint: cannot create " + tmp;
        return TBG_EINVAL;
    }
    bool ok = fwrite(&h, sizeof(h), 1, f) == 1;
    CkptFooter foot{};
    memcpy(foot.magic, kCkptMagic, 8);
    foot.header_checksum = header_checksum(h);
    {
        Stager st(ctx, f);
        ok = ok && st.ok;
        const auto secs = ckpt_sections(ctx, h.acc_rows_used, h.tr_rows_used,
                                        h.scalars.expiry_count, h.ae_used);
        for (size_t i = 0; i < secs.size(); i++)
            ok = ok && st.write(secs[i].first, secs[i].second, &foot.section_checksum[i]);
    }
    ok = ok && fwrite(&foot, sizeof(foot), 1, f) == 1;
    // Durable before it becomes the image: the data (fsync), then the name (rename + the
    // directory's fsync) -- the superblock's atomic switch.
    ok = fflush(f) == 0 && ok;
    ok = ok && fsync(fileno(f)) == 0;
    ok = fclose(f) == 0 && ok;
    if (ok) ok = rename(tmp.c_str(), path) == 0 && fsync_parent(path);
    if (!ok) {
        if (ctx->error.empty()) ctx->error = "checkpoint: write failed";
        remove(tmp.c_str());
        return TBG_EHIP;
    }
    return 0;
}

tbg_ctx* tbg_open_checkpoint(const tbg_options* options, const char* path) {
    if (!options || !path) return nullptr;
    FILE* f = fopen(path, "rb");
    if (!f) return nullptr;
    CkptHeader h{};
    if (fread(&h, sizeof(h), 1, f) != 1 || memcmp(h.magic, kCkptMagic, 8) != 0 ||
        h.version != kCkptVersion) {
        fclose(f);
        return nullptr;
    }
    tbg_ctx* ctx = tbg_open(options);
    if (!ctx) {
        fclose(f);
        return nullptr;
    }
    // The id tables are restored slot for slot: the table geometry must match the image's.
    bool ok = acc_slot_count(ctx) == h.acc_slots && tr_slot_count(ctx) == h.tr_slots &&
              acc_entry_count(ctx) == h.acc_entries &&
              h.acc_rows_used <= options->account_capacity &&
              h.tr_rows_used <= options->transfer_capacity &&
              h.scalars.expiry_count <= ctx->T.expiry_capacity && h.ae_used <= ctx->ae_cap;
    CkptFooter foot{};
    if (ok) {
        Stager st(ctx, f);
        ok = st.ok;
        const auto secs = ckpt_sections(ctx, h.acc_rows_used, h.tr_rows_used,
                                        h.scalars.expiry_count, h.ae_used);
        uint64_t sums[kCkptSections] = {};
        for (size_t i = 0; i < secs.size(); i++)
            ok = ok && st.read(secs[i].first, secs[i].second, &sums[i]);
        // Nothing is installed unless the header and every section match their checksums.
        ok = ok && fread(&foot, sizeof(foot), 1, f) == 1 &&
             memcmp(foot.magic, kCkptMagic, 8) == 0 &&
             foot.header_checksum == header_checksum(h);
        for (size_t i = 0; ok && i < secs.size(); i++) ok = foot.section_checksum[i] == sums[i];
        if (!ok) fprintf(stderr, "tbg_open_checkpoint: %s: image corrupt or truncated\n", path);
    }
    fclose(f);
    if (ok)
        ok = hip_ok(ctx, hipMemcpyAsync(ctx->d_scalars, &h.scalars, sizeof(DevScalars),
                                        hipMemcpyHostToDevice, ctx->stream), "scalars") &&
             hip_ok(ctx, hipStreamSynchronize(ctx->stream), "sync");
    if (!ok) {
        tbg_close(ctx);
        return nullptr;
    }
    ctx->T.acc_rows_used = h.acc_rows_used;
    ctx->T.tr_rows_used = h.tr_rows_used;
    ctx->epoch = h.epoch;  // (the epoch marks start zeroed: no stale mark matches a later call)
    ctx->ae_used = h.ae_used;
    ctx->ae_last_ts = h.ae_last_ts;
    ctx->ae_sorted = h.ae_sorted != 0;
    if (ctx->ae_log && ae_publish(ctx)) {
        tbg_close(ctx);
        return nullptr;
    }
    ctx->acc_ts_stale = ctx->tr_ts_stale = true;
    return ctx;
}

}  // extern "C"

// ---- Scans (queries.hpp) ---------------------------------------------------------------------------

namespace {

bool scan_ts_valid(uint64_t ts) { return ts >= TB_TIMESTAMP_MIN && ts <= TB_TIMESTAMP_MAX; }

// get_scan_from_account_filter's validity (:1743-1753).
bool account_filter_valid(const tb_account_filter_t* f) {
    bool reserved_zero = true;
    for (int i = 0; i < 58; i++) reserved_zero &= f->reserved[i] == 0;
    const u128 id = U(f->account_id);
    return id != 0 && id != kU128Max && (f->timestamp_min == 0 || scan_ts_valid(f->timestamp_min)) &&
           (f->timestamp_max == 0 || scan_ts_valid(f->timestamp_max)) &&
           (f->timestamp_max == 0 || f->timestamp_min <= f->timestamp_max) && f->limit != 0 &&
           (f->flags & (TB_ACCOUNT_FILTER_DEBITS | TB_ACCOUNT_FILTER_CREDITS)) &&
           !(f->flags & TB_ACCOUNT_FILTER_PADDING_MASK) && reserved_zero;
}

// get_scan_from_query_filter's validity (:2062-2070).
bool query_filter_valid(const tb_query_filter_t* f) {
    bool reserved_zero = true;
    for (int i = 0; i < 6; i++) reserved_zero &= f->reserved[i] == 0;
    return (f->timestamp_min == 0 || scan_ts_valid(f->timestamp_min)) &&
           (f->timestamp_max == 0 || scan_ts_valid(f->timestamp_max)) &&
           (f->timestamp_max == 0 || f->timestamp_min <= f->timestamp_max) && f->limit != 0 &&
           !(f->flags & TB_QUERY_FILTER_PADDING_MASK) && reserved_zero;
}

template <typename F>
ScanFilter scan_filter_common(const F* f) {
    ScanFilter s{};
    s.user_data_128 = U(f->user_data_128);
    s.user_data_64 = f->user_data_64;
    s.user_data_32 = f->user_data_32;
    s.code = f->code;
    s.ts_lo = f->timestamp_min ? f->timestamp_min : TB_TIMESTAMP_MIN;
    s.ts_hi = f->timestamp_max ? f->timestamp_max : TB_TIMESTAMP_MAX;
    return s;
}

// Matches one table's live rows (`launch` fills the match flags), selects them in row order and
// returns their count; the selected rows are ctx->sel_buf[0 .. count).
template <typename Launch>
int64_t scan_select(tbg_ctx* ctx, uint64_t used, Launch launch) {
    if (used == 0) return 0;
    uint8_t* match = nullptr;
    if (!dev_alloc(ctx, &match, used, false)) return TBG_ENOMEM;
    launch(match);
    unsigned int* d_count = &ctx->d_scalars->slow_count;
    int rc = hip_ok(ctx, hipGetLastError(), "scan match") ? 0 : TBG_EHIP;
    if (!rc) rc = select_flagged(ctx, match, used, ctx->sel_buf, d_count);
    unsigned int count = 0;
    if (!rc && !(hip_ok(ctx, hipMemcpyAsync(&count, d_count, 4, hipMemcpyDeviceToHost, ctx->stream),
                        "scan count") &&
                 hip_ok(ctx, hipStreamSynchronize(ctx->stream), "scan sync")))
        rc = TBG_EHIP;
    (void)hipFree(match);
    return rc ? rc : int64_t(count);
}

// The first n (or, reversed, the last n) selected rows of `rows`, copied to the host.
template <typename Row>
int64_t scan_output(tbg_ctx* ctx, const Row* rows, uint32_t count, uint32_t n, bool reversed,
                    Row* out) {
    if (n == 0) return 0;
    Row* d_out = nullptr;
    if (!dev_alloc(ctx, &d_out, n, false)) return TBG_ENOMEM;
    hipLaunchKernelGGL(scan_gather<Row>, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream, rows,
                       ctx->sel_buf, count, n, reversed ? 1 : 0, d_out);
    int64_t rc = n;
    if (!hip_ok(ctx, hipGetLastError(), "scan gather") ||
        !hip_ok(ctx, hipMemcpyAsync(out, d_out, size_t(n) * sizeof(Row), hipMemcpyDeviceToHost,
                                    ctx->stream), "scan copy") ||
        !hip_ok(ctx, hipStreamSynchronize(ctx->stream), "scan sync"))
        rc = TBG_EHIP;
    (void)hipFree(d_out);
    return rc;
}

// The transfers an AccountFilter selects (get_account_transfers / get_account_balances).
int64_t scan_account_transfers(tbg_ctx* ctx, const tb_account_filter_t* filter) {
    ScanFilter f = scan_filter_common(filter);
    f.account_id = U(filter->account_id);
    f.sides = filter->flags & (TB_ACCOUNT_FILTER_DEBITS | TB_ACCOUNT_FILTER_CREDITS);
    const uint64_t used = ctx->T.tr_rows_used;
    return scan_select(ctx, used, [&](uint8_t* match) {
        hipLaunchKernelGGL(scan_match_account_transfers, dim3(grid_for(used)), dim3(kBlock), 0,
                           ctx->stream, ctx->T.tr_rows, ctx->T.tr_live, used, f, match);
    });
}

}  // namespace

extern "C" {

int64_t tbg_get_account_transfers(tbg_ctx* ctx, const tb_account_filter_t* filter,
                                  uint32_t limit_max, tb_transfer_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || !filter) return TBG_EINVAL;
    if (!account_filter_valid(filter)) return 0;
    const int64_t count = scan_account_transfers(ctx, filter);
    if (count <= 0) return count;
    const uint32_t n = std::min<uint64_t>({uint64_t(count), filter->limit, limit_max});
    return scan_output(ctx, ctx->T.tr_rows, uint32_t(count), n,
                       (filter->flags & TB_ACCOUNT_FILTER_REVERSED) != 0, out);
}

int64_t tbg_get_account_balances(tbg_ctx* ctx, const tb_account_filter_t* filter,
                                 uint32_t limit_max, tb_account_balance_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || !filter) return TBG_EINVAL;
    if (!ctx->ae_log) {
        ctx->error = "get_account_balances needs account_events_capacity > 0";
        return TBG_EINVAL;
    }
    // The account must exist and keep history (:1624-1626).
    tb_account_t acc;
    const int64_t found = lookup_impl(ctx, &filter->account_id, 1, &acc, true);
    if (found < 0) return found;
    if (found == 0 || !(acc.flags & TB_ACCOUNT_HISTORY) || !account_filter_valid(filter)) return 0;
    const int64_t count = scan_account_transfers(ctx, filter);
    if (count <= 0) return count;
    const uint32_t n = std::min<uint64_t>({uint64_t(count), filter->limit, limit_max});
    int rc = ae_sort_log(ctx);
    if (rc) return rc;
    tb_account_balance_t* d_out = nullptr;
    unsigned int* d_missing = reinterpret_cast<unsigned int*>(ctx->ae_words);
    if (!dev_alloc(ctx, &d_out, n, false)) return TBG_ENOMEM;
    int64_t result = n;
    unsigned int missing = 0;
    if (!hip_ok(ctx, hipMemsetAsync(d_missing, 0, 4, ctx->stream), "memset")) result = TBG_EHIP;
    if (result >= 0) {
        hipLaunchKernelGGL(scan_balances, dim3(grid_for(n)), dim3(kBlock), 0, ctx->stream,
                           ctx->T.tr_rows, ctx->sel_buf, uint32_t(count), n,
                           (filter->flags & TB_ACCOUNT_FILTER_REVERSED) ? 1 : 0, ctx->ae_log,
                           ctx->ae_used, U(filter->account_id), d_out, d_missing);
        if (!hip_ok(ctx, hipGetLastError(), "scan balances") ||
            !hip_ok(ctx, hipMemcpyAsync(out, d_out, size_t(n) * sizeof(tb_account_balance_t),
                                        hipMemcpyDeviceToHost, ctx->stream), "balances copy") ||
            !hip_ok(ctx, hipMemcpyAsync(&missing, d_missing, 4, hipMemcpyDeviceToHost,
                                        ctx->stream), "missing") ||
            !hip_ok(ctx, hipStreamSynchronize(ctx->stream), "sync"))
            result = TBG_EHIP;
    }
    (void)hipFree(d_out);
    if (result >= 0 && missing) {
        ctx->error = "get_account_balances: a transfer without its AccountEvent";
        result = TBG_EINVAL;
    }
    return result;
}

int64_t tbg_query_accounts(tbg_ctx* ctx, const tb_query_filter_t* filter, uint32_t limit_max,
                           tb_account_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || !filter) return TBG_EINVAL;
    if (!query_filter_valid(filter)) return 0;
    ScanFilter f = scan_filter_common(filter);
    f.ledger = filter->ledger;
    const uint64_t used = ctx->T.acc_rows_used;
    const int64_t count = scan_select(ctx, used, [&](uint8_t* match) {
        hipLaunchKernelGGL(scan_match_query<tb_account_t>, dim3(grid_for(used)), dim3(kBlock), 0,
                           ctx->stream, ctx->T.acc_rows, ctx->T.acc_live, used, f, match);
    });
    if (count <= 0) return count;
    const uint32_t n = std::min<uint64_t>({uint64_t(count), filter->limit, limit_max});
    return scan_output(ctx, ctx->T.acc_rows, uint32_t(count), n,
                       (filter->flags & TB_QUERY_FILTER_REVERSED) != 0, out);
}

int64_t tbg_query_transfers(tbg_ctx* ctx, const tb_query_filter_t* filter, uint32_t limit_max,
                            tb_transfer_t* out) {
    TBG_DEVICE_SCOPE(ctx);
    if (!ctx || !filter) return TBG_EINVAL;
    if (!query_filter_valid(filter)) return 0;
    ScanFilter f = scan_filter_common(filter);
    f.ledger = filter->ledger;
    const uint64_t used = ctx->T.tr_rows_used;
    const int64_t count = scan_select(ctx, used, [&](uint8_t* match) {
        hipLaunchKernelGGL(scan_match_query<tb_transfer_t>, dim3(grid_for(used)), dim3(kBlock), 0,
                           ctx->stream, ctx->T.tr_rows, ctx->T.tr_live, used, f, match);
    });
    if (count <= 0) return count;
    const uint32_t n = std::min<uint64_t>({uint64_t(count), filter->limit, limit_max});
    return scan_output(ctx, ctx->T.tr_rows, uint32_t(count), n,
                       (filter->flags & TB_QUERY_FILTER_REVERSED) != 0, out);
}

}  // extern "C"
