// The ordered replay: execute_create restated for one device thread, over the HBM tables.
//
// The replay executes, in the serial order of the call, every event whose outcome can depend on
// in-call state: linked chains, duplicate ids, post/void, balancing, limits, closing, imported
// batches, overflow-risk amounts, and every event touching an account such events touch. It is a
// statement-for-statement restatement of src/state_machine.zig (execute_create :3002-3213,
// create_account :3613-3703, create_transfer :3719-4051, post_or_void_pending_transfer
// :4053-4382) with the groove operations mapped onto the HBM tables of device_common.hpp.
//
// In-call id visibility (the groove's get() during a batch): the slot of an id holds the ref of
// the earliest in-call event with that id (or a committed row). For a lookup made by event k, an
// in-call holder j is interpreted through results[j], which is final for every j < k (the parallel
// path and static checks ran before the replay; the replay runs in order):
//   j >= k                  -> not found (the holder has not executed yet)
//   results[j] == created   -> found (row row_base + j)
//   results[j] transient    -> orphaned id
//   otherwise               -> not found
// When an event that found its id "not found" creates it (or orphans it), it becomes the holder.
// A chain rollback rewrites results[] of the chain to linked_event_failed, which makes the ids the
// chain created read as "not found" again -- exactly the groove's scope discard.
#pragma once

#include "device_common.hpp"

namespace tbg {

struct DevScalars {
    unsigned long long pulse_next_timestamp;
    unsigned long long accounts_key_max;   // objects tree key_range.key_max (0 = no key_range)
    unsigned long long transfers_key_max;
    unsigned long long expiry_count;       // entries in the expires_at list
    unsigned int flags;                    // per call: kFlag*
    unsigned int slow_count;               // per call: events in the replay list
    unsigned long long stats[4];           // per call: slow, fast, replayed, static
    unsigned long long spec_fast;          // per call: FAST events as ingest classified them
    unsigned long long spec_ts_max;        // per call: their largest timestamp
    unsigned long long fixed;              // per call: tr_commit's fixed failures (Call::fix_slots)
};

enum : unsigned int {
    kFlagImported = 1u << 0,   // some event of the call has the imported flag
    kFlagPostVoid = 1u << 1,   // some event of the call posts or voids
    kFlagUndoOverflow = 1u << 2,
    kFlagTableFull = 1u << 3,
    kFlagDuplicate = 1u << 4,  // two events of the call carry the same id
    kFlagHot = 1u << 5,        // some account is marked hot (a SLOW event touches it)
    kFlagClosable = 1u << 6,   // some account is marked closable
    kFlagNeedCommit = 1u << 7, // some event is not a plain FAST event (tr_commit must run)
    kFlagFlowStalled = 1u << 8, // the flow replay's watchdog fired (a bug: the call fails)
    kFlagChain = 1u << 9,      // some linked chain's event is FAST (tr_commit decides the chain)
    // AccountEvents (events.hpp): the window emit takes calls whose created events are all plain
    // single-phase FAST events with a pair item and whose window sums stay below 2^32.
    kFlagAeSlow = 1u << 10,    // a FAST event the AccountEvents window cannot take
    kFlagWideSums = 1u << 11,  // a window key's sum reached 2^32
    kFlagWideItems = 1u << 12, // a pair item too wide to pack (the balance window's wide layout)
    kFlagFinished = 1u << 13,  // tr_ingest ended the call (Call::finish_done)
    // A replayed (SLOW) event the account lanes cannot take (lanes.hpp: not a plain unlinked
    // transfer): the flow replay runs, so the plan may drop doomed debits' keys (group.hpp).
    kFlagNoLanes = 1u << 14,
    // stage_out's last workgroup cleared the call's scalar words (StageOut::clear): the host
    // launches no tr_reset_scalars. Set in the host's copy only.
    kFlagStageCleared = 1u << 15,
};
// Call flags under which tr_commit re-validates (and may demote) ingest's FAST events.
constexpr unsigned int kCommitFlags = kFlagImported | kFlagPostVoid | kFlagDuplicate | kFlagHot |
                                      kFlagClosable | kFlagNeedCommit | kFlagChain;

enum : uint8_t { kClassDone = 0, kClassFast = 1, kClassSlow = 2 };

struct alignas(16) UndoEntry {
    uint64_t kind_index;  // kind in the top byte
    uint64_t pad;         // (the row 16-B aligned: store_balances writes 16-B words)
    tb_account_t row;     // kUndoAccount: the row's balances and flags before the update (the
                          // only fields a create_transfers replay changes)
};
constexpr uint64_t kUndoAccount = 1ull << 56;
constexpr uint64_t kUndoStatus = 2ull << 56;
constexpr uint64_t kUndoDelta = 3ull << 56;   // balance deltas added atomically (row's 4 fields)
constexpr uint64_t kUndoIndexMask = (1ull << 56) - 1;

// The four balances (16-B stores) and the flags of `src` into the row at `dst`.
__device__ inline void store_balances(tb_account_t* dst, const tb_account_t& src) {
    auto q = [](const tb_uint128_t& v) {
        return make_uint4(uint32_t(v.lo), uint32_t(v.lo >> 32), uint32_t(v.hi), uint32_t(v.hi >> 32));
    };
    *reinterpret_cast<uint4*>(&dst->debits_pending) = q(src.debits_pending);
    *reinterpret_cast<uint4*>(&dst->debits_posted) = q(src.debits_posted);
    *reinterpret_cast<uint4*>(&dst->credits_pending) = q(src.credits_pending);
    *reinterpret_cast<uint4*>(&dst->credits_posted) = q(src.credits_posted);
    dst->flags = src.flags;
}

// Everything a kernel needs, passed by value.
struct Tables {
    IdTable acc;             // id -> row claims of create_accounts (in-call visibility)
    AccIndex acc_index;      // id -> {row, ledger, flags, hazard} of committed accounts
    uint32_t* acc_entry_of;  // row -> its acc_index entry (0xFFFFFFFF until indexed)
    tb_account_t* acc_rows;
    uint8_t* acc_live;
    uint32_t* acc_hot;       // epoch of the last call that routed an event of this account to replay
    uint32_t* acc_closable;  // epoch of the last call whose events may change `closed` here
    uint64_t acc_rows_used;

    IdTable tr;
    tb_transfer_t* tr_rows;
    uint8_t* tr_live;
    uint8_t* tr_status;  // TransferPending.status per row (src/tigerbeetle.zig:118-130)
    uint64_t tr_rows_used;

    uint64_t* expiry;  // rows of pending transfers with timeout > 0 (the expires_at index)
    uint64_t expiry_capacity;

    const uint64_t* acc_ts_index;  // sorted timestamps of live accounts (imported checks)
    uint64_t acc_ts_count;
    const uint64_t* tr_ts_index;   // sorted timestamps of live transfers
    uint64_t tr_ts_count;

    DevScalars* scalars;
    UndoEntry* undo;
    uint64_t undo_capacity;
};

template <typename Event>
struct Call {
    const Event* events;
    uint32_t n;
    const uint32_t* batch_ends;
    const uint64_t* batch_ts;
    uint32_t n_batches;
    tb_create_result_t* results;
    uint64_t row_base;
    uint32_t epoch;
    uint32_t force_replay;
    // The whole call is one linked chain closed at its last event, whatever the events' linked
    // flags (tbg_create_*_stamped with TBG_ONE_CHAIN: a shard's part of a chain across shards).
    uint32_t one_chain;
    // per-event scratch (structure of arrays; kNone32 = absent)
    uint32_t* ev_slot;     // slot of the event's id in the id table
    uint32_t* ev_dr;       // account rows (create_transfers)
    uint32_t* ev_cr;
    uint64_t* ev_amount;   // amount low word of parallel-path candidates
    uint64_t* ev_prow;     // FAST post/void: its pending transfer's row (classify_post_void)
    uint8_t* ev_info;      // kInfo* bits
    uint8_t* ev_slow;      // 1 = executes in the ordered replay
    const uint32_t* slow_list;
    // Balance items of FAST events (create_transfers, sorted calls): item 2k / 2k+1 = the debit /
    // credit delta of event k, packed as (amount << key_bits) | account field key; ~0 = none.
    uint64_t* bal_items;
    uint32_t key_bits;
    // Pair items (the balance window path, key spaces of <= 2^14 accounts): pair_shift = s > 0,
    // one item per event, (amount << 2s + 1) | (pending << 2s) | (cr << s) | dr; ~0 = none.
    uint32_t pair_shift;
    // Calls whose ingest applies the FAST deltas itself (no balance items, sparse key spaces):
    // FAST events write no record either (kInfoLean); tr_commit looks their accounts up again.
    uint32_t lean_lookup;
    // Bucketed balance path (small key spaces): per-bucket item counts, bucket = key >> 13.
    unsigned int* bucket_counts;
    uint32_t n_buckets;
    // create_transfers: per 64-event chunk, its batch bounds (tr_chunk_info).
    const uint4* chunk_info;
    // Per-event timestamps (a ledger shard's slice of a routed call: its events keep their global
    // timestamps, which are not contiguous); nullptr: batch_ts[b] - batch_ends[b] + k + 1.
    const uint64_t* event_ts;
    // Calls with post/void: every pulse_next_timestamp update, per event (0: none; expires_at:
    // min; expires_at | kPntReset: reset-if-equal), resolved in call order after the replay.
    uint64_t* pnt_call;
    // Sharded calls (tbg_set_pnt_sharded): every update is recorded, whatever the call's flags,
    // and the resets are resolved across shards by the caller (pnt_resolve applies the mins).
    uint32_t pnt_force;
    // tr_ingest of a small host-buffer call reads the body straight from mapped host memory
    // (`events`) and leaves a copy here for the call's later kernels (null: no copy).
    tb_transfer_t* events_out;
    // ... and, with no stage_in launch, its batch bounds too (`batch_ends` / `batch_ts` then the
    // mapped pinned staging; workgroup 0 copies them here; null: no copy).
    uint32_t* ends_out;
    uint64_t* ts_out;
    // tr_commit's fixed failures (later_claim_status): the id slots they release, tombstoned by
    // the next kernel (stage_out) -- tr_commit's threads read other events' slots.
    uint32_t* fix_slots;
    unsigned long long* chain_planes;  // tr_chain_planes's words (null: tr_commit walks chains itself)
    // create_transfers: per-call claims of pending ids by post/void events (epoch:32 | event + 1;
    // words of other epochs are free): the earliest post/void of a pending transfer in the call.
    unsigned long long* pv_slots;
    uint64_t pv_mask;
    // Small device-buffer calls without balance items: the last tr_ingest workgroup to finish
    // ends a call that raised no commit flag (every event FAST, its effects all written) -- the
    // call's counters, the scalars block to its mapped copy, the call's scalar words cleared, the
    // sequence word for a spinning host -- and finish_done[1] = epoch tells the queued tr_commit
    // and stage_out to return at once. finish_done = null: no such ending.
    unsigned int* finish_done;       // ingest's finished workgroups (zero between calls), epoch
    unsigned long long* finish_scalars;  // mapped pinned copy of the scalars block
    unsigned int* finish_seq;        // the pinned sequence word, or null (the host synchronises)
    unsigned int seq;
    // The host launches tr_commit and stage_out only when the call needs them: the last ingest
    // workgroup publishes the sequence word either way, with the scalars block (kFlagFinished
    // set when it ended the call). 0: they are queued behind tr_ingest and it publishes only an end.
    uint32_t finish_always;
    // Large calls the host expects to replay (tbg_ctx::replay_hint): tr_commit's last workgroup
    // copies the scalars block (the replay count is final there) to its mapped copy and publishes
    // commit_seq_val, so that the host launches the replay while the balance kernels and stage_out
    // still run. commit_done = null: no such signal.
    unsigned int* commit_done;           // tr_commit's finished workgroups (zero between calls)
    unsigned long long* commit_scalars;  // mapped pinned copy of the scalars block
    unsigned int* commit_seq;            // the pinned sequence word
    unsigned int commit_seq_val;
};

constexpr uint32_t kNone32 = 0xFFFFFFFFu;

// ev_info bits written by the ingest pass and consumed by the commit pass.
enum : uint8_t {
    kInfoClassMask = 3,        // kClassDone / kClassFast / kClassSlow
    kInfoPostLookup = 1 << 2,  // status decided after the id lookup: valid only for the holder
    kInfoClosedDep = 1 << 3,   // status depends on `closed` of an account
    kInfoPending = 1 << 4,     // flags.pending
    kInfoTimeout = 1 << 5,     // timeout > 0
    kInfoClaimed = 1 << 6,     // the event claimed / found its id slot
    kInfoLean = 1 << 7,        // FAST without a record: ev_slot / ev_dr / ev_cr / ev_amount
                               // were not written (the packed balance items hold rows and
                               // amount, or, Call::lean_lookup, tr_commit looks them up)
};

template <typename C>
__device__ inline uint64_t slot_of(const C& c, uint32_t k) {
    const uint32_t s = c.ev_slot[k];
    return s == kNone32 ? kNone : uint64_t(s);
}

// An event's per-call records the replay reads: its id slot and account rows (kNone32 = none).
// An event's id slot and account rows, found before the replay. For a post/void the flow plan
// also resolves the pending transfer: `pslot` its id's slot (kNone32: not found) and dr / cr its
// accounts' rows (kNone32: look them up); kPvNoHint: nothing resolved (the replay looks up all).
// `add`: the flow plan's additive verdicts (Replay::additive) of dr (kAddDr) and cr (kAddCr),
// valid with kAddKnown.
constexpr uint32_t kPvNoHint = 0xFFFFFFFEu;
constexpr uint32_t kAddDr = 1, kAddCr = 2, kAddKnown = 4;
struct EvRefs {
    uint32_t slot, dr, cr;
    uint32_t pslot = kPvNoHint;
    uint32_t add = 0;
};
template <typename C>
__device__ inline EvRefs ev_refs(const C& c, uint32_t k) {
    return EvRefs{c.ev_slot[k], c.ev_dr ? c.ev_dr[k] : kNone32, c.ev_cr ? c.ev_cr[k] : kNone32,
                  kPvNoHint, 0};
}
// Batch facts of a replayed event (execute_multi_batch / execute_create): its timestamp, its batch,
// whether it is the batch's last event (a linked flag there is linked_event_chain_open) and
// whether its batch is imported.
struct StepInfo {
    uint64_t ts_event;
    uint32_t batch;
    uint32_t flags;
    static constexpr uint32_t kLastOfBatch = 1, kBatchImported = 2;
};

__device__ inline uint64_t slot_or_none(uint32_t s) { return s == kNone32 ? kNone : uint64_t(s); }

__device__ inline uint32_t batch_of(const uint32_t* ends, uint32_t n_batches, uint32_t k) {
    uint32_t lo = 0, hi = n_batches;  // first b with ends[b] > k
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (ends[mid] > k) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// batch_of with a guess: batches of (near-)uniform length resolve in one or two loads instead of
// a dependent binary search; otherwise fall back to the search.
__device__ inline uint32_t batch_of_guess(const uint32_t* ends, uint32_t n_batches, uint32_t n,
                                          uint32_t k) {
    const uint32_t avg = n_batches ? (n / n_batches > 0 ? n / n_batches : 1) : 1;
    uint32_t b = k / avg;
    if (b >= n_batches) b = n_batches - 1;
    for (int step = 0; step < 4; step++) {
        const bool above = ends[b] <= k;                 // k lies in a later batch
        const bool below = b > 0 && ends[b - 1] > k;     // k lies in an earlier batch
        if (!above && !below) return b;
        b = above ? b + 1 : b - 1;
        if (b >= n_batches) break;
    }
    return batch_of(ends, n_batches, k);
}

__device__ inline bool ts_index_contains(const uint64_t* idx, uint64_t n, uint64_t ts) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if (idx[mid] < ts) lo = mid + 1;
        else hi = mid;
    }
    return lo < n && idx[lo] == ts;
}

// ---- account lookup (accounts do not change during a create_transfers call) ----------------

__device__ inline uint64_t account_find(const Tables& T, const tb_uint128_t& id) {
    AccEntry e;
    if (acc_index_find(T.acc_index, T.acc_rows, id, &e) == kNone) return kNone;
    return e.ref - 1;
}

// An additive account of the call with this epoch (0: none; Replay::additive). Accounts with a
// limit flag are never additive: the account lanes' plan (lanes.hpp) lists their events by key.
__device__ inline bool acc_additive(const Tables& T, uint64_t row, uint32_t epoch) {
    return epoch != 0 && T.acc_hot[row] != epoch && T.acc_closable[row] != epoch &&
           !(T.acc_rows[row].flags & (TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS |
                                      TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS));
}

// ---- the replay state -------------------------------------------------------------------------

struct Scope {
    bool open = false;
    uint64_t undo_len = 0;
    unsigned long long accounts_key_max = 0, transfers_key_max = 0, expiry_count = 0;
};

// The replay state of one executing lane. Serial mode (replay_kernel: one lane, every replayed
// event of the call in order) keeps the reference's scope semantics on the shared scalars. Flow
// mode (flow_replay: many lanes, each executing whole units -- one event or one linked chain --
// that own every key they touch, see flow.hpp) touches no shared scalar a concurrent unit could
// also write: the undo log is the lane's own, the transfers key_max is folded in with atomicMax
// when the unit's effects persist, pulse_next_timestamp updates are recorded per replay position
// (resolved in order after the replay) or, in calls without post/void where only `min` updates
// exist, applied with atomicMin, and expires_at entries are appended atomically (entries of a
// discarded chain stay in the list and are dropped at the next pulse: their rows are not live).
constexpr uint64_t kPntReset = 1ull << 63;  // pnt_ops: a reset-if-equal (post/void of an expiry)

struct Replay {
    const Tables& T;
    Scope scope;
    uint64_t undo_len = 0;
    bool overflow = false;
    UndoEntry* undo;
    uint64_t undo_cap;
    // flow mode
    bool concurrent = false;
    uint64_t* pnt_ops = nullptr;  // calls with post/void: Call::pnt_call (per event)
    uint32_t pos = 0;             // the executing event (its index in the call)
    uint64_t key_max = 0, key_max_scope = 0;
    uint32_t add_epoch = 0;       // nonzero: additive accounts of this call (additive())
    bool expiry_planned = false;  // the flow plan wrote this call's expires_at entries

    __device__ explicit Replay(const Tables& t) : T(t), undo(t.undo), undo_cap(t.undo_capacity) {}

    __device__ void scope_open() {
        scope.open = true;
        scope.undo_len = undo_len;
        if (concurrent) {
            key_max_scope = 0;
            return;
        }
        scope.accounts_key_max = T.scalars->accounts_key_max;
        scope.transfers_key_max = T.scalars->transfers_key_max;
        scope.expiry_count = T.scalars->expiry_count;
    }
    __device__ void scope_close(bool discard) {
        if (discard) {
            for (uint64_t i = undo_len; i-- > scope.undo_len;) {
                const UndoEntry& u = undo[i];
                uint64_t idx = u.kind_index & kUndoIndexMask;
                const uint64_t kind = u.kind_index & ~kUndoIndexMask;
                if (kind == kUndoAccount) {
                    store_balances(&T.acc_rows[idx], u.row);
                } else if (kind == kUndoDelta) {
                    tb_account_t& a = T.acc_rows[idx];
                    if (!u128_is_zero(u.row.debits_pending))
                        atomic_add_u128(&a.debits_pending, u128(0) - U(u.row.debits_pending));
                    if (!u128_is_zero(u.row.debits_posted))
                        atomic_add_u128(&a.debits_posted, u128(0) - U(u.row.debits_posted));
                    if (!u128_is_zero(u.row.credits_pending))
                        atomic_add_u128(&a.credits_pending, u128(0) - U(u.row.credits_pending));
                    if (!u128_is_zero(u.row.credits_posted))
                        atomic_add_u128(&a.credits_posted, u128(0) - U(u.row.credits_posted));
                } else {
                    T.tr_status[idx] = (uint8_t)u.row.timestamp;
                }
            }
            if (!concurrent) {
                T.scalars->accounts_key_max = scope.accounts_key_max;
                T.scalars->transfers_key_max = scope.transfers_key_max;
                T.scalars->expiry_count = scope.expiry_count;
            }
        } else if (concurrent && key_max_scope > key_max) {
            key_max = key_max_scope;
        }
        key_max_scope = 0;
        undo_len = scope.undo_len;
        scope.open = false;
    }
    // (`old`: the status as the event read it -- a load here, behind the event's stores, waited
    // for all of them in issue order)
    __device__ void log_status(uint64_t row, uint8_t old) {
        if (!scope.open) return;
        if (undo_len >= undo_cap) {
            overflow = true;
            return;
        }
        undo[undo_len].kind_index = kUndoStatus | row;
        undo[undo_len].row.timestamp = old;
        undo_len++;
    }
    // (`old`: the row as this event read it, logged from registers). Only the balances and flags
    // are written: nothing else of an account changes in a create_transfers call, and whole-row
    // struct copies of register rows would go through scratch memory.
    __device__ void update_account(uint64_t row, const tb_account_t& old, const tb_account_t& next) {
        if (scope.open) {
            if (undo_len >= undo_cap) {
                overflow = true;
            } else {
                undo[undo_len].kind_index = kUndoAccount | row;
                store_balances(&undo[undo_len].row, old);
                undo_len++;
            }
        }
        store_balances(&T.acc_rows[row], next);
        // A rollback restores the row but keeps the hazard bits: they only over-approximate.
        const uint16_t h = acc_hazard_of(next);
        if (h) acc_hazard_set(T.acc_index, T.acc_entry_of, row, h);
    }
    // Additive accounts (flow mode, add_epoch != 0): accounts no replayed event of the call reads
    // a balance of (no acc_hot mark: no limit flag on a checked side, no balancing, no possible
    // overflow; and no limit flag at all) and whose `closed` flag no event of the call changes (no
    // acc_closable mark). A
    // replayed event's outcome does not depend on their balances, and its effect on them is a sum,
    // so the flow plan gives them no account key (flow_keys) and the replay adds its deltas with
    // u128 atomics, logged as deltas for a chain's rollback.
    __device__ bool additive(uint64_t row) const { return acc_additive(T, row, add_epoch); }
    __device__ bool additive(uint64_t row, const EvRefs& x, uint32_t bit) const {
        return (x.add & kAddKnown) ? (x.add & bit) != 0 : additive(row);
    }
    // Adds the four (modular) deltas d[0..3] to debits_pending, debits_posted, credits_pending,
    // credits_posted of row a (da) and of row b (db); kNone32 skips a row. Every low-word atomic
    // goes out before any returns (one round trip to the point of coherence, not one per field),
    // then the carries.
    // Adds pending delta P and posted delta Q to row a's debits and row b's credits (modular;
    // kNone32 skips a row): every call's deltas have this shape. The low-word atomics go out
    // together. Flow mode defers their returns: the carries into the high words (and the hazard
    // marks) are applied by flush_adds -- called after the next event's loads are issued, and at
    // the unit's end -- so that the atomics' round trip overlaps the next event's loads instead
    // of adding one to every event (a returned value is waited for in issue order, behind every
    // store the event made before it). No replayed event reads these balances, and the adds
    // commute (a chain's rollback subtracts whole deltas).
    // (scalar members, no array: an array member kept the whole Replay in scratch)
    uint64_t add_o0 = 0, add_o1 = 0, add_o2 = 0, add_o3 = 0;  // a.dpe, a.dpo, b.cpe, b.cpo
    uint64_t add_p_lo = 0, add_p_hi = 0, add_q_lo = 0, add_q_hi = 0;  // (no u128 members either)
    uint32_t add_a = kNone32, add_b = kNone32;
    bool add_pending = false;
    // The carry of one field's deferred add into its high word: returns the new high word (0: none).
    __device__ __attribute__((always_inline)) uint64_t add_carry(tb_uint128_t* f, uint64_t lo, uint64_t dhi, uint64_t old) {
        const uint64_t hi = dhi + ((lo != 0 && old + lo < old) ? 1 : 0);
        return hi ? atomicAdd((unsigned long long*)&f->hi, (unsigned long long)hi) + hi : 0;
    }
    __device__ __attribute__((always_inline)) void flush_adds() {
        if (!add_pending) return;
        add_pending = false;
        if (add_a != kNone32) {
            tb_account_t& r = T.acc_rows[add_a];
            const uint64_t h = add_carry(&r.debits_pending, add_p_lo, add_p_hi, add_o0) |
                               add_carry(&r.debits_posted, add_q_lo, add_q_hi, add_o1);
            if (h >= kHazardHiLimit) acc_hazard_set(T.acc_index, T.acc_entry_of, add_a, kHazardHigh);
        }
        if (add_b != kNone32) {
            tb_account_t& r = T.acc_rows[add_b];
            const uint64_t h = add_carry(&r.credits_pending, add_p_lo, add_p_hi, add_o2) |
                               add_carry(&r.credits_posted, add_q_lo, add_q_hi, add_o3);
            if (h >= kHazardHiLimit) acc_hazard_set(T.acc_index, T.acc_entry_of, add_b, kHazardHigh);
        }
    }
    __device__ __attribute__((always_inline)) void add_pq(uint32_t a, uint32_t b, u128 P, u128 Q) {
        flush_adds();
        auto add_lo = [&](uint32_t row, tb_uint128_t* f, u128 d) -> uint64_t {
            return row != kNone32 && uint64_t(d) != 0
                       ? atomicAdd((unsigned long long*)&f->lo, (unsigned long long)uint64_t(d))
                       : 0ull;
        };
        tb_account_t* A = T.acc_rows;
        add_o0 = add_lo(a, &A[a].debits_pending, P);
        add_o1 = add_lo(a, &A[a].debits_posted, Q);
        add_o2 = add_lo(b, &A[b].credits_pending, P);
        add_o3 = add_lo(b, &A[b].credits_posted, Q);
        add_a = a;
        add_b = b;
        add_p_lo = uint64_t(P);
        add_p_hi = uint64_t(P >> 64);
        add_q_lo = uint64_t(Q);
        add_q_hi = uint64_t(Q >> 64);
        add_pending = true;
        if (!concurrent) flush_adds();
        if (!scope.open) return;
        if (undo_len + (a != kNone32) + (b != kNone32) > undo_cap) {
            overflow = true;
            return;
        }
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const uint32_t row = r == 0 ? a : b;
            if (row == kNone32) continue;
            UndoEntry& u = undo[undo_len++];
            u.kind_index = kUndoDelta | row;
            u.row.debits_pending = W(r == 0 ? P : u128(0));
            u.row.debits_posted = W(r == 0 ? Q : u128(0));
            u.row.credits_pending = W(r == 0 ? u128(0) : P);
            u.row.credits_posted = W(r == 0 ? u128(0) : Q);
        }
    }
    __device__ void update_status(uint64_t row, uint8_t status, uint8_t old) {
        log_status(row, old);
        T.tr_status[row] = status;
    }
    // The transfers objects tree key_range.key_max (groove.zig:1780) after an insert at `ts`.
    __device__ void note_transfer_ts(uint64_t ts) {
        if (!concurrent) {
            if (ts > T.scalars->transfers_key_max) T.scalars->transfers_key_max = ts;
        } else if (scope.open) {
            if (ts > key_max_scope) key_max_scope = ts;
        } else if (ts > key_max) {
            key_max = ts;
        }
    }
    // create_transfer :3975-3982: pulse_next_timestamp = min(pulse_next_timestamp, expires_at).
    // In calls with post/void every update is recorded at its event (FAST pending transfers with
    // a timeout record theirs in tr_commit) and resolved in call order afterwards (pnt_resolve);
    // otherwise only `min` updates exist, which commute.
    __device__ void pulse_min(uint64_t expires_at) {
        if (pnt_ops) {
            pnt_ops[pos] = expires_at;
        } else if (!concurrent) {
            if (expires_at < T.scalars->pulse_next_timestamp)
                T.scalars->pulse_next_timestamp = expires_at;
        } else {
            atomicMin(&T.scalars->pulse_next_timestamp, (unsigned long long)expires_at);
        }
    }
    // post_or_void_pending_transfer :4227-4229: reset to timestamp_min if it names this expiry.
    __device__ void pulse_reset(uint64_t expires_at) { pnt_ops[pos] = expires_at | kPntReset; }
};

// ---- transfers --------------------------------------------------------------------------------

// groove.get for transfers as seen by in-call event k: 0 not found, 1 object (row), 2 orphaned.
template <typename C>
__device__ inline int replay_transfer_at_word(const C& c, uint64_t w, uint32_t k, uint64_t* row);
template <typename C>
__device__ inline int replay_get_transfer_at_slot(const Tables& T, const C& c, uint64_t s,
                                                  uint32_t k, uint64_t* row) {
    if (s == kNone) return 0;
    return replay_transfer_at_word(c, T.tr.slots[s], k, row);
}
// The same from the slot's word (kEmpty: no slot).
template <typename C>
__device__ inline int replay_transfer_at_word(const C& c, uint64_t w, uint32_t k, uint64_t* row) {
    if (w == kEmpty || w == kTomb) return 0;
    uint64_t r = (w & kRefMask) - 1;
    if (r < c.row_base) {
        if (w & kOrphanBit) return 2;
        *row = r;
        return 1;
    }
    uint64_t j = r - c.row_base;
    if (j >= k) return 0;
    uint32_t st = c.results[j].status;
    if (st == TB_STATUS_CREATED) {
        *row = r;
        return 1;
    }
    if (tb_transfer_status_transient(st)) return 2;
    return 0;
}

template <typename C>
__device__ inline uint64_t transfer_slot_find(const Tables& T, const C& c,
                                              const tb_uint128_t& id) {
    const tb_transfer_t* rows = T.tr_rows;
    const tb_transfer_t* events = c.events;
    uint64_t base = c.row_base;
    return probe_find(T.tr, id, [=](uint64_t r) {
        return r >= base ? events[r - base].id : rows[r].id;
    });
}

__device__ inline uint32_t post_or_void_pending_transfer_exists(const tb_transfer_t& t,
                                                               const tb_transfer_t& e,
                                                               const tb_transfer_t& p,
                                                               uint64_t* ts) {
    if (U(t.debit_account_id) != 0 && U(t.debit_account_id) != U(e.debit_account_id))
        return TB_CT_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (U(t.credit_account_id) != 0 && U(t.credit_account_id) != U(e.credit_account_id))
        return TB_CT_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (t.flags & TB_TRANSFER_VOID_PENDING) {
        if (U(t.amount) == 0) {
            if (U(e.amount) != U(p.amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
        } else if (U(t.amount) != U(e.amount)) {
            return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
        }
    }
    if (t.flags & TB_TRANSFER_POST_PENDING) {
        if (U(t.amount) == kU128Max) {
            if (U(e.amount) != U(p.amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
        } else if (U(t.amount) != U(e.amount)) {
            return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
        }
    }
    if (U(t.user_data_128) == 0) {
        if (U(e.user_data_128) != U(p.user_data_128))
            return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    } else if (U(t.user_data_128) != U(e.user_data_128)) {
        return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    }
    if (t.user_data_64 == 0) {
        if (e.user_data_64 != p.user_data_64) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    } else if (t.user_data_64 != e.user_data_64) {
        return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    }
    if (t.user_data_32 == 0) {
        if (e.user_data_32 != p.user_data_32) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    } else if (t.user_data_32 != e.user_data_32) {
        return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    }
    if (t.ledger != 0 && t.ledger != e.ledger) return TB_CT_EXISTS_WITH_DIFFERENT_LEDGER;
    if (t.code != 0 && t.code != e.code) return TB_CT_EXISTS_WITH_DIFFERENT_CODE;
    *ts = e.timestamp;
    return TB_CT_EXISTS;
}

// create_transfer_exists (:3988-4051) given the pending transfer p (post/void only).
__device__ inline uint32_t create_transfer_exists(const tb_transfer_t& t, const tb_transfer_t& e,
                                                  const tb_transfer_t* p, uint64_t* ts) {
    if (t.flags != e.flags) return TB_CT_EXISTS_WITH_DIFFERENT_FLAGS;
    if (U(t.pending_id) != U(e.pending_id)) return TB_CT_EXISTS_WITH_DIFFERENT_PENDING_ID;
    if (t.timeout != e.timeout) return TB_CT_EXISTS_WITH_DIFFERENT_TIMEOUT;
    if (t.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING))
        return post_or_void_pending_transfer_exists(t, e, *p, ts);
    if (U(t.debit_account_id) != U(e.debit_account_id))
        return TB_CT_EXISTS_WITH_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (U(t.credit_account_id) != U(e.credit_account_id))
        return TB_CT_EXISTS_WITH_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (t.flags & (TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT)) {
        if (U(t.amount) < U(e.amount)) return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    } else if (U(t.amount) != U(e.amount)) {
        return TB_CT_EXISTS_WITH_DIFFERENT_AMOUNT;
    }
    if (U(t.user_data_128) != U(e.user_data_128)) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (t.user_data_64 != e.user_data_64) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (t.user_data_32 != e.user_data_32) return TB_CT_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (t.ledger != e.ledger) return TB_CT_EXISTS_WITH_DIFFERENT_LEDGER;
    if (t.code != e.code) return TB_CT_EXISTS_WITH_DIFFERENT_CODE;
    *ts = e.timestamp;
    return TB_CT_EXISTS;
}

__device__ inline void expiry_append(const Tables& T, uint64_t row, bool serial) {
    unsigned long long i = serial ? T.scalars->expiry_count++
                                  : atomicAdd(&T.scalars->expiry_count, 1ull);
    if (i < T.expiry_capacity) T.expiry[i] = row;
    else atomicOr(&T.scalars->flags, kFlagTableFull);
}

template <typename C>
__device__ uint32_t replay_post_or_void(Replay& R, const C& c, uint32_t k, uint64_t ts_event,
                                        const tb_transfer_t& t, const EvRefs& x,
                                        uint64_t* ts_out) {
    const Tables& T = R.T;
    const uint16_t f = t.flags;
    if ((f & TB_TRANSFER_POST_PENDING) && (f & TB_TRANSFER_VOID_PENDING))
        return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (f & (TB_TRANSFER_PENDING | TB_TRANSFER_BALANCING_DEBIT | TB_TRANSFER_BALANCING_CREDIT |
             TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT))
        return TB_CT_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (u128_is_zero(t.pending_id)) return TB_CT_PENDING_ID_MUST_NOT_BE_ZERO;
    if (u128_is_max(t.pending_id)) return TB_CT_PENDING_ID_MUST_NOT_BE_INT_MAX;
    if (u128_eq(t.pending_id, t.id)) return TB_CT_PENDING_ID_MUST_BE_DIFFERENT;
    if (t.timeout != 0) return TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;

    // With the plan's resolution the account rows load alongside the pending id's slot instead
    // of after the pending row (the same rows: the pending transfer's accounts never change).
    const bool hinted = x.pslot != kPvNoHint && x.dr != kNone32 && x.cr != kNone32;
    tb_account_t dr, cr;
    if (hinted) {
        dr = T.acc_rows[x.dr];
        cr = T.acc_rows[x.cr];
    }
    const uint64_t ps = x.pslot != kPvNoHint ? slot_or_none(x.pslot)
                                             : transfer_slot_find(T, c, t.pending_id);
    uint64_t p_row = 0;
    if (replay_get_transfer_at_slot(T, c, ps, k, &p_row) != 1)
        return TB_CT_PENDING_TRANSFER_NOT_FOUND;
    const tb_transfer_t p = T.tr_rows[p_row];
    if (!(p.flags & TB_TRANSFER_PENDING)) return TB_CT_PENDING_TRANSFER_NOT_PENDING;

    uint64_t dr_row = x.dr, cr_row = x.cr;
    if (!hinted) {
        dr_row = account_find(T, p.debit_account_id);
        cr_row = account_find(T, p.credit_account_id);
        if (dr_row == kNone || cr_row == kNone) return TB_CT_PENDING_TRANSFER_NOT_FOUND;  // unreachable
        dr = T.acc_rows[dr_row];
        cr = T.acc_rows[cr_row];
    }

    if (!u128_is_zero(t.debit_account_id) && !u128_eq(t.debit_account_id, p.debit_account_id))
        return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_DEBIT_ACCOUNT_ID;
    if (!u128_is_zero(t.credit_account_id) && !u128_eq(t.credit_account_id, p.credit_account_id))
        return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CREDIT_ACCOUNT_ID;
    if (t.ledger > 0 && t.ledger != p.ledger) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_LEDGER;
    if (t.code > 0 && t.code != p.code) return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_CODE;

    u128 p_amount = U(p.amount);
    u128 amount = (f & TB_TRANSFER_VOID_PENDING)
                      ? (U(t.amount) == 0 ? p_amount : U(t.amount))
                      : (U(t.amount) == kU128Max ? p_amount : U(t.amount));
    if (amount > p_amount) return TB_CT_EXCEEDS_PENDING_TRANSFER_AMOUNT;
    if ((f & TB_TRANSFER_VOID_PENDING) && amount < p_amount)
        return TB_CT_PENDING_TRANSFER_HAS_DIFFERENT_AMOUNT;

    const uint8_t p_status = T.tr_status[p_row];
    switch (p_status) {
        case TB_PENDING_PENDING: break;
        case TB_PENDING_POSTED: return TB_CT_PENDING_TRANSFER_ALREADY_POSTED;
        case TB_PENDING_VOIDED: return TB_CT_PENDING_TRANSFER_ALREADY_VOIDED;
        default: return TB_CT_PENDING_TRANSFER_EXPIRED;
    }
    const bool has_expiry = p.timeout != 0;
    uint64_t expires_at = 0;
    if (has_expiry) {
        expires_at = p.timestamp + (uint64_t)p.timeout * TB_NS_PER_S;
        if (expires_at <= ts_event) return TB_CT_PENDING_TRANSFER_EXPIRED;
    }
    uint64_t ts_actual = ts_event;
    if (f & TB_TRANSFER_IMPORTED) {
        if (t.timestamp <= T.scalars->transfers_key_max)
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        if (ts_index_contains(T.acc_ts_index, T.acc_ts_count, t.timestamp))
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        ts_actual = t.timestamp;
    }
    if ((dr.flags & TB_ACCOUNT_CLOSED) && !(f & TB_TRANSFER_VOID_PENDING))
        return TB_CT_DEBIT_ACCOUNT_ALREADY_CLOSED;
    if ((cr.flags & TB_ACCOUNT_CLOSED) && !(f & TB_TRANSFER_VOID_PENDING))
        return TB_CT_CREDIT_ACCOUNT_ALREADY_CLOSED;

    // Insert the posting/voiding transfer at this event's row.
    const uint64_t row = c.row_base + k;
    tb_transfer_t o;
    o.id = t.id;
    o.debit_account_id = p.debit_account_id;
    o.credit_account_id = p.credit_account_id;
    o.amount = W(amount);
    o.pending_id = t.pending_id;
    o.user_data_128 = W(U(t.user_data_128) > 0 ? U(t.user_data_128) : U(p.user_data_128));  // (scalar select: a struct select keeps both rows in scratch)
    o.user_data_64 = t.user_data_64 > 0 ? t.user_data_64 : p.user_data_64;
    o.user_data_32 = t.user_data_32 > 0 ? t.user_data_32 : p.user_data_32;
    o.timeout = 0;
    o.ledger = p.ledger;
    o.code = p.code;
    o.flags = t.flags;
    o.timestamp = ts_actual;
    T.tr_rows[row] = o;
    T.tr_status[row] = TB_PENDING_NONE;
    R.note_transfer_ts(ts_actual);

    if (has_expiry) R.pulse_reset(expires_at);
    R.update_status(p_row, (f & TB_TRANSFER_POST_PENDING) ? TB_PENDING_POSTED : TB_PENDING_VOIDED,
                    p_status);

    tb_account_t dr_new = dr, cr_new = cr;
    dr_new.debits_pending = W(U(dr.debits_pending) - p_amount);
    cr_new.credits_pending = W(U(cr.credits_pending) - p_amount);
    if (f & TB_TRANSFER_POST_PENDING) {
        dr_new.debits_posted = W(U(dr.debits_posted) + amount);
        cr_new.credits_posted = W(U(cr.credits_posted) + amount);
    }
    if (f & TB_TRANSFER_VOID_PENDING) {
        if (p.flags & TB_TRANSFER_CLOSING_DEBIT) dr_new.flags &= (uint16_t)~TB_ACCOUNT_CLOSED;
        if (p.flags & TB_TRANSFER_CLOSING_CREDIT) cr_new.flags &= (uint16_t)~TB_ACCOUNT_CLOSED;
    }
    const u128 posted = (f & TB_TRANSFER_POST_PENDING) ? amount : u128(0);
    const EvRefs xa{x.slot, x.dr, x.cr, x.pslot, hinted ? x.add : 0u};
    // (additive rows: flags unchanged -- a void of a closing transfer marks closable)
    const bool add_dr = R.additive(dr_row, xa, kAddDr), add_cr = R.additive(cr_row, xa, kAddCr);
    if (add_dr || add_cr)
        R.add_pq(add_dr ? uint32_t(dr_row) : kNone32, add_cr ? uint32_t(cr_row) : kNone32,
                 u128(0) - p_amount, posted);
    if (!add_dr && (amount > 0 || p_amount > 0 || dr_new.flags != dr.flags))
        R.update_account(dr_row, dr, dr_new);
    if (!add_cr && (amount > 0 || p_amount > 0 || cr_new.flags != cr.flags))
        R.update_account(cr_row, cr, cr_new);
    *ts_out = ts_actual;
    return TB_STATUS_CREATED;
}

template <typename C>
__device__ uint32_t replay_create_transfer(Replay& R, const C& c, uint32_t k, uint64_t ts_event,
                                           const tb_transfer_t& t, const EvRefs& x,
                                           uint64_t* ts_out) {
    const Tables& T = R.T;
    const uint16_t f = t.flags;
    // Every load the outcome needs whose address is known goes out first (the id slot's word, then
    // both account rows): the checks below overlap them instead of waiting on each in turn.
    const uint64_t w_slot = x.slot != kNone32 ? T.tr.slots[x.slot] : kEmpty;
    const bool rows_early = !(f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING)) &&
                            x.dr != kNone32 && x.cr != kNone32;
    tb_account_t dr, cr;
    if (rows_early) {
        dr = T.acc_rows[x.dr];
        cr = T.acc_rows[x.cr];
    }
    R.flush_adds();  // (the previous event's carries, behind this event's loads)
    if (f & TB_TRANSFER_PADDING_MASK) return TB_CT_RESERVED_FLAG;
    if (u128_is_zero(t.id)) return TB_CT_ID_MUST_NOT_BE_ZERO;
    if (u128_is_max(t.id)) return TB_CT_ID_MUST_NOT_BE_INT_MAX;

    uint64_t e_row = 0;
    switch (replay_transfer_at_word(c, w_slot, k, &e_row)) {
        case 1: {
            const tb_transfer_t e = T.tr_rows[e_row];
            if ((t.flags == e.flags) && U(t.pending_id) == U(e.pending_id) &&
                t.timeout == e.timeout &&
                (t.flags & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING))) {
                uint64_t p_row = 0;
                replay_get_transfer_at_slot(T, c, transfer_slot_find(T, c, t.pending_id), k,
                                            &p_row);
                const tb_transfer_t p = T.tr_rows[p_row];
                return create_transfer_exists(t, e, &p, ts_out);
            }
            return create_transfer_exists(t, e, nullptr, ts_out);
        }
        case 2: return TB_CT_ID_ALREADY_FAILED;
        default: break;
    }

    if (f & (TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING))
        return replay_post_or_void(R, c, k, ts_event, t, x, ts_out);

    if (u128_is_zero(t.debit_account_id)) return TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (u128_is_max(t.debit_account_id)) return TB_CT_DEBIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (u128_is_zero(t.credit_account_id)) return TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_ZERO;
    if (u128_is_max(t.credit_account_id)) return TB_CT_CREDIT_ACCOUNT_ID_MUST_NOT_BE_INT_MAX;
    if (u128_eq(t.credit_account_id, t.debit_account_id)) return TB_CT_ACCOUNTS_MUST_BE_DIFFERENT;
    if (!u128_is_zero(t.pending_id)) return TB_CT_PENDING_ID_MUST_BE_ZERO;
    if (!(f & TB_TRANSFER_PENDING)) {
        if (t.timeout != 0) return TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
        if (f & (TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT))
            return TB_CT_CLOSING_TRANSFER_MUST_BE_PENDING;
    }
    if (t.ledger == 0) return TB_CT_LEDGER_MUST_NOT_BE_ZERO;
    if (t.code == 0) return TB_CT_CODE_MUST_NOT_BE_ZERO;

    const uint32_t dr_row = x.dr;
    if (dr_row == kNone32) return TB_CT_DEBIT_ACCOUNT_NOT_FOUND;
    const uint32_t cr_row = x.cr;
    if (cr_row == kNone32) return TB_CT_CREDIT_ACCOUNT_NOT_FOUND;
    // (rows_early holds here: both rows are loaded)
    if (dr.ledger != cr.ledger) return TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
    if (t.ledger != dr.ledger) return TB_CT_TRANSFER_MUST_HAVE_THE_SAME_LEDGER_AS_ACCOUNTS;

    uint64_t ts_actual = ts_event;
    if (f & TB_TRANSFER_IMPORTED) {
        if (t.timestamp <= T.scalars->transfers_key_max)
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        if (ts_index_contains(T.acc_ts_index, T.acc_ts_count, t.timestamp))
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        if (t.timestamp <= dr.timestamp)
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_POSTDATE_DEBIT_ACCOUNT;
        if (t.timestamp <= cr.timestamp)
            return TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_POSTDATE_CREDIT_ACCOUNT;
        if (t.timeout != 0) return TB_CT_IMPORTED_EVENT_TIMEOUT_MUST_BE_ZERO;
        ts_actual = t.timestamp;
    }
    if (dr.flags & TB_ACCOUNT_CLOSED) return TB_CT_DEBIT_ACCOUNT_ALREADY_CLOSED;
    if (cr.flags & TB_ACCOUNT_CLOSED) return TB_CT_CREDIT_ACCOUNT_ALREADY_CLOSED;

    u128 amount = U(t.amount);
    if (f & TB_TRANSFER_BALANCING_DEBIT) {
        u128 bal = U(dr.debits_posted) + U(dr.debits_pending);
        u128 cp = U(dr.credits_posted);
        u128 room = cp > bal ? cp - bal : 0;
        if (room < amount) amount = room;
    }
    if (f & TB_TRANSFER_BALANCING_CREDIT) {
        u128 bal = U(cr.credits_posted) + U(cr.credits_pending);
        u128 dp = U(cr.debits_posted);
        u128 room = dp > bal ? dp - bal : 0;
        if (room < amount) amount = room;
    }
    const u128 dpe = U(dr.debits_pending), dpo = U(dr.debits_posted);
    const u128 cpe = U(cr.credits_pending), cpo = U(cr.credits_posted);
    if (f & TB_TRANSFER_PENDING) {
        if (sum_overflows(amount, dpe)) return TB_CT_OVERFLOWS_DEBITS_PENDING;
        if (sum_overflows(amount, cpe)) return TB_CT_OVERFLOWS_CREDITS_PENDING;
    }
    if (sum_overflows(amount, dpo)) return TB_CT_OVERFLOWS_DEBITS_POSTED;
    if (sum_overflows(amount, cpo)) return TB_CT_OVERFLOWS_CREDITS_POSTED;
    if (sum_overflows(amount, dpe + dpo)) return TB_CT_OVERFLOWS_DEBITS;
    if (sum_overflows(amount, cpe + cpo)) return TB_CT_OVERFLOWS_CREDITS;
    if (ts_actual + (uint64_t)t.timeout * TB_NS_PER_S > TB_TIMESTAMP_MAX)
        return TB_CT_OVERFLOWS_TIMEOUT;
    if ((dr.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) && dpe + dpo + amount > U(dr.credits_posted))
        return TB_CT_EXCEEDS_CREDITS;
    if ((cr.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS) && cpe + cpo + amount > U(cr.debits_posted))
        return TB_CT_EXCEEDS_DEBITS;

    const uint64_t row = c.row_base + k;
    tb_transfer_t o = t;
    o.amount = W(amount);
    o.timestamp = ts_actual;
    T.tr_rows[row] = o;
    T.tr_status[row] = (f & TB_TRANSFER_PENDING) ? TB_PENDING_PENDING : TB_PENDING_NONE;
    R.note_transfer_ts(ts_actual);
    if ((f & TB_TRANSFER_PENDING) && t.timeout > 0 && !R.expiry_planned)
        expiry_append(T, row, !R.concurrent);

    tb_account_t dr_new = dr, cr_new = cr;
    if (f & TB_TRANSFER_PENDING) {
        dr_new.debits_pending = W(dpe + amount);
        cr_new.credits_pending = W(cpe + amount);
    } else {
        dr_new.debits_posted = W(dpo + amount);
        cr_new.credits_posted = W(cpo + amount);
    }
    if (f & TB_TRANSFER_CLOSING_DEBIT) dr_new.flags |= TB_ACCOUNT_CLOSED;
    if (f & TB_TRANSFER_CLOSING_CREDIT) cr_new.flags |= TB_ACCOUNT_CLOSED;
    const bool pend = (f & TB_TRANSFER_PENDING) != 0;
    // (additive rows are never closing: a closing transfer marks closable)
    const bool add_dr = R.additive(dr_row, x, kAddDr), add_cr = R.additive(cr_row, x, kAddCr);
    if (add_dr || add_cr)
        R.add_pq(add_dr ? dr_row : kNone32, add_cr ? cr_row : kNone32, pend ? amount : u128(0),
                 pend ? u128(0) : amount);
    if (!add_dr && (amount > 0 || (dr_new.flags & TB_ACCOUNT_CLOSED)))
        R.update_account(dr_row, dr, dr_new);
    if (!add_cr && (amount > 0 || (cr_new.flags & TB_ACCOUNT_CLOSED)))
        R.update_account(cr_row, cr, cr_new);

    if (t.timeout > 0) R.pulse_min(ts_actual + (uint64_t)t.timeout * TB_NS_PER_S);
    *ts_out = ts_actual;
    return TB_STATUS_CREATED;
}

// ---- accounts ---------------------------------------------------------------------------------

template <typename C>
__device__ inline int replay_get_account_at_slot(const Tables& T, const C& c, uint64_t s,
                                                 uint32_t k, uint64_t* row) {
    if (s == kNone) return 0;
    uint64_t w = T.acc.slots[s];
    if (w == kEmpty || w == kTomb) return 0;
    uint64_t r = (w & kRefMask) - 1;
    if (r < c.row_base) {
        *row = r;
        return 1;
    }
    uint64_t j = r - c.row_base;
    if (j >= k) return 0;
    if (c.results[j].status == TB_STATUS_CREATED) {
        *row = r;
        return 1;
    }
    return 0;
}

__device__ inline uint32_t create_account_exists(const tb_account_t& a, const tb_account_t& e,
                                                 uint64_t* ts) {
    if (a.flags != e.flags) return TB_CA_EXISTS_WITH_DIFFERENT_FLAGS;
    if (U(a.user_data_128) != U(e.user_data_128)) return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_128;
    if (a.user_data_64 != e.user_data_64) return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_64;
    if (a.user_data_32 != e.user_data_32) return TB_CA_EXISTS_WITH_DIFFERENT_USER_DATA_32;
    if (a.ledger != e.ledger) return TB_CA_EXISTS_WITH_DIFFERENT_LEDGER;
    if (a.code != e.code) return TB_CA_EXISTS_WITH_DIFFERENT_CODE;
    *ts = e.timestamp;
    return TB_CA_EXISTS;
}

// The checks of create_account after the id lookup (:3636-3650), shared by the parallel path.
__device__ inline uint32_t create_account_checks(const tb_account_t& a) {
    if ((a.flags & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) &&
        (a.flags & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS))
        return TB_CA_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    if (!u128_is_zero(a.debits_pending)) return TB_CA_DEBITS_PENDING_MUST_BE_ZERO;
    if (!u128_is_zero(a.debits_posted)) return TB_CA_DEBITS_POSTED_MUST_BE_ZERO;
    if (!u128_is_zero(a.credits_pending)) return TB_CA_CREDITS_PENDING_MUST_BE_ZERO;
    if (!u128_is_zero(a.credits_posted)) return TB_CA_CREDITS_POSTED_MUST_BE_ZERO;
    if (a.ledger == 0) return TB_CA_LEDGER_MUST_NOT_BE_ZERO;
    if (a.code == 0) return TB_CA_CODE_MUST_NOT_BE_ZERO;
    return TB_STATUS_CREATED;
}

__device__ inline tb_account_t account_row_of(const tb_account_t& a, uint64_t ts) {
    tb_account_t o;
    o.id = a.id;
    o.debits_pending = W(0);
    o.debits_posted = W(0);
    o.credits_pending = W(0);
    o.credits_posted = W(0);
    o.user_data_128 = a.user_data_128;
    o.user_data_64 = a.user_data_64;
    o.user_data_32 = a.user_data_32;
    o.reserved = 0;
    o.ledger = a.ledger;
    o.code = a.code;
    o.flags = a.flags;
    o.timestamp = ts;
    return o;
}

template <typename C>
__device__ uint32_t replay_create_account(Replay& R, const C& c, uint32_t k, uint64_t ts_event,
                                          const tb_account_t& a, const EvRefs& x,
                                          uint64_t* ts_out) {
    const Tables& T = R.T;
    if (a.reserved != 0) return TB_CA_RESERVED_FIELD;
    if (a.flags & TB_ACCOUNT_PADDING_MASK) return TB_CA_RESERVED_FLAG;
    if (u128_is_zero(a.id)) return TB_CA_ID_MUST_NOT_BE_ZERO;
    if (u128_is_max(a.id)) return TB_CA_ID_MUST_NOT_BE_INT_MAX;
    uint64_t e_row = 0;
    if (replay_get_account_at_slot(T, c, slot_or_none(x.slot), k, &e_row) == 1) {
        const tb_account_t e = T.acc_rows[e_row];
        return create_account_exists(a, e, ts_out);
    }
    uint32_t s = create_account_checks(a);
    if (s != TB_STATUS_CREATED) return s;
    uint64_t ts_actual = ts_event;
    if (a.flags & TB_ACCOUNT_IMPORTED) {
        if (a.timestamp <= T.scalars->accounts_key_max)
            return TB_CA_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        if (ts_index_contains(T.tr_ts_index, T.tr_ts_count, a.timestamp))
            return TB_CA_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS;
        ts_actual = a.timestamp;
    }
    T.acc_rows[c.row_base + k] = account_row_of(a, ts_actual);
    if (ts_actual > T.scalars->accounts_key_max) T.scalars->accounts_key_max = ts_actual;
    *ts_out = ts_actual;
    return TB_STATUS_CREATED;
}

}  // namespace tbg
