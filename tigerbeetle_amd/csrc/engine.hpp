// The exact engine of the ledger-sharded group (include/tbg_group.h): host C++
// that executes a call across shard executors exactly as the reference's serial execution would.
// It reads no HIP API: the executors are reached through tbg_shard_ops and the directories
// through the Directory interface, so the same code runs over HIP executors on N GPUs (shards.cpp)
// and over the CPU oracle in the tests.
//
// Placement (reference: src/state_machine.zig):
//  * an event whose id already exists goes to the id's holder: create_transfer_exists /
//    id_already_failed / create_account_exists are decided before any account lookup (:3629,
//    :3733-3738);
//  * a post/void goes to its pending transfer's shard (:4053-4299 read only the pending transfer,
//    its TransferPending status and its accounts); found nowhere, it fails
//    pending_transfer_not_found on any shard;
//  * a transfer goes to its accounts' shard, an account to its ledger's shard;
//  * a transfer whose accounts live on two shards fails accounts_must_have_the_same_ledger unless
//    an earlier static check fails first (:3748-3798) and never reads a balance: the shard runs a
//    surrogate (credit := debit), which fails at the same position with accounts_must_be_different
//    -- non-transient like the true status, which is patched in;
//  * an event whose status follows from its batch alone (the imported flag against the batch's
//    first event, execute_create :3050-3064) runs as an inert event (id 0, or an imported
//    timestamp 0) and gets the engine's status.
// Segments: maximal runs of whole linked chains whose events cannot observe another shard's state;
// a segment ends before a chain that repeats an id of the segment that would run elsewhere, an
// imported event at or below a timestamp another shard may create in the segment, or a linked
// chain across shards (a segment of its own, run by the chain protocol: every shard probes its
// part as one chain ending in a failing sentinel; the first failure across shards decides).
// pulse_next_timestamp: the shards record their updates with global timestamps (tbg_set_pnt_sharded);
// a post/void's reset-if-equal (:4227-4229) is resolved over all shards' updates in call order.
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../include/tbg_group.h"

namespace tbs {

using u128 = unsigned __int128;
constexpr u128 kU128Max = ~u128(0);

inline u128 U(const tb_uint128_t& x) { return (u128(x.hi) << 64) | x.lo; }
inline tb_uint128_t T128(u128 x) {
    tb_uint128_t r;
    r.lo = uint64_t(x);
    r.hi = uint64_t(x >> 64);
    return r;
}

// An engine failure: a shard returned an error (its code) or the call is malformed.
struct EngineError : std::runtime_error {
    int code;
    EngineError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

inline uint64_t mix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ull;
    x ^= x >> 33;
    return x;
}

// u128 -> int32, open addressing with linear probing; clear() is O(1) (generation stamps).
class IdMap {
    struct Slot {
        u128 key;
        int32_t val;
        uint32_t gen;
    };
    std::vector<Slot> slots_;
    size_t mask_ = 0, size_ = 0;
    uint32_t gen_ = 1;
    size_t home(u128 k) const { return mix64(uint64_t(k) ^ mix64(uint64_t(k >> 64))) & mask_; }
    void grow() {
        std::vector<Slot> old;
        old.swap(slots_);
        slots_.assign(old.size() * 2, Slot{0, 0, 0});
        mask_ = slots_.size() - 1;
        size_ = 0;
        for (const Slot& s : old)
            if (s.gen == gen_) insert(s.key, s.val);
    }

   public:
    explicit IdMap(size_t cap = 32) {
        size_t c = 16;
        while (c < cap * 2) c <<= 1;
        slots_.assign(c, Slot{0, 0, 0});
        mask_ = c - 1;
    }
    void clear() {
        size_ = 0;
        if (++gen_ == 0) {
            for (Slot& s : slots_) s.gen = 0;
            gen_ = 1;
        }
    }
    size_t size() const { return size_; }
    const int32_t* find(u128 k) const {
        for (size_t i = home(k);; i = (i + 1) & mask_) {
            const Slot& s = slots_[i];
            if (s.gen != gen_) return nullptr;
            if (s.key == k) return &s.val;
        }
    }
    bool has(u128 k) const { return find(k) != nullptr; }
    // Inserts unless present (the first value is kept); true if inserted.
    bool insert(u128 k, int32_t v) {
        if ((size_ + 1) * 2 > slots_.size()) grow();
        for (size_t i = home(k);; i = (i + 1) & mask_) {
            Slot& s = slots_[i];
            if (s.gen != gen_) {
                s = Slot{k, v, gen_};
                size_++;
                return true;
            }
            if (s.key == k) return false;
        }
    }
    void set(u128 k, int32_t v) {
        if (!insert(k, v)) {
            for (size_t i = home(k);; i = (i + 1) & mask_)
                if (slots_[i].key == k) {
                    slots_[i].val = v;
                    return;
                }
        }
    }
};

// Where every account id and every transfer id (created, or orphaned by a transient failure)
// lives: host maps (groups over other executors) or the device router's HBM directories.
struct Directory {
    virtual ~Directory() {}
    // out[i] = the shard, or -1
    virtual void account_shards(const std::vector<u128>& ids, std::vector<int32_t>& out) = 0;
    virtual void transfer_shards(const std::vector<u128>& ids, std::vector<int32_t>& out) = 0;
    // (a repeated id keeps its first holder)
    virtual void record_accounts(const std::vector<u128>& ids, const std::vector<uint8_t>& sh) = 0;
    virtual void record_transfers(const std::vector<u128>& ids, const std::vector<uint8_t>& sh) = 0;
};

struct HostDirectory : Directory {
    IdMap acc{1024}, tr{1024};
    void account_shards(const std::vector<u128>& ids, std::vector<int32_t>& out) override {
        out.resize(ids.size());
        for (size_t i = 0; i < ids.size(); i++) {
            const int32_t* v = acc.find(ids[i]);
            out[i] = v ? *v : -1;
        }
    }
    void transfer_shards(const std::vector<u128>& ids, std::vector<int32_t>& out) override {
        out.resize(ids.size());
        for (size_t i = 0; i < ids.size(); i++) {
            const int32_t* v = tr.find(ids[i]);
            out[i] = v ? *v : -1;
        }
    }
    void record_accounts(const std::vector<u128>& ids, const std::vector<uint8_t>& sh) override {
        for (size_t i = 0; i < ids.size(); i++) acc.insert(ids[i], sh[i]);
    }
    void record_transfers(const std::vector<u128>& ids, const std::vector<uint8_t>& sh) override {
        for (size_t i = 0; i < ids.size(); i++) tr.insert(ids[i], sh[i]);
    }
};

// Runs a function for a set of shards: one at a time, or on the group's per-shard threads.
struct Runner {
    virtual ~Runner() {}
    virtual void run(const std::vector<int>& shards, const std::function<int(int)>& fn,
                     std::vector<int>& rcs) {
        rcs.assign(shards.size(), 0);
        for (size_t i = 0; i < shards.size(); i++) rcs[i] = fn(shards[i]);
    }
};

enum Kind { kAccounts = 0, kTransfers = 1 };

struct KindInfo {
    uint16_t imported_flag;
    uint32_t inert_plain;     // an inert event's status in a non-imported batch (id_must_not_be_zero)
    uint32_t inert_imported;  // ... in an imported batch (imported_event_timestamp_out_of_range)
    uint32_t expected, not_expected, regress;
};
constexpr KindInfo kKinds[2] = {
    {TB_ACCOUNT_IMPORTED, TB_CA_ID_MUST_NOT_BE_ZERO, TB_CA_IMPORTED_EVENT_TIMESTAMP_OUT_OF_RANGE,
     TB_CA_IMPORTED_EVENT_EXPECTED, TB_CA_IMPORTED_EVENT_NOT_EXPECTED,
     TB_CA_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS},
    {TB_TRANSFER_IMPORTED, TB_CT_ID_MUST_NOT_BE_ZERO, TB_CT_IMPORTED_EVENT_TIMESTAMP_OUT_OF_RANGE,
     TB_CT_IMPORTED_EVENT_EXPECTED, TB_CT_IMPORTED_EVENT_NOT_EXPECTED,
     TB_CT_IMPORTED_EVENT_TIMESTAMP_MUST_NOT_REGRESS},
};

constexpr uint32_t kLinkedEventFailed = 1;  // (the same value for accounts and transfers)
constexpr uint32_t kLinkedEventChainOpen = 2;
constexpr uint64_t kPntReset = 1ull << 63;  // a recorded update that is a reset-if-equal
constexpr uint16_t kPostVoid = TB_TRANSFER_POST_PENDING | TB_TRANSFER_VOID_PENDING;
constexpr uint16_t kClosing = TB_TRANSFER_CLOSING_DEBIT | TB_TRANSFER_CLOSING_CREDIT;

// Event fields at their offsets: Account and Transfer share ledger (112), code (116), flags (118)
// and timestamp (120); src/tigerbeetle.zig:10-116.
inline uint16_t ev_flags(const uint8_t* e) { uint16_t v; memcpy(&v, e + 118, 2); return v; }
inline uint32_t ev_ledger(const uint8_t* e) { uint32_t v; memcpy(&v, e + 112, 4); return v; }
inline uint16_t ev_code(const uint8_t* e) { uint16_t v; memcpy(&v, e + 116, 2); return v; }
inline uint64_t ev_timestamp(const uint8_t* e) { uint64_t v; memcpy(&v, e + 120, 8); return v; }
inline u128 ev_u128(const uint8_t* e, int off) {
    tb_uint128_t v;
    memcpy(&v, e + off, 16);
    return U(v);
}
inline uint32_t ev_u32(const uint8_t* e, int off) { uint32_t v; memcpy(&v, e + off, 4); return v; }

// create_transfer's status (:3748-3798) for a transfer whose two accounts exist on different
// shards (so on different ledgers), from the checks after accounts_must_be_different.
inline uint32_t cross_status(u128 pending_id, uint16_t flags, uint32_t timeout, uint32_t ledger,
                             uint16_t code) {
    if (pending_id != 0) return TB_CT_PENDING_ID_MUST_BE_ZERO;
    if (!(flags & TB_TRANSFER_PENDING)) {
        if (timeout != 0) return TB_CT_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER;
        if (flags & kClosing) return TB_CT_CLOSING_TRANSFER_MUST_BE_PENDING;
    }
    if (ledger == 0) return TB_CT_LEDGER_MUST_NOT_BE_ZERO;
    if (code == 0) return TB_CT_CODE_MUST_NOT_BE_ZERO;
    return TB_CT_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER;
}

// create_account's checks that read no state (:3623-3646) except the id lookup: the first
// failing one, or 0.
inline uint32_t account_static_status(const uint8_t* a) {
    if (ev_u32(a, 108) != 0) return TB_CA_RESERVED_FIELD;
    const uint16_t f = ev_flags(a);
    if (f & TB_ACCOUNT_PADDING_MASK) return TB_CA_RESERVED_FLAG;
    const u128 id = ev_u128(a, 0);
    if (id == 0) return TB_CA_ID_MUST_NOT_BE_ZERO;
    if (id == kU128Max) return TB_CA_ID_MUST_NOT_BE_INT_MAX;
    if ((f & TB_ACCOUNT_DEBITS_MUST_NOT_EXCEED_CREDITS) &&
        (f & TB_ACCOUNT_CREDITS_MUST_NOT_EXCEED_DEBITS))
        return TB_CA_FLAGS_ARE_MUTUALLY_EXCLUSIVE;
    static const uint32_t st[4] = {TB_CA_DEBITS_PENDING_MUST_BE_ZERO,
                                   TB_CA_DEBITS_POSTED_MUST_BE_ZERO,
                                   TB_CA_CREDITS_PENDING_MUST_BE_ZERO,
                                   TB_CA_CREDITS_POSTED_MUST_BE_ZERO};
    for (int i = 0; i < 4; i++)
        if (ev_u128(a, 16 + 16 * i) != 0) return st[i];
    if (ev_ledger(a) == 0) return TB_CA_LEDGER_MUST_NOT_BE_ZERO;
    if (ev_code(a) == 0) return TB_CA_CODE_MUST_NOT_BE_ZERO;
    return 0;
}

using PntOps = std::vector<std::pair<uint64_t, uint64_t>>;  // (event timestamp, op)

// Does a reset of pulse_next_timestamp fire in the call's order across shards? `starts`: the
// shards' values at the segment's start; `ops`: per shard its recorded updates -- an expiry (a
// `min`) or an expiry | kPntReset (reset-if-equal, post_or_void_pending_transfer :4227-4229).
inline bool pnt_resets_fire(const std::vector<uint64_t>& starts, const std::vector<PntOps>& ops) {
    uint64_t value = ~0ull;
    for (uint64_t s : starts) value = std::min(value, s);
    PntOps all;
    for (const PntOps& o : ops) all.insert(all.end(), o.begin(), o.end());
    std::sort(all.begin(), all.end());
    for (const auto& e : all) {
        const uint64_t op = e.second;
        if (op & kPntReset) {
            if (value == (op & ~kPntReset)) return true;  // (timestamp_min from here on)
        } else if (op < value) {
            value = op;
        }
    }
    return false;
}

// One sharded pulse (ExpirePendingTransfersType :4875-5029 over all shards): every shard reports
// how many of its expires_at entries have expired and the first pulse_batch_max keys (expires_at,
// timestamp); below pulse_batch_max in total every shard expires all of its own, else the
// pulse_batch_max-th key across shards is the cut. Expiry i of the pulse's E (in key order over
// all shards) is stamped timestamp - E + i + 1 (:4540-4546).
struct PulsePlan {
    uint64_t cut_e = 0, cut_t = 0, pnt = 0;  // pnt 0: each shard's own next expiry
    std::vector<std::vector<uint64_t>> stamps;
};
inline PulsePlan pulse_plan(const std::vector<uint64_t>& counts,
                            const std::vector<std::vector<std::pair<uint64_t, uint64_t>>>& keys,
                            uint32_t pbm, uint64_t timestamp) {
    PulsePlan p;
    p.stamps.resize(keys.size());
    uint64_t total = 0;
    for (uint64_t c : counts) total += c;
    struct M {
        uint64_t e, t;
        uint32_t s;
        bool operator<(const M& o) const {
            return e != o.e ? e < o.e : (t != o.t ? t < o.t : s < o.s);
        }
    };
    std::vector<M> merged;
    for (uint32_t s = 0; s < keys.size(); s++)
        for (const auto& k : keys[s]) merged.push_back(M{k.first, k.second, s});
    std::sort(merged.begin(), merged.end());
    const bool cut = total >= pbm && pbm > 0;
    if (cut) {
        const M c = merged[pbm - 1];
        p.cut_e = c.e;
        p.cut_t = c.t;
        p.pnt = c.e;
        merged.resize(pbm);  // keys are unique: exactly the keys <= the cut
    } else if (!merged.empty()) {
        p.cut_e = merged.back().e;
        p.cut_t = merged.back().t;
    }
    const uint64_t E = merged.size();
    for (uint64_t i = 0; i < E; i++) p.stamps[merged[i].s].push_back(timestamp - E + i + 1);
    return p;
}

// One executor call of a shard: "batches" (lens, batch timestamps) or "stamped" (per-event
// timestamps, one batch whose timestamp is batch_ts; one_chain: the batch is one linked chain
// closed at its last event, whatever the events' linked flags -- a part of a chain across
// shards).
struct SubCall {
    bool stamped = false, one_chain = false;
    std::vector<uint32_t> pos;      // the events' positions in the call
    std::vector<uint8_t> ev;        // their exec form, 128 B each
    std::vector<uint32_t> lens;     // batches
    std::vector<uint64_t> ts;       // batch timestamps (batches) | event timestamps (stamped)
    uint64_t batch_ts = 0;          // stamped
    std::vector<tb_create_result_t> out;
    uint32_t n() const { return uint32_t(ev.size() / 128); }
};
struct ShardRun {
    std::vector<SubCall> calls;
    uint64_t pnt_start = 0;
    PntOps pnt;
};

struct EngineStats {
    uint64_t segments = 0, chain_segments = 0;
};

class Engine {
   public:
    Engine(uint32_t shards, uint32_t ledgers, uint32_t max_batches, const tbg_shard_ops* ops,
           std::vector<void*> selves, Directory* dir, Runner* runner)
        : W(shards), ledgers_(ledgers), max_batches_(max_batches), ops_(ops),
          self_(std::move(selves)), dir_(dir), runner_(runner) {}

    uint32_t shard_of_ledger(uint32_t ledger) const {
        if (ledger >= 1 && ledger <= ledgers_) return uint32_t(uint64_t(ledger - 1) * W / ledgers_);
        return ledger % W;
    }

    // Executes a call (module doc): results in call order.
    void run(Kind kind, const uint8_t* events, uint32_t n, const uint32_t* lens,
             const uint64_t* batch_ts, uint32_t nb, tb_create_result_t* results);

    // The segments a call is cut into against the current directories (nothing executes).
    struct PlannedSeg {
        uint32_t end;
        bool chain;
    };
    void plan_only(Kind kind, const uint8_t* events, uint32_t n, const uint32_t* lens,
                   const uint64_t* batch_ts, uint32_t nb, std::vector<PlannedSeg>& segs,
                   std::vector<int32_t>& shard_of);

    // The shard-group operations (also used by the group for pulses and key maxima).
    void execute(Kind kind, std::vector<ShardRun>& runs);
    std::vector<uint64_t> pnt_values();
    void set_pnt(const std::vector<uint64_t>& values);
    std::pair<uint64_t, uint64_t> sync_key_max();
    int64_t pulse(uint64_t timestamp, uint32_t pbm);
    uint64_t pulse_next_timestamp();

    EngineStats stats;
    const uint32_t W;

   private:
    // A call's events with everything placement reads, computed once.
    struct Call {
        Kind kind;
        bool is_tr;
        uint32_t n = 0, nb = 0;
        const uint8_t* ev = nullptr;
        std::vector<uint32_t> b_of, batch_start, batch_end;
        std::vector<uint64_t> batch_ts, stamp, ts;
        std::vector<uint8_t> g_batch, G, open_last, imp_live;
        std::vector<uint16_t> flags;
        std::vector<int32_t> pre;  // execute_create's batch-context status (:3050-3064) or -1
        std::vector<u128> ids, drs, crs, pids;
        std::vector<uint32_t> chain_end;  // at chain starts
        std::vector<int64_t> potential;   // a creation timestamp the event may take, or -1
    };
    struct Known {
        IdMap accounts{1024}, transfers{1024};
    };
    struct Seg {
        uint32_t start = 0, end = 0;
        bool chain = false, imported = false, post_void = false, tprime = false;
    };
    static constexpr int32_t kNone = -1, kCross = -2;

    void make_call(Call& c, Kind kind, const uint8_t* events, uint32_t n, const uint32_t* lens,
                   const uint64_t* batch_ts, uint32_t nb);
    void known_for(const Call& c, Known& kn);
    void collisions_for(const Call& c);
    void reset_call_arrays(uint32_t n);
    int32_t natural_transfer(const Call& c, const Known& kn, uint32_t k, const IdMap& chain_first,
                             const IdMap& seg_ids) const;
    bool place_chain(const Call& c, const Known& kn, uint32_t a, uint32_t z, const IdMap& seg_ids,
                     uint64_t* shard_mask);
    bool imported_decisions(const Call& c, const Known& kn, uint32_t a, uint32_t z, bool multi,
                            const IdMap& seg_ids);
    Seg plan(const Call& c, const Known& kn, uint32_t start);
    std::vector<uint8_t> exec_events(const Call& c, const Seg& seg, uint32_t a, uint32_t z);
    void tprime_values(const Call& c, const Seg& seg);
    void run_segment(const Call& c, const Seg& seg, tb_create_result_t* results);
    void run_chain(const Call& c, const Seg& seg, tb_create_result_t* results);
    void patch(tb_create_result_t* results, uint32_t k) const {
        if (patch_status_[k] && results[k].status == patch_expect_[k])
            results[k].status = patch_status_[k];
    }
    void record(const Call& c, const Seg& seg, const tb_create_result_t* results, Known& kn);
    void fail(int rc, const char* what) const;

    uint32_t ledgers_, max_batches_;
    const tbg_shard_ops* ops_;
    std::vector<void*> self_;
    Directory* dir_;
    Runner* runner_;

    // per call, indexed by event: the planner's decisions (place, surrogates, inert statuses,
    // timestamp surrogates) and the result patches
    std::vector<int32_t> place_, tprime_;
    std::vector<uint32_t> cross_, decided_, patch_expect_, patch_status_;
    std::vector<uint64_t> tprime_ts_;
    // imported timestamp -> shards holding an object of the other groove (bit s)
    std::vector<std::pair<uint64_t, uint64_t>> coll_;
    uint64_t coll_of(uint64_t t) const {
        auto it = std::lower_bound(coll_.begin(), coll_.end(), std::make_pair(t, uint64_t(0)));
        return it != coll_.end() && it->first == t ? it->second : 0;
    }
};

}  // namespace tbs
