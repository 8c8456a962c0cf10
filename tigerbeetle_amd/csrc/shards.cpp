// The ledger-sharded executor group (include/tbg_group.h): one process owns N executors, the
// device router and the exact engine (engine.cpp).
//
// Threads: a group of HIP executors runs one host thread per shard, its HIP device current, for
// the work every shard does at once -- a routed call's slices (peer copy in, execute, peer copy
// out), the exact engine's sub-calls of a segment. Everything else runs on the caller's thread
// (every tbg_* entry point makes its executor's device current).
//
// Transport: the router's scatter (tbr_pass2) stores each shard's slice straight into that shard's
// buffers in its own GPU's HBM (stores across xGMI; peer access enabled at open), and settle reads
// the results the shard's executor wrote there: no staging copy and no DMA-engine hand-off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/tb_state_machine.h"
#include "../../include/tbg.h"
#include "../../include/tbg_group.h"
#include "../../include/tbr.h"
#include "engine.hpp"

using tbs::u128;

namespace {

// The device router's directories behind the engine's Directory interface.
struct DeviceDirectory : tbs::Directory {
    tbr_ctx* r;
    explicit DeviceDirectory(tbr_ctx* ctx) : r(ctx) {}
    static std::vector<tb_uint128_t> pack(const std::vector<u128>& ids) {
        std::vector<tb_uint128_t> q(ids.size());
        for (size_t i = 0; i < ids.size(); i++) q[i] = tbs::T128(ids[i]);
        return q;
    }
    void lookup(bool transfers, const std::vector<u128>& ids, std::vector<int32_t>& out) {
        out.assign(ids.size(), -1);
        if (ids.empty()) return;
        const std::vector<tb_uint128_t> q = pack(ids);
        const int64_t rc = transfers ? tbr_transfer_shards(r, q.data(), uint32_t(q.size()), out.data())
                                     : tbr_account_shards(r, q.data(), uint32_t(q.size()), out.data());
        if (rc < 0) throw tbs::EngineError(int(rc), "directory lookup failed");
        for (int32_t& x : out)
            if (x >= 0) x &= 0x7F;
    }
    void account_shards(const std::vector<u128>& ids, std::vector<int32_t>& out) override {
        lookup(false, ids, out);
    }
    void transfer_shards(const std::vector<u128>& ids, std::vector<int32_t>& out) override {
        lookup(true, ids, out);
    }
    void record(bool transfers, const std::vector<u128>& ids, const std::vector<uint8_t>& sh) {
        if (ids.empty()) return;
        const std::vector<tb_uint128_t> q = pack(ids);
        const int rc = transfers ? tbr_record_transfers(r, q.data(), sh.data(), uint32_t(q.size()))
                                 : tbr_record_accounts(r, q.data(), sh.data(), uint32_t(q.size()));
        if (rc != 0) throw tbs::EngineError(rc, "directory record failed (capacity?)");
    }
    void record_accounts(const std::vector<u128>& ids, const std::vector<uint8_t>& sh) override {
        record(false, ids, sh);
    }
    void record_transfers(const std::vector<u128>& ids, const std::vector<uint8_t>& sh) override {
        record(true, ids, sh);
    }
};

// One host thread per shard, its device current: the Runner of a group of HIP executors.
class PoolRunner : public tbs::Runner {
    struct Worker {
        std::thread th;
        std::function<int()> job;
        bool has = false;
        int rc = 0;
    };
    std::vector<Worker> w_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    size_t pending_ = 0;
    bool stop_ = false;

    void loop(size_t i, int device) {
        (void)hipSetDevice(device);
        std::unique_lock<std::mutex> lk(m_);
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || w_[i].has; });
            if (stop_ && !w_[i].has) return;
            std::function<int()> job = std::move(w_[i].job);
            lk.unlock();
            int rc;
            try {
                rc = job();
            } catch (const std::exception&) {
                rc = TBG_EHIP;
            }
            lk.lock();
            w_[i].rc = rc;
            w_[i].has = false;
            if (--pending_ == 0) done_cv_.notify_all();
        }
    }

   public:
    explicit PoolRunner(const std::vector<uint32_t>& devices) : w_(devices.size()) {
        for (size_t i = 0; i < devices.size(); i++)
            w_[i].th = std::thread(&PoolRunner::loop, this, i, int(devices[i]));
    }
    ~PoolRunner() override {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (Worker& x : w_)
            if (x.th.joinable()) x.th.join();
    }
    void run(const std::vector<int>& shards, const std::function<int(int)>& fn,
             std::vector<int>& rcs) override {
        rcs.assign(shards.size(), 0);
        if (shards.empty()) return;
        {
            std::lock_guard<std::mutex> lk(m_);
            for (int s : shards) {
                w_[s].job = [&fn, s] { return fn(s); };
                w_[s].has = true;
                w_[s].rc = 0;
            }
            pending_ = shards.size();
        }
        cv_.notify_all();
        std::unique_lock<std::mutex> lk(m_);
        done_cv_.wait(lk, [&] { return pending_ == 0; });
        for (size_t i = 0; i < shards.size(); i++) rcs[i] = w_[shards[i]].rc;
    }
};

// The tbg.h executor as a shard (tbg_shard_ops): the tbg_* functions themselves.
tbg_shard_ops tbg_ops() {
    tbg_shard_ops o;
    o.create_accounts = reinterpret_cast<decltype(o.create_accounts)>(&tbg_create_accounts);
    o.create_transfers = reinterpret_cast<decltype(o.create_transfers)>(&tbg_create_transfers);
    o.create_accounts_stamped =
        reinterpret_cast<decltype(o.create_accounts_stamped)>(&tbg_create_accounts_stamped);
    o.create_transfers_stamped =
        reinterpret_cast<decltype(o.create_transfers_stamped)>(&tbg_create_transfers_stamped);
    o.forget_orphans = reinterpret_cast<decltype(o.forget_orphans)>(&tbg_forget_orphans);
    o.timestamps_exist = reinterpret_cast<decltype(o.timestamps_exist)>(&tbg_timestamps_exist);
    o.key_max = reinterpret_cast<decltype(o.key_max)>(&tbg_key_max);
    o.raise_key_max = reinterpret_cast<decltype(o.raise_key_max)>(&tbg_raise_key_max);
    o.set_pnt_sharded = reinterpret_cast<decltype(o.set_pnt_sharded)>(&tbg_set_pnt_sharded);
    o.pnt_ops = reinterpret_cast<decltype(o.pnt_ops)>(&tbg_pnt_ops);
    o.pulse_next_timestamp =
        reinterpret_cast<decltype(o.pulse_next_timestamp)>(&tbg_pulse_next_timestamp);
    o.set_pulse_next_timestamp =
        reinterpret_cast<decltype(o.set_pulse_next_timestamp)>(&tbg_set_pulse_next_timestamp);
    o.pulse_candidates = reinterpret_cast<decltype(o.pulse_candidates)>(&tbg_pulse_candidates);
    o.pulse_cut = reinterpret_cast<decltype(o.pulse_cut)>(&tbg_pulse_cut);
    o.lookup_accounts = reinterpret_cast<decltype(o.lookup_accounts)>(&tbg_lookup_accounts);
    o.lookup_transfers = reinterpret_cast<decltype(o.lookup_transfers)>(&tbg_lookup_transfers);
    return o;
}

// A shard's slice buffers, in its own GPU's HBM.
struct ShardLink {
    uint32_t device = 0;
    uint64_t cap = 0;  // events its slice holds (its executor's batch_events_max)
    tb_transfer_t* ev = nullptr;
    uint64_t* ts = nullptr;
    tb_create_result_t* res = nullptr;
};

template <typename T>
bool dalloc(T** p, uint64_t count) {
    return hipMalloc(reinterpret_cast<void**>(p), std::max<size_t>(count * sizeof(T), 16)) ==
           hipSuccess;
}

// Makes `device` current for the scope (restores the caller's).
struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != device) (void)hipSetDevice(device);
    }
    ~DeviceScope() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace

struct tbg_group {
    tbg_group_options o{};
    bool gpu = false;
    tbg_shard_ops ops{};
    std::vector<void*> shards;
    std::unique_ptr<tbs::Directory> dir;
    std::unique_ptr<tbs::Runner> runner;
    std::unique_ptr<tbs::Engine> eng;
    std::string error = "";
    tbg_group_stats st{};
    // groups of HIP executors
    tbr_ctx* tbr = nullptr;
    std::vector<ShardLink> link;
    tb_transfer_t* d_in_ev = nullptr;  // host-buffer calls' staging (router GPU)
    uint32_t* d_in_ends = nullptr;
    uint64_t* d_in_ts = nullptr;
    tb_create_result_t* d_in_res = nullptr;
    uint32_t* d_pos = nullptr;  // the scatter's positions (router GPU)
    uint64_t floor = ~0ull;  // the imported floor (unknown until an engine call)
    bool floor_known = false;
};

namespace {

uint64_t now_ns() {
    return uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now().time_since_epoch())
                        .count());
}

int fail(tbg_group* g, int rc, const std::string& what) {
    g->error = what;
    return rc < 0 ? rc : TBG_EHIP;
}

// After a call the exact engine executed: every shard's key maxima raised to the maxima over all
// shards, and their maximum is the device router's imported floor (tbr.h).
void refresh_floor(tbg_group* g) {
    if (!g->tbr) return;
    const auto km = g->eng->sync_key_max();
    g->floor = std::max(km.first, km.second);
    g->floor_known = true;
    tbr_set_imported_floor(g->tbr, g->floor);
}

int engine_call(tbg_group* g, tbs::Kind kind, const void* events, uint32_t n,
                const uint32_t* lens, const uint64_t* bts, uint32_t nb,
                tb_create_result_t* results) {
    const uint64_t t0 = now_ns();
    try {
        const tbs::EngineStats before = g->eng->stats;
        g->eng->run(kind, static_cast<const uint8_t*>(events), n, lens, bts, nb, results);
        g->st.segments += g->eng->stats.segments - before.segments;
        g->st.chain_segments += g->eng->stats.chain_segments - before.chain_segments;
        g->st.engine_calls++;
        refresh_floor(g);
    } catch (const tbs::EngineError& e) {
        return fail(g, e.code, e.what());
    }
    g->st.engine_ns += now_ns() - t0;
    return 0;
}

// The device path of a routed call (events resident on the router's GPU). Returns 0 when the
// call executed, 1 when it holds a hazard (nothing executed), < 0 on error.
int route_device(tbg_group* g, const tb_transfer_t* d_ev, uint32_t n, const uint32_t* d_ends,
                 const uint64_t* d_ts, uint32_t nb, tb_create_result_t* d_res) {
    const uint32_t W = g->o.shards;
    std::vector<uint32_t> counts(W, 0);
    std::vector<tbr_slice> slices(W);
    for (uint32_t s = 0; s < W; s++)
        slices[s] = tbr_slice{g->link[s].ev, g->link[s].ts, g->link[s].res, g->link[s].cap};
    const uint64_t t0 = now_ns();
    const int64_t mode = tbr_route_device_slices(g->tbr, d_ev, n, d_ends, d_ts, nb, slices.data(),
                                                 g->d_pos, counts.data());
    if (mode == TBG_EINVAL)
        return fail(g, TBG_EINVAL, "a shard's part of the call exceeds its batch_events_max");
    if (mode < 0) return fail(g, int(mode), "tbr_route_device");
    if (mode == 1) return 1;
    std::vector<int> run;
    for (uint32_t s = 0; s < W; s++)
        if (counts[s]) run.push_back(int(s));
    std::vector<int> rcs;
    const uint64_t t1 = now_ns();
    g->st.route_ns += t1 - t0;
    g->runner->run(run, [&](int s) -> int {
        const ShardLink& L = g->link[s];
        int rc = tbg_create_transfers_stamped_device(static_cast<tbg_ctx*>(g->shards[s]), L.ev,
                                                     counts[s], L.ts, L.res, nullptr);
        // (the executor may leave AccountEvents appends reading the slice behind the call)
        if (rc == 0) rc = tbg_synchronize(static_cast<tbg_ctx*>(g->shards[s]));
        return rc;
    }, rcs);
    for (size_t i = 0; i < rcs.size(); i++)
        if (rcs[i] != 0)
            return fail(g, rcs[i], "shard " + std::to_string(run[i]) + ": " +
                                       tbg_last_error(static_cast<tbg_ctx*>(g->shards[run[i]])) +
                                       " (the shards' state is undefined)");
    const uint64_t t2 = now_ns();
    g->st.execute_ns += t2 - t1;
    uint64_t km = 0;
    const int rc = tbr_settle_device(g->tbr, nullptr, g->d_pos, n, d_res, &km);
    if (rc != 0) return fail(g, rc, "tbr_settle_device");
    if (g->floor_known) {
        g->floor = std::max(g->floor, km);
        tbr_set_imported_floor(g->tbr, g->floor);
    }
    uint64_t rs[3] = {0, 0, 0};
    tbr_route_stats(g->tbr, rs);
    g->st.anywhere += rs[0];
    g->st.surrogates += rs[1];
    g->st.repeats += rs[2];
    g->st.device_calls++;
    if (mode == 2) {
        // a post/void may reset pulse_next_timestamp against the value over all shards
        // (:4227-4229): every shard's recorded updates replayed in call order
        std::vector<uint64_t> starts(W);
        std::vector<tbs::PntOps> ops(W);
        for (uint32_t s = 0; s < W; s++) {
            tbg_ctx* ctx = static_cast<tbg_ctx*>(g->shards[s]);
            if (!counts[s]) {
                starts[s] = tbg_pulse_next_timestamp(ctx);
                continue;
            }
            const int64_t m = tbg_pnt_ops(ctx, nullptr, nullptr, 0, &starts[s]);
            if (m < 0) return fail(g, int(m), "tbg_pnt_ops");
            std::vector<uint64_t> t(size_t(m) + 1), o(size_t(m) + 1);
            if (m && tbg_pnt_ops(ctx, t.data(), o.data(), uint64_t(m), &starts[s]) != m)
                return fail(g, TBG_EHIP, "tbg_pnt_ops");
            for (int64_t j = 0; j < m; j++) ops[s].emplace_back(t[j], o[j]);
        }
        if (tbs::pnt_resets_fire(starts, ops))
            for (uint32_t s = 0; s < W; s++)
                tbg_set_pulse_next_timestamp(static_cast<tbg_ctx*>(g->shards[s]), TB_TIMESTAMP_MIN);
    }
    g->st.settle_ns += now_ns() - t2;
    return 0;
}

bool valid_options(const tbg_group_options* o) {
    return o && o->shards >= 1 && o->shards <= TBG_GROUP_SHARDS_MAX && o->events_max > 0 &&
           o->batch_count_max > 0 && o->ledgers > 0;
}

void destroy(tbg_group* g) {
    if (!g) return;
    g->eng.reset();
    g->runner.reset();  // (joins the shard threads)
    if (g->gpu) {
        DeviceScope ds(int(g->o.router_device));
        for (ShardLink& L : g->link) {
            DeviceScope d2(int(L.device));
            void* ptrs[] = {L.ev, L.ts, L.res};
            for (void* p : ptrs)
                if (p) (void)hipFree(p);
        }
        void* ptrs[] = {g->d_in_ev, g->d_in_ends, g->d_in_ts, g->d_in_res, g->d_pos};
        {
            DeviceScope d3(int(g->o.router_device));
            for (void* p : ptrs)
                if (p) (void)hipFree(p);
        }
        if (g->tbr) tbr_close(g->tbr);
        for (void* s : g->shards)
            if (s) tbg_close(static_cast<tbg_ctx*>(s));
    }
    delete g;
}

// Lookups over every shard, found objects in request order.
template <typename Row>
int64_t lookup_all(tbg_group* g, const tb_uint128_t* ids, uint32_t n, Row* out,
                   int64_t (*fn)(void*, const tb_uint128_t*, uint32_t, Row*)) {
    std::vector<Row> rows;
    tbs::IdMap at(n + 16);
    std::vector<Row> buf(std::max<uint32_t>(n, 1));
    for (uint32_t s = 0; s < g->o.shards; s++) {
        const int64_t m = fn(g->shards[s], ids, n, buf.data());
        if (m < 0) return fail(g, int(m), "lookup");
        for (int64_t j = 0; j < m; j++)
            if (at.insert(tbs::U(buf[j].id), int32_t(rows.size()))) rows.push_back(buf[j]);
    }
    int64_t w = 0;
    for (uint32_t i = 0; i < n; i++)
        if (const int32_t* r = at.find(tbs::U(ids[i]))) out[w++] = rows[*r];
    return w;
}

// ---- the group as a tb_executor (tb_state_machine.h) ----------------------------------------

int gx_create_accounts(void* self, const tb_account_t* ev, uint32_t n, const uint32_t* lens,
                       const uint64_t* bts, uint32_t nb, tb_create_result_t* out) {
    return tbg_group_create_accounts(static_cast<tbg_group*>(self), ev, n, lens, bts, nb, out);
}
int gx_create_transfers(void* self, const tb_transfer_t* ev, uint32_t n, const uint32_t* lens,
                        const uint64_t* bts, uint32_t nb, tb_create_result_t* out) {
    return tbg_group_create_transfers(static_cast<tbg_group*>(self), ev, n, lens, bts, nb, out);
}
int64_t gx_pulse(void* self, uint64_t ts) { return tbg_group_pulse(static_cast<tbg_group*>(self), ts); }
uint64_t gx_pulse_next(void* self) {
    return tbg_group_pulse_next_timestamp(static_cast<tbg_group*>(self));
}
int64_t gx_lookup_accounts(void* self, const tb_uint128_t* ids, uint32_t n, tb_account_t* out) {
    return tbg_group_lookup_accounts(static_cast<tbg_group*>(self), ids, n, out);
}
int64_t gx_lookup_transfers(void* self, const tb_uint128_t* ids, uint32_t n, tb_transfer_t* out) {
    return tbg_group_lookup_transfers(static_cast<tbg_group*>(self), ids, n, out);
}

// A scan over every shard: each shard's first `limit` matches in the scan's order, merged by
// timestamp (descending when reversed), the first `limit` kept -- the reference's single scan over
// the union of the shards' objects (timestamps are unique across shards).
template <typename Row, typename Filter>
int64_t merged_scan(tbg_group* g, const Filter* f, uint32_t limit_max, Row* out, bool reversed,
                    uint64_t (*ts_of)(const Row&),
                    int64_t (*fn)(tbg_ctx*, const Filter*, uint32_t, Row*)) {
    if (!g->gpu) return fail(g, TBG_EINVAL, "scans need a group of HIP executors");
    std::vector<Row> all;
    std::vector<Row> buf(std::max<uint32_t>(limit_max, 1));
    for (uint32_t s = 0; s < g->o.shards; s++) {
        const int64_t m = fn(static_cast<tbg_ctx*>(g->shards[s]), f, limit_max, buf.data());
        if (m < 0) return fail(g, int(m), "scan");
        all.insert(all.end(), buf.begin(), buf.begin() + m);
    }
    std::stable_sort(all.begin(), all.end(), [&](const Row& x, const Row& y) {
        return reversed ? ts_of(x) > ts_of(y) : ts_of(x) < ts_of(y);
    });
    const uint32_t limit = std::min<uint32_t>(limit_max, f->limit);
    const size_t k = std::min<size_t>(all.size(), limit);
    std::copy(all.begin(), all.begin() + k, out);
    return int64_t(k);
}
uint64_t ce_ts(const tb_change_event_t& e) { return e.timestamp; }
uint64_t tr_ts(const tb_transfer_t& e) { return e.timestamp; }
uint64_t ac_ts(const tb_account_t& e) { return e.timestamp; }
uint64_t ab_ts(const tb_account_balance_t& e) { return e.timestamp; }

int64_t gx_change_events(void* self, const tb_change_events_filter_t* f, uint32_t m,
                         tb_change_event_t* out) {
    return merged_scan(static_cast<tbg_group*>(self), f, m, out, false, ce_ts,
                       &tbg_get_change_events);
}
int64_t gx_account_transfers(void* self, const tb_account_filter_t* f, uint32_t m,
                             tb_transfer_t* out) {
    return merged_scan(static_cast<tbg_group*>(self), f, m, out,
                       (f->flags & TB_ACCOUNT_FILTER_REVERSED) != 0, tr_ts,
                       &tbg_get_account_transfers);
}
int64_t gx_account_balances(void* self, const tb_account_filter_t* f, uint32_t m,
                            tb_account_balance_t* out) {
    return merged_scan(static_cast<tbg_group*>(self), f, m, out,
                       (f->flags & TB_ACCOUNT_FILTER_REVERSED) != 0, ab_ts,
                       &tbg_get_account_balances);
}
int64_t gx_query_accounts(void* self, const tb_query_filter_t* f, uint32_t m, tb_account_t* out) {
    return merged_scan(static_cast<tbg_group*>(self), f, m, out,
                       (f->flags & TB_QUERY_FILTER_REVERSED) != 0, ac_ts, &tbg_query_accounts);
}
int64_t gx_query_transfers(void* self, const tb_query_filter_t* f, uint32_t m,
                           tb_transfer_t* out) {
    return merged_scan(static_cast<tbg_group*>(self), f, m, out,
                       (f->flags & TB_QUERY_FILTER_REVERSED) != 0, tr_ts, &tbg_query_transfers);
}

}  // namespace

extern "C" {

tbg_group* tbg_group_open_shards(const tbg_group_options* options, const tbg_shard_ops* ops,
                                 void* const* shards) {
    if (!valid_options(options) || !ops || !shards) return nullptr;
    tbg_group* g = new tbg_group();
    g->o = *options;
    g->ops = *ops;
    g->shards.assign(shards, shards + options->shards);
    g->dir.reset(new tbs::HostDirectory());
    g->runner.reset(new tbs::Runner());
    g->eng.reset(new tbs::Engine(options->shards, options->ledgers, options->batch_count_max,
                                 &g->ops, g->shards, g->dir.get(), g->runner.get()));
    if (options->shards > 1)
        for (void* s : g->shards) g->ops.set_pnt_sharded(s, 1);
    return g;
}

}  // extern "C"

namespace {

// A group reopened from its shards' checkpoints: the router's directories hold every account id
// and every transfer id (created or orphaned) at its shard again, and the imported floor is the
// largest timestamp over the shards (the shards' own state -- tables, AccountEvents,
// pulse_next_timestamp, key ranges -- comes with their images).
int rebuild_directories(tbg_group* g) {
    DeviceScope ds(int(g->o.router_device));
    for (uint32_t s = 0; s < g->o.shards; s++) {
        tbg_ctx* ctx = static_cast<tbg_ctx*>(g->shards[s]);
        const int64_t na = tbg_dump_accounts(ctx, nullptr);
        if (na < 0) return int(na);
        std::vector<tb_account_t> a(static_cast<size_t>(na));
        if (na && tbg_dump_accounts(ctx, a.data()) != na) return TBG_EHIP;
        std::vector<tb_uint128_t> ids(a.size());
        for (size_t i = 0; i < a.size(); i++) ids[i] = a[i].id;
        std::vector<uint8_t> sh(ids.size(), uint8_t(s));
        int rc = tbr_record_accounts(g->tbr, ids.data(), sh.data(), uint32_t(ids.size()));
        if (rc) return rc;
        const int64_t nt = tbg_dump_transfer_ids(ctx, nullptr);
        if (nt < 0) return int(nt);
        ids.assign(size_t(nt), tb_uint128_t{});
        if (nt && tbg_dump_transfer_ids(ctx, ids.data()) != nt) return TBG_EHIP;
        sh.assign(ids.size(), uint8_t(s));
        rc = tbr_record_transfers(g->tbr, ids.data(), sh.data(), uint32_t(ids.size()));
        if (rc) return rc;
    }
    try {
        refresh_floor(g);
    } catch (const tbs::EngineError& e) {
        return e.code < 0 ? e.code : TBG_EHIP;
    }
    return 0;
}

tbg_group* open_gpu_group(const tbg_group_options* options, const tbg_options* shard_options,
                          const char* const* paths) {
    if (!valid_options(options) || !shard_options) return nullptr;
    if (options->router_transfer_capacity >= (1ull << 31) ||
        options->router_account_capacity >= (1ull << 31))
        return nullptr;
    const uint32_t W = options->shards;
    for (uint32_t s = 0; s < W; s++)
        if (shard_options[s].batch_count_max < options->batch_count_max)
            return nullptr;
    tbg_group* g = new tbg_group();
    g->o = *options;
    g->gpu = true;
    g->ops = tbg_ops();
    g->shards.assign(W, nullptr);
    g->link.resize(W);
    const int rdev = int(options->router_device);
    bool ok = true;
    for (uint32_t s = 0; s < W && ok; s++) {
        g->shards[s] = paths ? tbg_open_checkpoint(&shard_options[s], paths[s])
                             : tbg_open(&shard_options[s]);
        ok = g->shards[s] != nullptr;
        g->link[s].device = shard_options[s].device;
    }
    if (ok && W > 1) {
        const uint64_t E = options->events_max;
        DeviceScope ds(rdev);
        g->tbr = tbr_open(W, options->router_account_capacity, options->router_transfer_capacity,
                          options->events_max, uint32_t(rdev));
        ok = g->tbr && dalloc(&g->d_in_ev, E) && dalloc(&g->d_in_ends, E) &&
             dalloc(&g->d_in_ts, E) && dalloc(&g->d_in_res, E) && dalloc(&g->d_pos, E);
        for (uint32_t s = 0; s < W && ok; s++) {
            ShardLink& L = g->link[s];
            // a shard's slice can hold the whole call (every event may go to one shard)
            const uint64_t cap = std::min<uint64_t>(E, shard_options[s].batch_events_max);
            L.cap = cap;
            if (int(L.device) != rdev) {
                {
                    DeviceScope d2(rdev);  // (the router's kernels store and load there)
                    (void)hipDeviceEnablePeerAccess(int(L.device), 0);  // (already enabled: fine)
                }
                DeviceScope d3(int(L.device));
                (void)hipDeviceEnablePeerAccess(rdev, 0);
                (void)hipGetLastError();
            }
            DeviceScope d4(int(L.device));
            ok = dalloc(&L.ev, cap) && dalloc(&L.ts, cap) && dalloc(&L.res, cap);
        }
        (void)hipGetLastError();
    }
    if (!ok) {
        fprintf(stderr, "tbg_group_open: failed to open the shards or the router\n");
        destroy(g);
        return nullptr;
    }
    if (W > 1) {
        g->dir.reset(new DeviceDirectory(g->tbr));
        std::vector<uint32_t> devs(W);
        for (uint32_t s = 0; s < W; s++) devs[s] = g->link[s].device;
        g->runner.reset(new PoolRunner(devs));
        for (void* s : g->shards) tbg_set_pnt_sharded(static_cast<tbg_ctx*>(s), 1);
    } else {
        g->dir.reset(new tbs::HostDirectory());
        g->runner.reset(new tbs::Runner());
    }
    g->eng.reset(new tbs::Engine(W, options->ledgers, options->batch_count_max, &g->ops,
                                 g->shards, g->dir.get(), g->runner.get()));
    if (paths && W > 1) {
        const int rc = rebuild_directories(g);
        if (rc) {
            fprintf(stderr, "tbg_group_open_checkpoint: rebuilding the directories failed (%d)\n",
                    rc);
            destroy(g);
            return nullptr;
        }
    }
    return g;
}

}  // namespace

extern "C" {

tbg_group* tbg_group_open(const tbg_group_options* options, const tbg_options* shard_options) {
    return open_gpu_group(options, shard_options, nullptr);
}

void tbg_group_hip_shard_ops(tbg_shard_ops* out) {
    if (out) *out = tbg_ops();
}

tbg_group* tbg_group_open_checkpoint(const tbg_group_options* options,
                                     const tbg_options* shard_options, const char* const* paths) {
    return paths ? open_gpu_group(options, shard_options, paths) : nullptr;
}

int tbg_group_checkpoint(tbg_group* g, const char* const* paths) {
    if (!g || !g->gpu || !paths) return TBG_EINVAL;
    for (uint32_t s = 0; s < g->o.shards; s++) {
        tbg_ctx* ctx = static_cast<tbg_ctx*>(g->shards[s]);
        const int rc = tbg_checkpoint(ctx, paths[s]);
        if (rc) return fail(g, rc, "shard " + std::to_string(s) + " checkpoint: " + tbg_last_error(ctx));
    }
    return 0;
}

void tbg_group_close(tbg_group* g) { destroy(g); }

const char* tbg_group_last_error(const tbg_group* g) {
    return g ? g->error.c_str() : "no group";
}

void* tbg_group_shard(tbg_group* g, uint32_t s) {
    return g && s < g->o.shards ? g->shards[s] : nullptr;
}

int tbg_group_create_accounts(tbg_group* g, const tb_account_t* events, uint32_t n,
                              const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                              uint32_t n_batches, tb_create_result_t* results) {
    if (!g || n > g->o.events_max || (n && (!events || !results))) return TBG_EINVAL;
    g->st.calls++;
    if (g->o.shards == 1)
        return g->ops.create_accounts(g->shards[0], events, n, batch_lens, batch_timestamps,
                                      n_batches, results);
    return engine_call(g, tbs::kAccounts, events, n, batch_lens, batch_timestamps, n_batches,
                       results);
}

int tbg_group_create_transfers(tbg_group* g, const tb_transfer_t* events, uint32_t n,
                               const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                               uint32_t n_batches, tb_create_result_t* results) {
    if (!g || n > g->o.events_max || (n && (!events || !results))) return TBG_EINVAL;
    g->st.calls++;
    if (g->o.shards == 1)
        return g->ops.create_transfers(g->shards[0], events, n, batch_lens, batch_timestamps,
                                       n_batches, results);
    if (n && g->tbr && n_batches > 0) {
        // the device path: the call staged on the router's GPU
        DeviceScope ds(int(g->o.router_device));
        std::vector<uint32_t> ends(n_batches);
        uint64_t e = 0;
        for (uint32_t b = 0; b < n_batches; b++) ends[b] = uint32_t(e += batch_lens[b]);
        if (e != n) return fail(g, TBG_EINVAL, "batch lengths do not cover the events");
        if (hipMemcpy(g->d_in_ev, events, size_t(n) * 128, hipMemcpyHostToDevice) ||
            hipMemcpy(g->d_in_ends, ends.data(), size_t(n_batches) * 4, hipMemcpyHostToDevice) ||
            hipMemcpy(g->d_in_ts, batch_timestamps, size_t(n_batches) * 8, hipMemcpyHostToDevice))
            return fail(g, TBG_EHIP, "upload");
        const int rc = route_device(g, g->d_in_ev, n, g->d_in_ends, g->d_in_ts, n_batches,
                                    g->d_in_res);
        if (rc < 0) return rc;
        if (rc == 0) {
            if (hipMemcpy(results, g->d_in_res, size_t(n) * 16, hipMemcpyDeviceToHost))
                return fail(g, TBG_EHIP, "download");
            return 0;
        }
    }
    return engine_call(g, tbs::kTransfers, events, n, batch_lens, batch_timestamps, n_batches,
                       results);
}

int tbg_group_create_transfers_device(tbg_group* g, const tb_transfer_t* d_events, uint32_t n,
                                      const uint32_t* d_batch_ends,
                                      const uint64_t* d_batch_timestamps, uint32_t n_batches,
                                      tb_create_result_t* d_results) {
    if (!g || !g->gpu || n > g->o.events_max || n_batches == 0) return TBG_EINVAL;
    if (n == 0) return 0;
    g->st.calls++;
    if (g->o.shards == 1) {
        tbg_ctx* ctx = static_cast<tbg_ctx*>(g->shards[0]);
        int rc = tbg_create_transfers_device(ctx, d_events, n, d_batch_ends, d_batch_timestamps,
                                             n_batches, d_results, nullptr);
        return rc ? rc : tbg_synchronize(ctx);
    }
    DeviceScope ds(int(g->o.router_device));
    const int rc = route_device(g, d_events, n, d_batch_ends, d_batch_timestamps, n_batches,
                                d_results);
    if (rc <= 0) return rc;
    // a hazard: the call to the host for the exact engine, its results back
    std::vector<tb_transfer_t> ev(n);
    std::vector<uint32_t> ends(n_batches), lens(n_batches);
    std::vector<uint64_t> bts(n_batches);
    std::vector<tb_create_result_t> res(n);
    if (hipMemcpy(ev.data(), d_events, size_t(n) * 128, hipMemcpyDeviceToHost) ||
        hipMemcpy(ends.data(), d_batch_ends, size_t(n_batches) * 4, hipMemcpyDeviceToHost) ||
        hipMemcpy(bts.data(), d_batch_timestamps, size_t(n_batches) * 8, hipMemcpyDeviceToHost))
        return fail(g, TBG_EHIP, "download");
    for (uint32_t b = 0; b < n_batches; b++) lens[b] = ends[b] - (b ? ends[b - 1] : 0);
    const int erc = engine_call(g, tbs::kTransfers, ev.data(), n, lens.data(), bts.data(),
                                n_batches, res.data());
    if (erc) return erc;
    if (hipMemcpy(d_results, res.data(), size_t(n) * 16, hipMemcpyHostToDevice))
        return fail(g, TBG_EHIP, "upload");
    return 0;
}

int64_t tbg_group_pulse(tbg_group* g, uint64_t timestamp) {
    if (!g) return TBG_EINVAL;
    if (g->o.shards == 1) {
        if (g->gpu) return tbg_pulse(static_cast<tbg_ctx*>(g->shards[0]), timestamp);
    }
    try {
        return g->eng->pulse(timestamp, g->o.pulse_batch_max);
    } catch (const tbs::EngineError& e) {
        return fail(g, e.code, e.what());
    }
}

uint64_t tbg_group_pulse_next_timestamp(tbg_group* g) {
    if (!g) return 0;
    return g->eng->pulse_next_timestamp();
}

int64_t tbg_group_lookup_accounts(tbg_group* g, const tb_uint128_t* ids, uint32_t n,
                                  tb_account_t* out) {
    if (!g || (n && (!ids || !out))) return TBG_EINVAL;
    return lookup_all<tb_account_t>(g, ids, n, out, g->ops.lookup_accounts);
}

int64_t tbg_group_lookup_transfers(tbg_group* g, const tb_uint128_t* ids, uint32_t n,
                                   tb_transfer_t* out) {
    if (!g || (n && (!ids || !out))) return TBG_EINVAL;
    return lookup_all<tb_transfer_t>(g, ids, n, out, g->ops.lookup_transfers);
}

void tbg_group_executor(tbg_group* g, tb_executor* ex) {
    if (!ex) return;
    ex->self = g;
    ex->create_accounts = gx_create_accounts;
    ex->create_transfers = gx_create_transfers;
    ex->pulse = gx_pulse;
    ex->pulse_next_timestamp = gx_pulse_next;
    ex->lookup_accounts = gx_lookup_accounts;
    ex->lookup_transfers = gx_lookup_transfers;
    ex->get_change_events = gx_change_events;
    ex->get_account_transfers = gx_account_transfers;
    ex->get_account_balances = gx_account_balances;
    ex->query_accounts = gx_query_accounts;
    ex->query_transfers = gx_query_transfers;
}

int tbg_group_stats_read(tbg_group* g, tbg_group_stats* out) {
    if (!g || !out) return TBG_EINVAL;
    *out = g->st;
    return 0;
}

int64_t tbg_group_plan(tbg_group* g, int transfers, const void* events, uint32_t n,
                       const uint32_t* batch_lens, const uint64_t* batch_timestamps,
                       uint32_t n_batches, uint32_t* seg_ends, uint8_t* seg_flags,
                       int32_t* shard_of, uint32_t max_segments) {
    if (!g || (n && !events)) return TBG_EINVAL;
    try {
        std::vector<tbs::Engine::PlannedSeg> segs;
        std::vector<int32_t> place;
        g->eng->plan_only(transfers ? tbs::kTransfers : tbs::kAccounts,
                          static_cast<const uint8_t*>(events), n, batch_lens, batch_timestamps,
                          n_batches, segs, place);
        const size_t m = std::min<size_t>(segs.size(), max_segments);
        for (size_t i = 0; i < m; i++) {
            if (seg_ends) seg_ends[i] = segs[i].end;
            if (seg_flags) seg_flags[i] = segs[i].chain ? 1 : 0;
        }
        if (shard_of) std::copy(place.begin(), place.end(), shard_of);
        return int64_t(segs.size());
    } catch (const tbs::EngineError& e) {
        return fail(g, e.code, e.what());
    }
}

int tbg_group_record_accounts(tbg_group* g, const tb_uint128_t* ids, const uint8_t* shards,
                              uint32_t n) {
    if (!g || (n && (!ids || !shards))) return TBG_EINVAL;
    try {
        std::vector<u128> v(n);
        for (uint32_t i = 0; i < n; i++) v[i] = tbs::U(ids[i]);
        g->dir->record_accounts(v, std::vector<uint8_t>(shards, shards + n));
    } catch (const tbs::EngineError& e) {
        return fail(g, e.code, e.what());
    }
    return 0;
}

int tbg_group_record_transfers(tbg_group* g, const tb_uint128_t* ids, const uint8_t* shards,
                               uint32_t n) {
    if (!g || (n && (!ids || !shards))) return TBG_EINVAL;
    try {
        std::vector<u128> v(n);
        for (uint32_t i = 0; i < n; i++) v[i] = tbs::U(ids[i]);
        g->dir->record_transfers(v, std::vector<uint8_t>(shards, shards + n));
    } catch (const tbs::EngineError& e) {
        return fail(g, e.code, e.what());
    }
    return 0;
}

}  // extern "C"
