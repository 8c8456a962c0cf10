// The exact engine (engine.hpp): placement, segments, the chain protocol across shards, imported
// events across shards, pulse_next_timestamp across shards. Reference: src/state_machine.zig
// execute_create :3002-3213 (chains, imported batches, transient_error :3215-3252),
// create_transfer :3719-3986, post_or_void_pending_transfer :4053-4299, create_account :3613-3703.
#include "engine.hpp"

#include <map>

namespace tbs {

namespace {

inline bool transient(uint32_t st) { return tb_transfer_status_transient(st) != 0; }

inline void set_u16(uint8_t* e, int off, uint16_t v) { memcpy(e + off, &v, 2); }
inline void set_u64(uint8_t* e, int off, uint64_t v) { memcpy(e + off, &v, 8); }

}  // namespace

void Engine::fail(int rc, const char* what) const {
    throw EngineError(rc < 0 ? rc : TBG_EHIP, std::string(what) + " failed (" +
                                                   std::to_string(rc) + ")");
}

void Engine::make_call(Call& c, Kind kind, const uint8_t* events, uint32_t n,
                       const uint32_t* lens, const uint64_t* bts, uint32_t nb) {
    const KindInfo& K = kKinds[kind];
    c.kind = kind;
    c.is_tr = kind == kTransfers;
    c.n = n;
    c.nb = nb;
    c.ev = events;
    uint64_t sum = 0;
    for (uint32_t b = 0; b < nb; b++) sum += lens[b];
    if (sum != n) throw EngineError(TBG_EINVAL, "batch lengths do not cover the events");
    c.batch_start.resize(nb);
    c.batch_end.resize(nb);
    c.batch_ts.assign(bts, bts + nb);
    c.g_batch.assign(nb, 0);
    c.b_of.resize(n);
    c.stamp.resize(n);
    c.ts.resize(n);
    c.flags.resize(n);
    c.G.resize(n);
    c.open_last.resize(n);
    c.imp_live.resize(n);
    c.pre.assign(n, -1);
    c.ids.resize(n);
    c.potential.resize(n);
    c.chain_end.assign(n, 0);
    if (c.is_tr) {
        c.drs.resize(n);
        c.crs.resize(n);
        c.pids.resize(n);
    }
    std::vector<uint8_t> start(n, 0);
    uint32_t off = 0;
    for (uint32_t b = 0; b < nb; b++) {
        c.batch_start[b] = off;
        c.batch_end[b] = off + lens[b];
        if (lens[b]) {
            c.g_batch[b] = (ev_flags(events + uint64_t(off) * 128) & K.imported_flag) != 0;
            start[off] = 1;
        }
        for (uint32_t k = off; k < off + lens[b]; k++) {
            const uint8_t* e = events + uint64_t(k) * 128;
            const uint32_t within = k - off;
            const uint16_t f = ev_flags(e);
            const bool linked = f & 1, last = within == lens[b] - 1;
            const bool imp = (f & K.imported_flag) != 0;
            c.b_of[k] = b;
            c.stamp[k] = bts[b] - lens[b] + within + 1;
            c.flags[k] = f;
            c.ts[k] = ev_timestamp(e);
            c.G[k] = c.g_batch[b];
            c.open_last[k] = linked && last;
            if (imp != bool(c.G[k]) && !(linked && last))
                c.pre[k] = int32_t(imp ? K.not_expected : K.expected);
            c.imp_live[k] = imp && c.G[k] && c.ts[k] >= TB_TIMESTAMP_MIN &&
                            c.ts[k] <= TB_TIMESTAMP_MAX && c.ts[k] < bts[b];
            c.ids[k] = ev_u128(e, 0);
            if (c.is_tr) {
                c.drs[k] = ev_u128(e, 16);
                c.crs[k] = ev_u128(e, 32);
                c.pids[k] = ev_u128(e, 64);
            }
            c.potential[k] = c.imp_live[k] ? int64_t(c.ts[k]) : (imp ? -1 : int64_t(c.stamp[k]));
            if (k > 0 && !(c.flags[k - 1] & 1)) start[k] = 1;
        }
        off += lens[b];
    }
    if (n) start[0] = 1;
    uint32_t next = n;
    for (uint32_t k = n; k-- > 0;) {
        if (start[k]) {
            c.chain_end[k] = next;
            next = k;
        }
    }
}

void Engine::known_for(const Call& c, Known& kn) {
    IdMap seen(c.n + 16);
    std::vector<u128> q;
    std::vector<int32_t> out;
    auto add = [&](u128 id) {
        if (seen.insert(id, 0)) q.push_back(id);
    };
    if (c.is_tr) {
        for (uint32_t k = 0; k < c.n; k++) {
            add(c.ids[k]);
            add(c.pids[k]);
        }
        dir_->transfer_shards(q, out);
        for (size_t i = 0; i < q.size(); i++)
            if (out[i] >= 0) kn.transfers.set(q[i], out[i]);
        seen.clear();
        q.clear();
        for (uint32_t k = 0; k < c.n; k++) {
            add(c.drs[k]);
            add(c.crs[k]);
        }
    } else {
        for (uint32_t k = 0; k < c.n; k++) add(c.ids[k]);
    }
    dir_->account_shards(q, out);
    for (size_t i = 0; i < q.size(); i++)
        if (out[i] >= 0) kn.accounts.set(q[i], out[i]);
}

void Engine::collisions_for(const Call& c) {
    coll_.clear();
    std::vector<uint64_t> ts;
    for (uint32_t k = 0; k < c.n; k++)
        if (c.imp_live[k]) ts.push_back(c.ts[k]);
    if (ts.empty()) return;
    std::sort(ts.begin(), ts.end());
    ts.erase(std::unique(ts.begin(), ts.end()), ts.end());
    std::vector<uint64_t> mask(ts.size(), 0);
    std::vector<uint8_t> found(ts.size());
    for (uint32_t s = 0; s < W; s++) {
        // imported accounts collide with the transfers groove's timestamps and vice versa
        // (indirect_lookup, :3661-3665, :3813-3817)
        const int64_t rc = ops_->timestamps_exist(self_[s], c.is_tr ? 0 : 1, ts.data(),
                                                  uint32_t(ts.size()), found.data());
        if (rc < 0) fail(int(rc), "timestamps_exist");
        for (size_t i = 0; i < ts.size(); i++)
            if (found[i]) mask[i] |= 1ull << s;
    }
    for (size_t i = 0; i < ts.size(); i++)
        if (mask[i]) coll_.emplace_back(ts[i], mask[i]);
}

void Engine::reset_call_arrays(uint32_t n) {
    place_.assign(n, kNone);
    tprime_.assign(n, -1);
    tprime_ts_.assign(n, 0);
    cross_.assign(n, 0);
    decided_.assign(n, 0);
    patch_expect_.assign(n, 0);
    patch_status_.assign(n, 0);
}

// Where transfer k runs by what it names (not its own id): a shard, kNone (anywhere), or kCross
// (two accounts on two shards).
int32_t Engine::natural_transfer(const Call& c, const Known& kn, uint32_t k,
                                 const IdMap& chain_first, const IdMap& seg_ids) const {
    if (c.flags[k] & kPostVoid) {
        const u128 p = c.pids[k];
        if (const int32_t* v = kn.transfers.find(p)) return *v;
        if (const int32_t* v = chain_first.find(p)) return *v;
        if (const int32_t* v = seg_ids.find(p)) return *v;
        return kNone;
    }
    const int32_t* dr = kn.accounts.find(c.drs[k]);
    const int32_t* cr = kn.accounts.find(c.crs[k]);
    if (dr && cr && *dr != *cr) return kCross;
    return dr ? *dr : (cr ? *cr : kNone);
}

namespace {
thread_local IdMap tl_chain_first(64), tl_seen(64);
}

// Places the chain [a, z): every event pinned by its id's holder, by the first occurrence of its
// id in the chain, or by what it names; unpinned events (inert ones, surrogates, events found
// nowhere) run with their neighbours. false: an id of an earlier chain of the segment that would
// run elsewhere (the segment ends before this chain).
bool Engine::place_chain(const Call& c, const Known& kn, uint32_t a, uint32_t z,
                         const IdMap& seg_ids, uint64_t* shard_mask) {
    IdMap& chain_first = tl_chain_first;
    chain_first.clear();
    const IdMap& holders = c.is_tr ? kn.transfers : kn.accounts;
    uint64_t mask = 0;
    for (uint32_t k = a; k < z; k++) {
        cross_[k] = 0;
        int32_t s = kNone;
        if (c.pre[k] < 0) {
            const u128 i = c.ids[k];
            if (const int32_t* h = holders.find(i)) {
                s = *h;
            } else if (const int32_t* f = chain_first.find(i)) {
                s = *f;  // the chain reaches it only if the first occurrence created the id
            } else {
                const uint8_t* e = c.ev + uint64_t(k) * 128;
                const int32_t nat = c.is_tr ? natural_transfer(c, kn, k, chain_first, seg_ids)
                                            : int32_t(shard_of_ledger(ev_ledger(e)));
                if (const int32_t* si = seg_ids.find(i)) {
                    if (nat == kNone || nat == *si)
                        s = *si;
                    else
                        return false;
                } else if (nat == kCross) {
                    cross_[k] = cross_status(c.pids[k], c.flags[k], ev_u32(e, 108), ev_ledger(e),
                                             ev_code(e));
                } else {
                    s = nat;
                }
            }
            if (s != kNone && i != 0 && i != kU128Max && !holders.has(i)) chain_first.insert(i, s);
        }
        place_[k] = s;
        if (s != kNone) mask |= 1ull << s;
    }
    if (!mask) mask = 1ull << shard_of_ledger(ev_ledger(c.ev + uint64_t(a) * 128));
    int32_t last = __builtin_ctzll(mask);
    for (uint32_t k = a; k < z; k++) {
        if (place_[k] == kNone)
            place_[k] = last;
        else
            last = place_[k];
    }
    *shard_mask = mask;
    return true;
}

// Imported events whose must_not_regress checks read another shard: a transfer runs with a
// timestamp surrogate, an account gets the engine's status. false: the chain must start a new
// segment instead.
bool Engine::imported_decisions(const Call& c, const Known& kn, uint32_t a, uint32_t z, bool multi,
                                const IdMap& seg_ids) {
    std::vector<int64_t> chain_max(W, -1);  // shard -> largest imported timestamp created so far
    const IdMap& holders = c.is_tr ? kn.transfers : kn.accounts;
    IdMap& seen = tl_seen;
    seen.clear();
    for (uint32_t k = a; k < z; k++) {
        if (c.pre[k] >= 0 || !c.imp_live[k] || cross_[k]) continue;
        const int32_t s = place_[k];
        const uint64_t t = c.ts[k];
        const uint64_t cm = coll_of(t);
        bool hazard = cm != 0 && !((cm >> s) & 1);
        if (multi)
            for (uint32_t o = 0; o < W; o++)
                if (int32_t(o) != s && chain_max[o] >= int64_t(t)) hazard = true;
        if (hazard) {
            const u128 i = c.ids[k];
            if (c.is_tr) {
                tprime_[k] = s;
            } else if (holders.has(i) || seen.has(i)) {
                // create_account_exists decides it first (:3629), on the holder
            } else if (seg_ids.has(i)) {
                return false;  // (whether it exists is known once the segment has run)
            } else {
                const uint32_t st = account_static_status(c.ev + uint64_t(k) * 128);
                decided_[k] = st ? st : kKinds[c.kind].regress;
            }
        }
        chain_max[s] = std::max<int64_t>(std::max<int64_t>(chain_max[s], 0), int64_t(t));
        seen.insert(c.ids[k], 0);
    }
    return true;
}

Engine::Seg Engine::plan(const Call& c, const Known& kn, uint32_t start) {
    static thread_local IdMap seg_ids(1024);
    seg_ids.clear();
    Seg seg;
    seg.start = start;
    std::vector<int64_t> seg_pot(W, -1);
    uint32_t a = start;
    while (a < c.n) {
        const uint32_t z = c.chain_end[a];
        uint64_t mask = 0;
        if (!place_chain(c, kn, a, z, seg_ids, &mask)) break;
        for (uint32_t k = a; k < z; k++) {
            decided_[k] = 0;
            tprime_[k] = -1;
        }
        const bool multi = __builtin_popcountll(mask) > 1;
        if (multi && a > start) break;
        if (!imported_decisions(c, kn, a, z, multi, seg_ids)) break;
        if (a > start) {  // regress across shards within the segment
            bool cut = false;
            for (uint32_t k = a; k < z && !cut; k++) {
                if (!c.imp_live[k] || c.pre[k] >= 0 || decided_[k]) continue;
                const int32_t s = place_[k];
                for (uint32_t o = 0; o < W; o++)
                    if (int32_t(o) != s && seg_pot[o] >= int64_t(c.ts[k])) cut = true;
            }
            if (cut) break;
        }
        for (uint32_t k = a; k < z; k++) {
            if (tprime_[k] >= 0) seg.tprime = true;
            if (c.pre[k] >= 0 || cross_[k] || decided_[k] || tprime_[k] >= 0) continue;
            const u128 i = c.ids[k];
            if (i != 0 && i != kU128Max) seg_ids.insert(i, place_[k]);
            const int32_t s = place_[k];
            seg_pot[s] = std::max(seg_pot[s], c.potential[k]);
            if (c.imp_live[k]) seg.imported = true;
            if (c.is_tr && (c.flags[k] & kPostVoid)) seg.post_void = true;
        }
        a = z;
        if (multi) {
            seg.chain = true;
            break;
        }
    }
    seg.end = a;
    if (seg.end == start) throw EngineError(TBG_EHIP, "empty segment");  // (a first chain fits)
    return seg;
}

// The segment's events as their shards run them (inert events, surrogates, timestamp surrogates)
// and the result patches: event k's status becomes patch_status_[k] when the shard reports
// patch_expect_[k].
std::vector<uint8_t> Engine::exec_events(const Call& c, const Seg& seg, uint32_t a, uint32_t z) {
    const KindInfo& K = kKinds[c.kind];
    std::vector<uint8_t> ev(c.ev + uint64_t(a) * 128, c.ev + uint64_t(z) * 128);
    for (uint32_t k = a; k < z; k++) {
        uint8_t* e = ev.data() + uint64_t(k - a) * 128;
        patch_status_[k] = 0;
        const bool g = c.G[k];
        if (c.pre[k] >= 0 || decided_[k]) {
            memset(e, 0, 128);
            set_u16(e, 118, uint16_t((g ? K.imported_flag : 0) | (c.flags[k] & 1)));
            patch_expect_[k] = g ? K.inert_imported : K.inert_plain;
            patch_status_[k] = c.pre[k] >= 0 ? uint32_t(c.pre[k]) : decided_[k];
        } else if (cross_[k]) {
            memcpy(e + 32, e + 16, 16);  // credit_account_id := debit_account_id
            patch_expect_[k] = TB_CT_ACCOUNTS_MUST_BE_DIFFERENT;
            patch_status_[k] = cross_[k];
        }
    }
    if (seg.tprime) {
        tprime_values(c, seg);
        for (uint32_t k = a; k < z; k++)
            if (tprime_[k] >= 0) set_u64(ev.data() + uint64_t(k - a) * 128, 120, tprime_ts_[k]);
    }
    return ev;
}

// A timestamp that fails must_not_regress on the event's shard once the event reaches the
// imported checks: its debit account's (a post/void's: its pending transfer's), found in the
// shard's accounts by timestamp (:3813-3817); 1 when that account is not on the shard (the event
// fails before the imported checks).
void Engine::tprime_values(const Call& c, const Seg& seg) {
    std::vector<std::vector<u128>> need_acc(W), need_pend(W);
    for (uint32_t k = seg.start; k < seg.end; k++) {
        const int32_t s = tprime_[k];
        if (s < 0) continue;
        if (c.flags[k] & kPostVoid)
            need_pend[s].push_back(c.pids[k]);
        else
            need_acc[s].push_back(c.drs[k]);
    }
    std::map<std::pair<int32_t, u128>, u128> pend_dr;
    std::map<std::pair<int32_t, u128>, uint64_t> acc_ts;
    for (uint32_t s = 0; s < W; s++) {
        auto& ids = need_pend[s];
        if (ids.empty()) continue;
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
        std::vector<tb_uint128_t> q(ids.size());
        for (size_t i = 0; i < ids.size(); i++) q[i] = T128(ids[i]);
        std::vector<tb_transfer_t> rows(ids.size());
        const int64_t m = ops_->lookup_transfers(self_[s], q.data(), uint32_t(q.size()), rows.data());
        if (m < 0) fail(int(m), "lookup_transfers");
        for (int64_t j = 0; j < m; j++) {
            const u128 dr = U(rows[j].debit_account_id);
            pend_dr[{int32_t(s), U(rows[j].id)}] = dr;
            need_acc[s].push_back(dr);
        }
    }
    for (uint32_t s = 0; s < W; s++) {
        auto& ids = need_acc[s];
        if (ids.empty()) continue;
        std::sort(ids.begin(), ids.end());
        ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
        std::vector<tb_uint128_t> q(ids.size());
        for (size_t i = 0; i < ids.size(); i++) q[i] = T128(ids[i]);
        std::vector<tb_account_t> rows(ids.size());
        const int64_t m = ops_->lookup_accounts(self_[s], q.data(), uint32_t(q.size()), rows.data());
        if (m < 0) fail(int(m), "lookup_accounts");
        for (int64_t j = 0; j < m; j++) acc_ts[{int32_t(s), U(rows[j].id)}] = rows[j].timestamp;
    }
    for (uint32_t k = seg.start; k < seg.end; k++) {
        const int32_t s = tprime_[k];
        if (s < 0) continue;
        uint64_t v = 1;
        bool have = true;
        u128 dr = c.drs[k];
        if (c.flags[k] & kPostVoid) {
            auto it = pend_dr.find({s, c.pids[k]});
            have = it != pend_dr.end();
            if (have) dr = it->second;
        }
        if (have) {
            auto it = acc_ts.find({s, dr});
            if (it != acc_ts.end()) v = it->second;
        }
        tprime_ts_[k] = v;
    }
}

void Engine::execute(Kind kind, std::vector<ShardRun>& runs) {
    std::vector<int> shards;
    for (uint32_t s = 0; s < W; s++)
        if (!runs[s].calls.empty() || kind == kTransfers) shards.push_back(int(s));
    std::vector<int> rcs;
    runner_->run(shards, [&](int s) -> int {
        ShardRun& r = runs[s];
        void* self = self_[s];
        bool have_start = false;
        r.pnt.clear();
        for (SubCall& sc : r.calls) {
            const uint32_t n = sc.n();
            sc.out.assign(n, tb_create_result_t{0, 0, 0});
            int rc;
            if (sc.stamped) {
                const uint32_t opt = sc.one_chain ? TBG_ONE_CHAIN : 0u;
                rc = kind == kTransfers
                         ? ops_->create_transfers_stamped(
                               self, reinterpret_cast<const tb_transfer_t*>(sc.ev.data()), n,
                               sc.ts.data(), sc.batch_ts, opt, sc.out.data())
                         : ops_->create_accounts_stamped(
                               self, reinterpret_cast<const tb_account_t*>(sc.ev.data()), n,
                               sc.ts.data(), sc.batch_ts, opt, sc.out.data());
            } else {
                rc = kind == kTransfers
                         ? ops_->create_transfers(
                               self, reinterpret_cast<const tb_transfer_t*>(sc.ev.data()), n,
                               sc.lens.data(), sc.ts.data(), uint32_t(sc.lens.size()),
                               sc.out.data())
                         : ops_->create_accounts(
                               self, reinterpret_cast<const tb_account_t*>(sc.ev.data()), n,
                               sc.lens.data(), sc.ts.data(), uint32_t(sc.lens.size()),
                               sc.out.data());
            }
            if (rc != 0) return rc;
            if (kind == kTransfers) {
                uint64_t start = 0;
                const int64_t m = ops_->pnt_ops(self, nullptr, nullptr, 0, &start);
                if (m < 0) return int(m);
                std::vector<uint64_t> t(size_t(m) + 1), o(size_t(m) + 1);
                if (m > 0) {
                    uint64_t start2 = 0;
                    const int64_t m2 = ops_->pnt_ops(self, t.data(), o.data(), uint64_t(m), &start2);
                    if (m2 != m) return m2 < 0 ? int(m2) : TBG_EHIP;
                }
                if (!have_start) {
                    r.pnt_start = start;
                    have_start = true;
                }
                for (int64_t j = 0; j < m; j++) r.pnt.emplace_back(t[j], o[j]);
            }
        }
        if (kind == kTransfers && !have_start) r.pnt_start = ops_->pulse_next_timestamp(self);
        return 0;
    }, rcs);
    for (size_t i = 0; i < rcs.size(); i++)
        if (rcs[i] != 0)
            throw EngineError(rcs[i] < 0 ? rcs[i] : TBG_EHIP,
                              "shard " + std::to_string(shards[i]) + " failed (" +
                                  std::to_string(rcs[i]) + "); the shards' state is undefined");
}

std::vector<uint64_t> Engine::pnt_values() {
    std::vector<uint64_t> v(W);
    for (uint32_t s = 0; s < W; s++) v[s] = ops_->pulse_next_timestamp(self_[s]);
    return v;
}

void Engine::set_pnt(const std::vector<uint64_t>& values) {
    for (uint32_t s = 0; s < W; s++) {
        const int rc = ops_->set_pulse_next_timestamp(self_[s], values[s]);
        if (rc != 0) fail(rc, "set_pulse_next_timestamp");
    }
}

std::pair<uint64_t, uint64_t> Engine::sync_key_max() {
    uint64_t a = 0, t = 0;
    for (uint32_t s = 0; s < W; s++) {
        uint64_t x = 0, y = 0;
        const int rc = ops_->key_max(self_[s], &x, &y);
        if (rc != 0) fail(rc, "key_max");
        a = std::max(a, x);
        t = std::max(t, y);
    }
    for (uint32_t s = 0; s < W; s++) {
        const int rc = ops_->raise_key_max(self_[s], a, t);
        if (rc != 0) fail(rc, "raise_key_max");
    }
    return {a, t};
}

uint64_t Engine::pulse_next_timestamp() {
    uint64_t v = ~0ull;
    for (uint32_t s = 0; s < W; s++) v = std::min(v, ops_->pulse_next_timestamp(self_[s]));
    return v;
}

int64_t Engine::pulse(uint64_t timestamp, uint32_t pbm) {
    std::vector<uint64_t> counts(W);
    std::vector<std::vector<std::pair<uint64_t, uint64_t>>> keys(W);
    std::vector<uint64_t> e(std::max<uint32_t>(pbm, 1)), t(std::max<uint32_t>(pbm, 1));
    for (uint32_t s = 0; s < W; s++) {
        const int64_t m = ops_->pulse_candidates(self_[s], timestamp, e.data(), t.data(), pbm);
        if (m < 0) fail(int(m), "pulse_candidates");
        counts[s] = uint64_t(m);
        const uint64_t kk = std::min<uint64_t>(uint64_t(m), pbm);
        for (uint64_t j = 0; j < kk; j++) keys[s].emplace_back(e[j], t[j]);
    }
    const PulsePlan p = pulse_plan(counts, keys, pbm, timestamp);
    int64_t total = 0;
    for (uint32_t s = 0; s < W; s++) {
        const int64_t m = ops_->pulse_cut(self_[s], timestamp, p.cut_e, p.cut_t, p.pnt,
                                          p.stamps[s].empty() ? nullptr : p.stamps[s].data());
        if (m < 0) fail(int(m), "pulse_cut");
        total += m;
    }
    return total;
}

void Engine::run_segment(const Call& c, const Seg& seg, tb_create_result_t* results) {
    std::vector<ShardRun> runs(W);
    const std::vector<uint8_t> ev_all = exec_events(c, seg, seg.start, seg.end);
    const uint32_t off = seg.start;
    std::vector<SubCall> open(W);
    std::vector<uint8_t> is_open(W, 0);
    auto flush = [&](uint32_t s) {
        if (is_open[s]) {
            runs[s].calls.push_back(std::move(open[s]));
            open[s] = SubCall();
            is_open[s] = 0;
        }
    };
    auto append = [&](SubCall& sc, uint32_t k) {
        sc.pos.push_back(k);
        const uint8_t* e = ev_all.data() + uint64_t(k - off) * 128;
        sc.ev.insert(sc.ev.end(), e, e + 128);
    };
    std::vector<std::vector<uint32_t>> per(W);
    for (uint32_t b = c.b_of[seg.start]; b < c.nb && c.batch_start[b] < seg.end; b++) {
        const uint32_t lo = std::max(seg.start, c.batch_start[b]);
        const uint32_t hi = std::min(seg.end, c.batch_end[b]);
        if (lo >= hi) continue;
        if (c.g_batch[b]) {
            // an imported batch: one stamped batch per shard (the batch's timestamp is imported
            // events' must_not_advance bound, :3073)
            for (auto& p : per) p.clear();
            for (uint32_t k = lo; k < hi; k++) per[place_[k]].push_back(k);
            for (uint32_t s = 0; s < W; s++) {
                if (per[s].empty()) continue;
                flush(s);
                SubCall sc;
                sc.stamped = true;
                sc.batch_ts = c.batch_ts[b];
                for (uint32_t k : per[s]) {
                    append(sc, k);
                    sc.ts.push_back(c.stamp[k]);
                }
                runs[s].calls.push_back(std::move(sc));
            }
        } else {
            // maximal runs of consecutive positions, each a sub-batch stamped by its last event
            uint32_t k = lo;
            while (k < hi) {
                const uint32_t s = uint32_t(place_[k]);
                uint32_t j = k;
                while (j < hi && place_[j] == int32_t(s)) j++;
                if (is_open[s] && open[s].lens.size() >= max_batches_) flush(s);
                is_open[s] = 1;
                for (uint32_t x = k; x < j; x++) append(open[s], x);
                open[s].lens.push_back(j - k);
                open[s].ts.push_back(c.stamp[j - 1]);
                k = j;
            }
        }
    }
    for (uint32_t s = 0; s < W; s++) flush(s);
    if (seg.imported) sync_key_max();
    execute(c.kind, runs);
    for (uint32_t s = 0; s < W; s++)
        for (const SubCall& sc : runs[s].calls)
            for (size_t i = 0; i < sc.pos.size(); i++) results[sc.pos[i]] = sc.out[i];
    for (uint32_t k = seg.start; k < seg.end; k++) patch(results, k);
    if (c.is_tr && seg.post_void) {
        std::vector<uint64_t> starts(W);
        std::vector<PntOps> ops(W);
        for (uint32_t s = 0; s < W; s++) {
            starts[s] = runs[s].pnt_start;
            ops[s] = runs[s].pnt;
        }
        if (pnt_resets_fire(starts, ops)) set_pnt(std::vector<uint64_t>(W, TB_TIMESTAMP_MIN));
    }
}

// One linked chain across shards (:3033-3207). Every shard probes its part without the chain's
// last event -- one chain (TBG_ONE_CHAIN) ending in an inert sentinel, so it always rolls back and
// reports its first failure. No failure before the last event: the last event's shard commits its
// part with it -- the chain's outcome; if that succeeds, every other shard commits its part (the
// state its probe saw: it succeeds). A failure: the reference executed (and rolled back) the
// events before it; the probes' orphans past it are forgotten and pulse_next_timestamp is set
// back to the shards' values before the probe lowered by the pending transfers the reference did
// execute (:3975-3982 are not undone by a discard).
void Engine::run_chain(const Call& c, const Seg& seg, tb_create_result_t* results) {
    const KindInfo& K = kKinds[c.kind];
    const uint32_t a = seg.start, z = seg.end, last = z - 1;
    const bool open_ = c.open_last[last];
    const uint32_t b = c.b_of[a];
    const uint64_t T_b = c.batch_ts[b];
    const bool g = c.g_batch[b];
    const uint32_t s_last = uint32_t(place_[last]);
    std::vector<std::vector<uint32_t>> parts(W);
    for (uint32_t k = a; k < last; k++) parts[place_[k]].push_back(k);
    const std::vector<uint8_t> ev_all = exec_events(c, seg, a, z);

    auto part_call = [&](const std::vector<uint32_t>& ks, bool sentinel) {
        SubCall sc;
        sc.stamped = true;
        sc.one_chain = true;
        sc.batch_ts = T_b;
        for (uint32_t k : ks) {
            sc.pos.push_back(k);
            const uint8_t* e = ev_all.data() + uint64_t(k - a) * 128;
            sc.ev.insert(sc.ev.end(), e, e + 128);
            sc.ts.push_back(c.stamp[k]);
        }
        if (sentinel) {
            uint8_t inert[128];
            memset(inert, 0, sizeof inert);
            set_u16(inert, 118, uint16_t(g ? K.imported_flag : 0));
            sc.ev.insert(sc.ev.end(), inert, inert + 128);
            sc.ts.push_back(sc.ts.back() + 1);
        }
        return sc;
    };

    if (seg.imported) sync_key_max();
    std::vector<uint64_t> saved;
    if (c.is_tr) saved = pnt_values();
    std::vector<ShardRun> probe(W);
    for (uint32_t s = 0; s < W; s++)
        if (!parts[s].empty()) probe[s].calls.push_back(part_call(parts[s], true));
    execute(c.kind, probe);
    std::vector<int64_t> first(W, -1);  // shard -> its part's first failing event
    int64_t fail_at = -1;
    for (uint32_t s = 0; s < W; s++) {
        if (parts[s].empty()) continue;
        const std::vector<tb_create_result_t>& r = probe[s].calls[0].out;
        for (size_t j = 0; j < parts[s].size(); j++) results[parts[s][j]] = r[j];
        for (size_t j = 0; j < parts[s].size(); j++)
            if (r[j].status != kLinkedEventFailed) {
                first[s] = parts[s][j];
                break;
            }
        if (first[s] >= 0 && (fail_at < 0 || first[s] < fail_at)) fail_at = first[s];
    }
    if (fail_at < 0 && open_) fail_at = last;  // linked_event_chain_open (:3039-3042)
    if (fail_at < 0) {
        // the last event decides: its shard commits its part with it
        std::vector<uint32_t> ks = parts[s_last];
        ks.push_back(last);
        std::vector<ShardRun> commit(W);
        commit[s_last].calls.push_back(part_call(ks, false));
        execute(c.kind, commit);
        const std::vector<tb_create_result_t>& r = commit[s_last].calls[0].out;
        for (size_t j = 0; j < ks.size(); j++) results[ks[j]] = r[j];
        std::vector<PntOps> ops_lists(W);
        if (c.is_tr) {
            for (uint32_t s = 0; s < W; s++) ops_lists[s] = probe[s].pnt;
            ops_lists[s_last] = commit[s_last].pnt;
        }
        if (results[last].status == TB_STATUS_CREATED) {
            std::vector<ShardRun> rest(W);
            bool any = false;
            for (uint32_t s = 0; s < W; s++)
                if (!parts[s].empty() && s != s_last) {
                    rest[s].calls.push_back(part_call(parts[s], false));
                    any = true;
                }
            if (any) {
                execute(c.kind, rest);
                for (uint32_t s = 0; s < W; s++) {
                    if (rest[s].calls.empty()) continue;
                    const std::vector<tb_create_result_t>& r2 = rest[s].calls[0].out;
                    for (size_t j = 0; j < parts[s].size(); j++) results[parts[s][j]] = r2[j];
                    if (c.is_tr) ops_lists[s] = rest[s].pnt;
                }
            }
            for (uint32_t k = a; k < z; k++)
                if (results[k].status != TB_STATUS_CREATED)
                    throw EngineError(TBG_EHIP,
                                      "a linked chain across shards failed on its commit after its "
                                      "probe succeeded: the shards' state is undefined");
        } else {
            // failed at its last event: that shard rolled back (orphaning it if transient,
            // :3172); the other shards' probes already did
            patch(results, last);
        }
        if (c.is_tr && seg.post_void && pnt_resets_fire(saved, ops_lists))
            set_pnt(std::vector<uint64_t>(W, TB_TIMESTAMP_MIN));
        return;
    }
    // The chain fails at `fail_at`.
    for (uint32_t k = uint32_t(fail_at) + 1; k < z; k++) {
        results[k].timestamp = c.stamp[k];
        results[k].status = kLinkedEventFailed;
        results[k].reserved = 0;
    }
    if (open_) {
        results[last].timestamp = c.stamp[last];
        results[last].status = kLinkedEventChainOpen;
        results[last].reserved = 0;
    }
    for (uint32_t k = a; k <= uint32_t(fail_at); k++) patch(results, k);
    if (c.is_tr) {
        bool any = false;
        std::vector<std::vector<tb_uint128_t>> forget(W);
        for (uint32_t s = 0; s < W; s++) {
            const int64_t k = first[s];
            if (k < 0 || k == fail_at) continue;
            const auto& ps = parts[s];
            const size_t j = size_t(std::find(ps.begin(), ps.end(), uint32_t(k)) - ps.begin());
            if (transient(probe[s].calls[0].out[j].status)) {
                forget[s].push_back(T128(c.ids[k]));
                any = true;
            }
        }
        if (any)
            for (uint32_t s = 0; s < W; s++)
                if (!forget[s].empty()) {
                    const int64_t m = ops_->forget_orphans(self_[s], forget[s].data(),
                                                           uint32_t(forget[s].size()));
                    if (m < 0) fail(int(m), "forget_orphans");
                }
        // pulse_next_timestamp: the values before the probe, lowered by the updates of the events
        // the reference executed (those before the failure)
        const uint64_t cut = c.stamp[fail_at];
        std::vector<PntOps> kept(W);
        std::vector<uint64_t> values(W);
        for (uint32_t s = 0; s < W; s++) {
            uint64_t v = saved[s];
            for (const auto& e : probe[s].pnt)
                if (e.first < cut) {
                    kept[s].push_back(e);
                    if (!(e.second & kPntReset) && e.second < v) v = e.second;
                }
            values[s] = v;
        }
        if (pnt_resets_fire(saved, kept)) values.assign(W, TB_TIMESTAMP_MIN);
        set_pnt(values);
    }
}

// Records where the segment's new objects (and orphaned transfer ids) now live; a repeated id
// keeps its first holder.
void Engine::record(const Call& c, const Seg& seg, const tb_create_result_t* results, Known& kn) {
    IdMap& seen = tl_seen;
    seen.clear();
    std::vector<u128> ids;
    std::vector<uint8_t> sh;
    for (uint32_t k = seg.start; k < seg.end; k++) {
        const uint32_t st = results[k].status;
        const bool keep = st == TB_STATUS_CREATED || (c.is_tr && transient(st));
        if (keep && seen.insert(c.ids[k], 0)) {
            ids.push_back(c.ids[k]);
            sh.push_back(uint8_t(place_[k]));
        }
    }
    if (ids.empty()) return;
    if (c.is_tr) {
        dir_->record_transfers(ids, sh);
        for (size_t i = 0; i < ids.size(); i++) kn.transfers.insert(ids[i], sh[i]);
    } else {
        dir_->record_accounts(ids, sh);
        for (size_t i = 0; i < ids.size(); i++) kn.accounts.set(ids[i], sh[i]);
    }
}

void Engine::run(Kind kind, const uint8_t* events, uint32_t n, const uint32_t* lens,
                 const uint64_t* batch_ts, uint32_t nb, tb_create_result_t* results) {
    Call c;
    make_call(c, kind, events, n, lens, batch_ts, nb);
    memset(results, 0, sizeof(tb_create_result_t) * size_t(n));
    if (n == 0) return;
    reset_call_arrays(n);
    Known kn;
    known_for(c, kn);
    collisions_for(c);
    uint32_t pos = 0;
    while (pos < n) {
        const Seg seg = plan(c, kn, pos);
        if (seg.chain) {
            run_chain(c, seg, results);
            stats.chain_segments++;
        } else {
            run_segment(c, seg, results);
        }
        stats.segments++;
        record(c, seg, results, kn);
        pos = seg.end;
    }
}

void Engine::plan_only(Kind kind, const uint8_t* events, uint32_t n, const uint32_t* lens,
                       const uint64_t* batch_ts, uint32_t nb, std::vector<PlannedSeg>& segs,
                       std::vector<int32_t>& shard_of) {
    Call c;
    make_call(c, kind, events, n, lens, batch_ts, nb);
    segs.clear();
    shard_of.assign(n, -1);
    if (n == 0) return;
    reset_call_arrays(n);
    Known kn;
    known_for(c, kn);
    collisions_for(c);
    uint32_t pos = 0;
    while (pos < n) {
        const Seg seg = plan(c, kn, pos);
        segs.push_back(PlannedSeg{seg.end, seg.chain});
        for (uint32_t k = seg.start; k < seg.end; k++) shard_of[k] = place_[k];
        pos = seg.end;
    }
}

}  // namespace tbs
