"""HIP executor vs CPU oracle on seeded synthetic workloads (bit-exact results and state)."""
import numpy as np
import pytest

from parity import Pair
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import NS_PER_S, TIMESTAMP_MAX, TRANSFER_DTYPE

pytestmark = pytest.mark.gpu


def _split(n, rng, max_batch):
    lens = []
    while n > 0:
        b = int(min(n, rng.integers(1, max_batch + 1)))
        lens.append(b)
        n -= b
    return lens


@pytest.mark.parametrize("registered", [False, True], ids=["pageable", "registered"])
@pytest.mark.parametrize("force_replay", [False, True, "serial"], ids=["parallel", "flow", "serial"])
@pytest.mark.parametrize("seed", range(6))
def test_fuzz(seed, force_replay, registered):
    """Executor-level fuzzing against the oracle; `registered`: bodies and results in a registered
    host pool (the kernels read / write them over PCIe, the appends on the side stream)."""
    rng = np.random.default_rng(1000 + seed)
    p = Pair(account_capacity=1 << 12, transfer_capacity=1 << 15, batch_events_max=4096,
             pulse_batch_max=16, pulse_next_timestamp_init=TIMESTAMP_MAX,
             force_replay=force_replay, registered=registered)
    try:
        n_acc = 24
        a = workload.fuzz_accounts(rng, 40, n_acc)
        p.create_accounts(a, _split(len(a), rng, 12))
        # A clean set of accounts so that most transfers reach the deep checks.
        clean = workload.accounts(n_acc, seed=seed, id_offset=0, ledger=1)
        clean["flags"] = rng.choice([0, 0, 2, 4, 8], size=n_acc).astype(np.uint16)
        p.create_accounts(clean, _split(n_acc, rng, 8))
        ids_seen = []
        for step in range(8):
            pend = np.array(ids_seen[-200:], dtype=np.uint64) if ids_seen else None
            t = workload.fuzz_transfers(rng, 300, 400, n_acc + 1, pending_ids=pend)
            ids_seen.extend(int(x) for x in t["id"][:, 0])
            p.create_transfers(t, _split(len(t), rng, 64))
            if step % 3 == 2:
                p.tick(int(rng.integers(1, 3)) * NS_PER_S)
        p.compare_state()
        assert p.compare_scans(rng, n=60) > 0
    finally:
        p.close()


@pytest.mark.parametrize("seed", range(3))
def test_scans_at_scale(seed):
    """The scans (get_account_transfers / _balances, query_accounts / _transfers) over 12k accounts
    with history and 100k transfers -- pending, posted, voided and single-phase, user data drawn
    from small sets so that conditions intersect -- against the oracle, with the reply limit of
    production (8190 results) and the reference's test configuration (29)."""
    rng = np.random.default_rng(500 + seed)
    p = Pair(account_capacity=1 << 15, transfer_capacity=1 << 18, batch_events_max=1 << 15)
    try:
        n_acc = 12_000
        acc = workload.accounts(n_acc, seed=seed, ledger=1)
        acc["flags"] = rng.choice([0, 8], size=n_acc).astype(np.uint16)  # history on half
        acc["user_data_64"] = rng.integers(1, 20, size=n_acc).astype(np.uint64)
        acc["code"] = rng.integers(1, 5, size=n_acc).astype(np.uint16)
        acc["ledger"] = rng.integers(1, 3, size=n_acc).astype(np.uint32)
        p.create_accounts(acc, _split(n_acc, rng, 8189))
        # accounts of each ledger: transfers stay within one
        by_ledger = {lg: np.nonzero(acc["ledger"] == lg)[0] + 1 for lg in (1, 2)}
        for call in range(4):
            n = 25_000
            t = workload.transfers_uniform(n, 100, seed=seed * 10 + call, id_offset=call * n)
            lg = rng.integers(1, 3, size=n)
            for v in (1, 2):
                ids = by_ledger[v]
                m = lg == v
                dr = rng.choice(ids[:200], size=m.sum())
                cr = rng.choice(ids[:200], size=m.sum())
                cr = np.where(cr == dr, ids[200], cr)
                t["debit_account_id"][m, 0] = dr
                t["credit_account_id"][m, 0] = cr
            t["ledger"] = lg.astype(np.uint32)
            t["user_data_128"][:, 0] = rng.integers(1, 7, size=n).astype(np.uint64)
            t["user_data_128"][:, 1] = 0
            t["user_data_64"] = rng.integers(1, 11, size=n).astype(np.uint64)
            t["user_data_32"] = rng.integers(1, 4, size=n).astype(np.uint32)
            t["code"] = rng.integers(1, 9, size=n).astype(np.uint16)
            t["flags"] = np.where(rng.random(n) < 0.3, 2, 0).astype(np.uint16)  # pending
            p.create_transfers(t, _split(n, rng, 8189))
            if call:
                prev = np.arange((call - 1) * n, call * n, dtype=np.uint64) + 1
                pv = workload.transfers_uniform(4000, 100, seed=99 + call,
                                                id_offset=10_000_000 + call * 4000)
                pv["pending_id"][:, 0] = rng.choice(prev, size=4000, replace=False)
                pv["debit_account_id"] = 0
                pv["credit_account_id"] = 0
                pv["ledger"] = 0
                pv["code"] = 0
                pv["amount"] = 0
                pv["flags"] = rng.choice([4, 8], size=4000).astype(np.uint16)
                p.create_transfers(pv, _split(4000, rng, 8189))
        assert p.compare_scans(rng, n=60, limit_max=8190) > 1000
        assert p.compare_scans(rng, n=60, limit_max=29) > 0
    finally:
        p.close()


@pytest.mark.parametrize("amounts", ["exp", "wide"])
def test_uniform_config2_full_size(amounts):
    """BASELINE configs[1] at its own size against the oracle: 10k accounts, ONE call of 10M
    uniform create_transfers in 8189-event batches (the bench's step), every result, row and
    AccountEvent compared (Pair.compare_state). `wide`: amounts log-uniform over [1, 2^63) --
    beyond the packed balance items (tr_commit's atomics) and the one-pass AccountEvents."""
    n = 10_000_000
    p = Pair(account_capacity=1 << 14, transfer_capacity=n + (1 << 14), batch_events_max=n,
             batch_count_max=1 << 11)
    try:
        acc = workload.accounts(10_000, seed=42)
        r = p.create_accounts(acc, [8189, 10_000 - 8189])
        assert (r["status"] == 0xFFFFFFFF).all()
        t = workload.transfers_uniform(n, 10_000, seed=42, amounts=amounts)
        lens = [8189] * (n // 8189) + [n % 8189]
        r = p.create_transfers(t, lens)
        assert (r["status"] == 0xFFFFFFFF).all()
        assert p.stats["replayed"] == 0
        p.compare_state()
    finally:
        p.close()


def test_uniform_config2_small():
    """Config 2 shape at small scale: 10k accounts, 8189-event batches; all `created`."""
    p = Pair(account_capacity=1 << 14, transfer_capacity=1 << 17, batch_events_max=1 << 17)
    try:
        acc = workload.accounts(10_000, seed=42)
        r = p.create_accounts(acc, [8189, 10_000 - 8189])
        assert (r["status"] == 0xFFFFFFFF).all()
        t = workload.transfers_uniform(100_000, 10_000, seed=42)
        lens = [8189] * (100_000 // 8189) + [100_000 % 8189]
        r = p.create_transfers(t, lens)
        assert (r["status"] == 0xFFFFFFFF).all()
        assert p.stats["replayed"] == 0
        assert p.stats["ae_window"] == 1  # (the one-pass AccountEvents)
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("mode", ["spin", "stream-sync"])
def test_many_small_registered_calls(mode, monkeypatch):
    """The host's end-of-call wait: stage_out's last workgroup publishes a sequence word after every
    workgroup's results and scalar words (each thread releases its stores at system scope). 300
    small calls from a registered pool, every third one clean, each reply compared with the oracle
    as soon as the call returns (Pair checks every result); TBG_NO_SPIN_SYNC (a stream
    synchronisation) is the control."""
    if mode == "stream-sync":
        monkeypatch.setenv("TBG_NO_SPIN_SYNC", "1")
    rng = np.random.default_rng(31)
    p = Pair(account_capacity=1 << 12, transfer_capacity=1 << 20, batch_events_max=8189,
             registered=True)
    try:
        n_acc = 500
        p.create_accounts(workload.accounts(n_acc, seed=4))
        off = 0
        for call in range(300):
            n = int(rng.integers(1, 3000)) if call % 10 else 8189
            t = workload.transfers_uniform(n, n_acc, seed=call, id_offset=off)
            off += n
            if call % 3:
                bad = rng.random(n) < 0.05
                t["id"][bad] = 0
            p.create_transfers(t, _split(n, rng, 8189))
        assert p.stats["ingest_finished"] == 0  # (host-buffer calls end in stage_out)
        p.compare_state()
    finally:
        p.close()


def test_sort_path_large_key_space():
    """More than 262,144 accounts with at most 8 account fields per balance item: balance items
    take the radix sort + run reduction -- short runs (uniform over 300k accounts) and runs that
    span lanes and tiles (2,000 accounts)."""
    p = Pair(account_capacity=1 << 19, transfer_capacity=1 << 19, batch_events_max=1 << 17)
    try:
        n_acc = 300_000
        acc = workload.accounts(n_acc, seed=5)
        for i in range(0, n_acc, 100_000):
            p.create_accounts(acc[i:i + 100_000], [8189] * 12 + [100_000 - 12 * 8189])
        t = workload.transfers_uniform(130_000, n_acc, seed=5)
        r = p.create_transfers(t, [8189] * 15 + [130_000 - 15 * 8189])
        assert (r["status"] == 0xFFFFFFFF).all()
        t = workload.transfers_uniform(130_000, 2_000, seed=6, id_offset=130_000)
        p.create_transfers(t, [65_000, 65_000])
        p.compare_state()
    finally:
        p.close()


def test_atomic_path_sparse_keys():
    """More than 8 account fields per balance item (config 5's shape): balance items are applied
    with u128 atomics; then a call whose items collide on few accounts."""
    p = Pair(account_capacity=1 << 19, transfer_capacity=1 << 18, batch_events_max=1 << 17)
    try:
        n_acc = 300_000
        acc = workload.accounts(n_acc, seed=7)
        for i in range(0, n_acc, 100_000):
            p.create_accounts(acc[i:i + 100_000], [8189] * 12 + [100_000 - 12 * 8189])
        t = workload.transfers_uniform(70_000, n_acc, seed=7)
        r = p.create_transfers(t, [8189] * 8 + [70_000 - 8 * 8189])
        assert (r["status"] == 0xFFFFFFFF).all()
        t = workload.transfers_uniform(70_000, 1_000, seed=8, id_offset=70_000)
        p.create_transfers(t, [35_000, 35_000])
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("lean", [True, False], ids=["lean", "records"])
def test_atomic_path_sparse_demotions(lean, monkeypatch):
    """Sparse key spaces (config 5's shape, >= 65,536 events): tr_ingest applies the FAST deltas
    itself and, `lean`, writes no per-event record (tr_commit looks the accounts up again). A call
    that makes tr_commit demote and fix events: limit-flag accounts, duplicate ids, closing flags,
    post/voids (several of one pending transfer) -- TBG_NO_LEAN_LOOKUP writes the records."""
    if not lean:
        monkeypatch.setenv("TBG_NO_LEAN_LOOKUP", "1")
    rng = np.random.default_rng(21)
    p = Pair(account_capacity=1 << 19, transfer_capacity=1 << 19, batch_events_max=1 << 17)
    try:
        n_acc = 300_000
        acc = workload.accounts(n_acc, seed=7)
        acc["flags"][rng.random(n_acc) < 0.01] |= 2  # debits_must_not_exceed_credits
        for i in range(0, n_acc, 100_000):
            p.create_accounts(acc[i:i + 100_000], [8189] * 12 + [100_000 - 12 * 8189])
        n = 70_000
        split = [8189] * 8 + [n - 8 * 8189]
        t = workload.transfers_uniform(n, n_acc, seed=7)
        pend = rng.random(n) < 0.1
        t["flags"][pend] |= 2
        t["timeout"][pend & (rng.random(n) < 0.5)] = 5
        r = p.create_transfers(t, split)
        pending_ids = t["id"][pend & (r["status"] == 0xFFFFFFFF), 0]
        u = workload.transfers_uniform(n, n_acc, seed=8, id_offset=1_000_000)
        dup = rng.random(n) < 0.005
        u["id"][dup] = u["id"][rng.integers(0, n, size=int(dup.sum()))]
        u["flags"][rng.random(n) < 0.002] |= 64   # closing_debit
        u["flags"][rng.random(n) < 0.002] |= 128  # closing_credit
        u["flags"][rng.random(n) < 0.01] |= 2     # pending
        pv = rng.random(n) < 0.03
        u["flags"][pv] = np.where(rng.random(int(pv.sum())) < 0.5, 4, 8)  # post / void
        u["pending_id"][pv, 0] = pending_ids[rng.integers(0, len(pending_ids) // 4,
                                                          size=int(pv.sum()))]
        u["debit_account_id"][pv] = 0
        u["credit_account_id"][pv] = 0
        u["ledger"][pv] = 0
        u["code"][pv] = 0
        u["amount"][pv, 0] = np.where(rng.random(int(pv.sum())) < 0.5, 0, 2**64 - 1)
        u["amount"][pv, 1] = np.where(u["amount"][pv, 0] == 0, 0, 2**64 - 1)
        p.create_transfers(u, split)
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("window", [True, False], ids=["window", "buckets"])
def test_bucket_path_hot_skew(window, monkeypatch):
    """One call of >= 65,536 events over hot limited accounts: window (pair items, LDS counters)
    or bucketed balances (TBG_NO_WINDOW) with 90% of the items on few accounts, next to replayed
    limit checks."""
    if not window:
        monkeypatch.setenv("TBG_NO_WINDOW", "1")
    p = Pair(account_capacity=1 << 14, transfer_capacity=1 << 18, batch_events_max=1 << 17)
    try:
        acc = workload.accounts(6_000, seed=7)
        acc["flags"][1:101] |= 2
        p.create_accounts(acc)
        p.create_transfers(workload.funding_transfers(100, 200_000, id_offset=10_000_000))
        t = workload.transfers_hot_limits(80_000, n_accounts=6_000, n_hot=100, seed=7)
        p.create_transfers(t, [8189] * 9 + [80_000 - 9 * 8189])
        t = workload.transfers_uniform(70_000, 6_000, seed=8, id_offset=20_000_000)
        p.create_transfers(t, [70_000])
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("n_acc", [5_000, 9_000], ids=["4-fields", "posted-only"])
def test_balance_window_edges(n_acc):
    """The balance window (kernels.hpp): calls of >= 65,536 events over <= 2^14 accounts. With
    5,000 accounts all four balance fields sit in the LDS window; with 9,000 only the posted ones
    (pending deltas take u128 atomics on the row). Amounts from 1 to 2^32 - 1 (u32 LDS sums that
    wrap: the carry words), 2^32 .. 2^35 (the high part through the carry words), >= 2^35 (too
    wide for a pair item: tr_commit's atomics), pending transfers, and limited accounts whose
    SLOW events demote FAST events (their items withdrawn); a second call checks that the carry
    words were consumed."""
    rng = np.random.default_rng(n_acc)
    p = Pair(account_capacity=1 << 14, transfer_capacity=1 << 19, batch_events_max=1 << 17)
    try:
        acc = workload.accounts(n_acc, seed=9, ledger=2)
        acc["flags"][1:41] |= 2  # debits_must_not_exceed_credits
        p.create_accounts(acc, _split(n_acc, rng, 8189))
        p.create_transfers(workload.funding_transfers(40, 10**12, id_offset=50_000_000))
        off = 0
        for call in range(2):
            n = 90_000
            t = workload.transfers_uniform(n, n_acc, seed=call + 17, id_offset=off)
            off += n
            kind = rng.random(n)
            amt = t["amount"][:, 0]
            amt[kind < 0.3] = rng.integers(2**31, 2**32, size=int((kind < 0.3).sum()),
                                           dtype=np.uint64)
            big = (kind >= 0.3) & (kind < 0.35)
            amt[big] = rng.integers(2**32, 2**35, size=int(big.sum()), dtype=np.uint64)
            wide = (kind >= 0.35) & (kind < 0.37)
            amt[wide] = rng.integers(2**35, 2**40, size=int(wide.sum()), dtype=np.uint64)
            t["amount"][:, 0] = amt
            pend = (kind >= 0.37) & (kind < 0.5)
            t["flags"][pend] |= 2
            r = p.create_transfers(t, _split(n, rng, 8189))
            assert (r["status"] == 0xFFFFFFFF).mean() > 0.9
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("case", ["window", "no-window", "skew", "wide-rows"])
def test_account_events_window(case, monkeypatch):
    """AccountEvents of balance-window calls in one pass (events.hpp ae_window_emit): calls of
    >= 65,536 events over <= 12,288 accounts whose created events are plain single-phase, with
    statically failed events between them (ids 0, same accounts, existing ids of an earlier call:
    no record), interleaved with small calls (side-stream appends) and a pulse, compared with the
    oracle's log byte for byte and through get_change_events. `skew`: 90 % of the touches on 8
    accounts (long per-round lists); `no-window`: TBG_NO_AE_WINDOW (the general appends);
    `wide-rows`: 13,000 accounts (above the window emit's LDS) take the general appends; a call with
    pending transfers takes the dense emit (ae_dense_*)."""
    if case == "no-window":
        monkeypatch.setenv("TBG_NO_AE_WINDOW", "1")
    rng = np.random.default_rng(77)
    n_acc = 13_000 if case == "wide-rows" else 10_000
    p = Pair(account_capacity=1 << 14, transfer_capacity=1 << 20, batch_events_max=1 << 17,
             pulse_batch_max=64, pulse_next_timestamp_init=TIMESTAMP_MAX)
    try:
        acc = workload.accounts(n_acc, seed=3)
        p.create_accounts(acc, _split(n_acc, rng, 8189))
        off = 0
        windows = 0
        for call in range(4):
            n = 70_000 + 10_000 * call
            t = workload.transfers_uniform(n, n_acc, seed=100 + call, id_offset=off)
            off += n
            if case == "skew":
                hot = rng.random(n) < 0.9
                t["debit_account_id"][hot, 0] = rng.integers(1, 5, size=int(hot.sum()))
                hot = rng.random(n) < 0.9
                t["credit_account_id"][hot, 0] = rng.integers(5, 9, size=int(hot.sum()))
            fail = rng.random(n)
            t["id"][fail < 0.01] = 0                                    # id_must_not_be_zero
            same = (fail >= 0.01) & (fail < 0.02)
            t["credit_account_id"][same] = t["debit_account_id"][same]  # accounts_must_be_different
            if call:
                old = (fail >= 0.02) & (fail < 0.03)                    # exists / exists_with_*
                t["id"][old, 0] = rng.integers(1, off - n, size=int(old.sum()))
            if call == 2:
                pend = fail >= 0.995                                    # pending: general appends
                t["flags"][pend] |= 2
            r = p.create_transfers(t, _split(n, rng, 8189))
            assert (r["status"] == 0xFFFFFFFF).mean() > 0.9
            path = p.last_stats["ae_window"]  # 1: window emit, 2: dense emit, 0: general
            if case in ("no-window", "wide-rows"):
                assert path == 0
            elif call == 2:
                assert path == 2  # (pending transfers: the dense emit)
            mid_ts = int(r["timestamp"][n // 2])
            windows += path == 1
            # small calls (side stream) and a pulse between the window calls
            s = workload.transfers_uniform(3_000, n_acc, seed=200 + call, id_offset=off)
            off += 3_000
            s["flags"][rng.random(3_000) < 0.2] |= 2
            s["timeout"][s["flags"] & 2 != 0] = 1
            p.create_transfers(s, _split(3_000, rng, 1000))
            p.tick(2 * NS_PER_S)
        p.compare_state()
        assert len(p.change_events()) > 0
        assert len(p.change_events(timestamp_min=mid_ts)) > 0  # (inside the last window call)
        if case in ("window", "skew"):
            assert windows >= 2  # (calls with in-call duplicates of failed ids replay)
    finally:
        p.close()


@pytest.mark.parametrize("case", ["wide", "wide-skew", "carry"])
def test_account_events_window_wide(case):
    """AccountEvents of balance-window calls with wide amounts in one pass (events.hpp ae_wide_*:
    u128 sums, the emit's rounds from the last one back): `wide`: amounts log-uniform below 2^63
    and 1 % of them within 2^20 of 2^64 (slice sums past 2^64 in the partials' third limb);
    `wide-skew`: the same amounts with 90 % of the touches on 8 accounts (long round lists, later
    sums near 2^80); `carry`: packed amounts of ~2^30 on 8 hot accounts (no wide item, a window
    key's sum past 2^32: kFlagWideSums). Statically failed events between the created ones, small
    calls and a pulse between the window calls; the log compared with the oracle's byte for byte."""
    rng = np.random.default_rng(78)
    n_acc = 10_000
    p = Pair(account_capacity=1 << 14, transfer_capacity=1 << 20, batch_events_max=1 << 17,
             pulse_batch_max=64, pulse_next_timestamp_init=TIMESTAMP_MAX)
    try:
        acc = workload.accounts(n_acc, seed=4)
        p.create_accounts(acc, _split(n_acc, rng, 8189))
        off = 0
        paths = []
        for call in range(3):
            n = 70_000 + 13_333 * call  # (slices of 16,384 events: the last one partial)
            t = workload.transfers_uniform(n, n_acc, seed=300 + call, id_offset=off,
                                           amounts="exp" if case == "carry" else "wide")
            off += n
            if case in ("wide-skew", "carry"):
                hot = rng.random(n) < 0.9
                t["debit_account_id"][hot, 0] = rng.integers(1, 5, size=int(hot.sum()))
                hot = rng.random(n) < 0.9
                t["credit_account_id"][hot, 0] = rng.integers(5, 9, size=int(hot.sum()))
            if case == "carry":
                t["amount"][:, 0] = rng.integers(1 << 29, 1 << 30, size=n, dtype=np.uint64)
            else:
                top = rng.random(n) < 0.01
                t["amount"][top, 0] = np.uint64(2**64 - 1) - rng.integers(0, 1 << 20, size=int(top.sum()), dtype=np.uint64)
            fail = rng.random(n)
            t["id"][fail < 0.01] = 0                                    # id_must_not_be_zero
            same = (fail >= 0.01) & (fail < 0.02)
            t["credit_account_id"][same] = t["debit_account_id"][same]  # accounts_must_be_different
            r = p.create_transfers(t, _split(n, rng, 8189))
            assert (r["status"] == 0xFFFFFFFF).mean() > 0.95
            paths.append(p.last_stats["ae_window"])
            s = workload.transfers_uniform(3_000, n_acc, seed=400 + call, id_offset=off)
            off += 3_000
            s["flags"][rng.random(3_000) < 0.2] |= 2
            s["timeout"][s["flags"] & 2 != 0] = 1
            p.create_transfers(s, _split(3_000, rng, 1000))
            p.tick(2 * NS_PER_S)
        assert paths == [3] * 3  # (3: the wide window emit)
        p.compare_state()
        assert len(p.change_events()) > 0
    finally:
        p.close()


@pytest.mark.parametrize("case", ["dense", "closing", "wide", "suffix", "no-window"])
def test_account_events_dense(case, monkeypatch):
    """AccountEvents of general calls in one pass (events.hpp ae_dense_*): calls of > 8,192 events
    with pending transfers, posts and voids of them (replayed and FAST), linked chains with
    injected failures and limited accounts, against the oracle's log byte for byte. `closing`:
    pending transfers that close accounts (a `closed` flip) and `wide`: amounts of 2^19 and more
    make the call take the general appends; `suffix`: 3,000 created transfers of 2^19 - 1 on one
    debit account -- every amount passes ae_dense_stage, but the account's later-delta suffix
    crosses 2^30 and ae_dense_suffix must refuse the call; `no-window`:
    TBG_NO_AE_WINDOW."""
    if case == "no-window":
        monkeypatch.setenv("TBG_NO_AE_WINDOW", "1")
    rng = np.random.default_rng(91)
    p = Pair(account_capacity=1 << 12, transfer_capacity=1 << 18, batch_events_max=1 << 16,
             pulse_batch_max=8190)
    try:
        acc = workload.accounts(2_000, seed=5)
        acc["flags"][:8] |= 2
        p.create_accounts(acc)
        pending, seen = np.zeros(0, dtype=np.uint64), np.zeros(0, dtype=np.uint64)
        resolved = np.zeros(0, dtype=np.uint64)
        offset = 0
        paths = []
        for step in range(5):
            n = 20_000
            t = workload.transfers_two_phase(n, 2_000, seed=70 + step, id_offset=offset,
                                             prior_pending_ids=pending, prior_ids=seen,
                                             prior_resolved_ids=resolved, n_limited=8)
            offset += n
            if case == "closing" and step == 3:
                pend = np.nonzero((t["flags"] & 2) != 0)[0][:20]
                t["flags"][pend] |= 64  # closing_debit
            if case == "wide" and step == 3:
                single = np.nonzero(t["flags"] == 0)[0][:20]
                t["amount"][single, 0] = 1 << 20
            if case == "suffix" and step == 3:
                single = np.nonzero((t["flags"] == 0) & (t["debit_account_id"][:, 0] > 8) &
                                    (t["credit_account_id"][:, 0] != 100))[0][:3_000]
                assert len(single) == 3_000 and single[-1] - single[0] > 2 * 2_048
                t["debit_account_id"][single, 0] = 100
                t["amount"][single, 0] = (1 << 19) - 1
            r = p.create_transfers(t, _split(n, rng, 8189))
            if case == "suffix" and step == 3:  # (some close failing chains or repeat ids)
                assert (r["status"][single] == 0xFFFFFFFF).sum() * ((1 << 19) - 1) > 1 << 30
            paths.append(p.last_stats["ae_window"])
            made = r["status"] == 0xFFFFFFFF
            ids = t["id"][:, 0]
            pending = np.concatenate([pending, ids[made & ((t["flags"] & 2) != 0)]])[-20_000:]
            resolved = np.concatenate([resolved, t["pending_id"][made & ((t["flags"] & 12) != 0), 0]])
            seen = np.concatenate([seen, ids])[-20_000:]
            p.tick(NS_PER_S)
        if case == "no-window":
            assert paths == [0] * 5
        elif case == "dense":
            assert paths == [2] * 5
        else:  # (after the closing step, voids of its closing transfers flip `closed` back too)
            assert paths[:3] == [2] * 3 and paths[3] == 0
        p.compare_state()
        assert len(p.change_events()) > 0
    finally:
        p.close()


def test_account_events_dense_hot():
    """The one-pass AccountEvents (ae_dense_emit's sorted touches) under config 3's skew: a
    Zipfian hot account takes ~1 in 6 debits (hundreds of touches per 2,048-event slice), limited
    accounts run out of credits mid-call; the log against the oracle's byte for byte."""
    rng = np.random.default_rng(33)
    p = Pair(account_capacity=1 << 14, transfer_capacity=1 << 17, batch_events_max=1 << 16)
    try:
        acc = workload.accounts(3_000, seed=8)
        acc["flags"][1:101] |= 2
        p.create_accounts(acc)
        p.create_transfers(workload.funding_transfers(100, 300_000, id_offset=10_000_000))
        paths = []
        for step in range(3):
            n = 30_000
            t = workload.transfers_hot_limits(n, n_accounts=3_000, n_hot=100, seed=50 + step,
                                              id_offset=step * n)
            r = p.create_transfers(t, _split(n, rng, 8189))
            paths.append(p.last_stats["ae_window"])
            assert (r["status"] == 54).sum() > 0 or step == 0
        assert paths == [2] * 3
        p.compare_state()
        assert len(p.change_events()) > 0
    finally:
        p.close()


def test_hot_limits_config3_small():
    """Config 3 shape at small scale: Zipfian hot accounts with debits_must_not_exceed_credits."""
    p = Pair(account_capacity=1 << 14, transfer_capacity=1 << 16, batch_events_max=1 << 15)
    try:
        acc = workload.accounts(2_000, seed=3)
        acc["flags"][1:101] |= 2
        p.create_accounts(acc)
        p.create_transfers(workload.funding_transfers(100, 200_000, id_offset=10_000_000))
        t = workload.transfers_hot_limits(20_000, n_accounts=2_000, n_hot=100, seed=3)
        r = p.create_transfers(t, [8189, 8189, 20_000 - 2 * 8189])
        failed = (r["status"] == 54).sum()
        assert failed > 0, "the workload should exercise exceeds_credits"
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("registered", [True, False], ids=["registered", "pageable"])
def test_small_calls_alternating_with_pulses(registered):
    """The round-3 fault's shape (config 4's single-batch commits): small calls whose
    AccountEvents appends run on the side stream behind the next call, alternating with pulses
    whose expiries touch the same few accounts while those appends are in flight (the staging
    buffers reused two calls back, the pulse's own staged expiries between them); the log and
    every row against the oracle."""
    rng = np.random.default_rng(13)
    p = Pair(account_capacity=1 << 10, transfer_capacity=1 << 19, batch_events_max=8189,
             pulse_batch_max=8190, registered=registered)
    try:
        n_acc = 64  # (every call and every pulse touch the same accounts)
        p.create_accounts(workload.accounts(n_acc, seed=13))
        pending, seen = np.zeros(0, dtype=np.uint64), np.zeros(0, dtype=np.uint64)
        resolved = np.zeros(0, dtype=np.uint64)
        offset = 0
        for step in range(40):
            n = 8189 if step % 3 == 0 else int(rng.integers(500, 8189))
            t = workload.transfers_two_phase(n, n_acc, seed=300 + step, id_offset=offset,
                                             prior_pending_ids=pending, prior_ids=seen,
                                             prior_resolved_ids=resolved, n_limited=0)
            offset += n
            r = p.create_transfers(t, [n])
            created = r["status"] == 0xFFFFFFFF
            is_pending = (t["flags"] & 2) != 0
            pv = (t["flags"] & 12) != 0
            pending = np.concatenate([pending, t["id"][created & is_pending, 0]])[-8_000:]
            resolved = np.concatenate([resolved, t["pending_id"][created & pv, 0]])[-8_000:]
            seen = np.concatenate([seen, t["id"][:, 0]])[-20_000:]
            p.tick(int(rng.integers(1, 3)) * NS_PER_S)
        p.compare_state()
        assert len(p.change_events()) > 0
    finally:
        p.close()


@pytest.mark.parametrize("span", ["packed", "wide"])
def test_pulse_many_candidates(span):
    """Pulses over ~45k expired pending transfers with pulse_batch_max 8,190: 22 sorted runs, five
    merge levels of several workgroups per pair, each pulse taking the first 8,190 in
    (expires_at, timestamp) order. `packed`: timeouts of 1-600 s (one-word keys); `wide`: timeouts
    up to 2^32 - 1 s, an expiry span past the one-word key's reach (the two-word path). The
    expired counts, pulse_next_timestamp, rows and AccountEvents against the oracle."""
    rng = np.random.default_rng(71 if span == "packed" else 72)
    p = Pair(account_capacity=1 << 10, transfer_capacity=1 << 17, batch_events_max=1 << 14,
             pulse_batch_max=8190)
    try:
        p.create_accounts(workload.accounts(200, seed=71))
        hi = 600 if span == "packed" else (1 << 32) - 1
        for step in range(3):
            n = 15_000
            t = workload.transfers_uniform(n, 200, seed=710 + step, id_offset=step * n)
            t["flags"] |= 2  # pending
            t["timeout"] = rng.integers(1, hi, size=n, dtype=np.int64)
            t["timeout"][rng.random(n) < 0.3] = int(rng.integers(1, 4))  # (equal expiries: ties)
            r = p.create_transfers(t, [8189, n - 8189])
            assert (r["status"] == 0xFFFFFFFF).all()
        before = len(p.pulses)
        p.tick(hi * NS_PER_S + NS_PER_S)
        for _ in range(8):
            p.tick(1)
        expired = [e for _, e in p.pulses[before:]]
        assert expired[:5] == [8190] * 5 and sum(expired) == 45_000, expired
        p.compare_state()
    finally:
        p.close()


def test_two_phase_config4_small():
    """Config 4 shape: pending with timeouts, post/void, linked chains with failures, resubmits,
    pulses."""
    rng = np.random.default_rng(4)
    p = Pair(account_capacity=1 << 12, transfer_capacity=1 << 17, batch_events_max=1 << 15,
             pulse_batch_max=8190)
    try:
        acc = workload.accounts(1_000, seed=4)
        acc["flags"][:8] |= 2  # the injected exceeds_credits failures debit these
        p.create_accounts(acc)
        pending, seen = np.zeros(0, dtype=np.uint64), np.zeros(0, dtype=np.uint64)
        resolved = np.zeros(0, dtype=np.uint64)
        offset = 0
        seen_status = set()
        for step in range(6):
            t = workload.transfers_two_phase(8_000, 1_000, seed=40 + step, id_offset=offset,
                                             prior_pending_ids=pending, prior_ids=seen,
                                             prior_resolved_ids=resolved, n_limited=8)
            offset += 8_000
            r = p.create_transfers(t, [4_000, 4_000])
            seen_status |= set(int(x) for x in r["status"])
            created = r["status"] == 0xFFFFFFFF
            is_pending = (t["flags"] & 2) != 0
            pv = (t["flags"] & 12) != 0
            pending = np.concatenate([pending, t["id"][created & is_pending, 0]])[-5_000:]
            resolved = np.concatenate([resolved, t["pending_id"][created & pv, 0]])[-5_000:]
            seen = np.concatenate([seen, t["id"][:, 0]])[-20_000:]
            p.tick(int(rng.integers(1, 3)) * NS_PER_S)
        # injected failures: exceeds_credits, pending_transfer_already_posted / _voided,
        # transfer_must_have_the_same_ledger_as_accounts, pending_transfer_has_different_amount
        for st in (54, 24, 32):
            assert st in seen_status, st
        assert 33 in seen_status or 34 in seen_status
        p.compare_state()
    finally:
        p.close()


def _transfers(rows):
    t = np.zeros(len(rows), dtype=TRANSFER_DTYPE)
    for i, r in enumerate(rows):
        for k, v in r.items():
            if k in ("id", "debit_account_id", "credit_account_id", "pending_id", "amount"):
                t[k][i, 0] = v & ((1 << 64) - 1)
                t[k][i, 1] = v >> 64
            else:
                t[k][i] = v
    return t


@pytest.mark.parametrize("force_replay", [False, True, "serial"], ids=["parallel", "flow", "serial"])
def test_reopened_account_with_limit(force_replay):
    """A transfer that fails `closed` against an account a void in the same call reopens must
    replay with the serial balances of its limited debit account: a later parallel credit to that
    account may not leak into its exceeds_credits check."""
    p = Pair(account_capacity=64, transfer_capacity=1024, batch_events_max=256,
             force_replay=force_replay)
    try:
        acc = workload.accounts(4, seed=1, ledger=1)
        acc["flags"] = [2, 0, 0, 0]  # A: debits_must_not_exceed_credits; B, S, C plain
        p.create_accounts(acc)
        # S -> A 100 (A's credits); a pending closing_credit transfer C -> B closes B.
        p.create_transfers(_transfers([
            dict(id=10, debit_account_id=3, credit_account_id=1, amount=100, ledger=1, code=1),
            dict(id=11, debit_account_id=4, credit_account_id=2, amount=5, ledger=1, code=1,
                 flags=2 | 128),
        ]))
        r = p.create_transfers(_transfers([
            dict(id=20, pending_id=11, flags=8),                                       # void: reopens B
            dict(id=21, debit_account_id=1, credit_account_id=2, amount=150, ledger=1, code=1),
            dict(id=22, debit_account_id=3, credit_account_id=1, amount=100, ledger=1, code=1),
        ]))
        assert list(r["status"]) == [0xFFFFFFFF, 54, 0xFFFFFFFF]  # 54: exceeds_credits
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("force_replay", [False, True, "serial"], ids=["parallel", "flow", "serial"])
def test_account_index_hazards(force_replay):
    """The account index answers the create_transfers checks without the row while an account's
    hazard bits are clear; every way an account becomes closed or gets a balance near 2^128 must
    set them: created closed, closed by a replayed closing transfer (seen by the next call),
    balances set to 2^127 (overflow checks)."""
    p = Pair(account_capacity=64, transfer_capacity=1024, batch_events_max=256,
             force_replay=force_replay)
    try:
        acc = workload.accounts(6, seed=2, ledger=1)
        acc["flags"] = [32, 0, 0, 0, 0, 0]  # A created closed; B, C, D, E, F plain
        p.create_accounts(acc)
        r = p.create_transfers(_transfers([
            dict(id=100, debit_account_id=2, credit_account_id=1, amount=5, ledger=1, code=1),
            dict(id=101, debit_account_id=3, credit_account_id=4, amount=7, ledger=1, code=1,
                 flags=2 | 64),                                                 # closes C (debit)
            dict(id=102, debit_account_id=2, credit_account_id=4, amount=9, ledger=1, code=1),
        ]))
        assert list(r["status"]) == [66, 0xFFFFFFFF, 0xFFFFFFFF]
        r = p.create_transfers(_transfers([
            dict(id=110, debit_account_id=3, credit_account_id=2, amount=1, ledger=1, code=1),
            dict(id=111, debit_account_id=2, credit_account_id=3, amount=1, ledger=1, code=1),
            dict(id=112, debit_account_id=2, credit_account_id=4, amount=1, ledger=1, code=1),
        ]))
        assert list(r["status"]) == [65, 66, 0xFFFFFFFF]
        p.set_balances(5, dpo=1 << 127)
        p.set_balances(6, cp=(1 << 128) - 10)
        r = p.create_transfers(_transfers([
            dict(id=120, debit_account_id=5, credit_account_id=2, amount=1 << 127 | 1,
                 ledger=1, code=1),
            dict(id=121, debit_account_id=2, credit_account_id=6, amount=20, ledger=1, code=1,
                 flags=2),
            dict(id=122, debit_account_id=5, credit_account_id=2, amount=3, ledger=1, code=1),
            dict(id=123, debit_account_id=4, credit_account_id=6, amount=3, ledger=1, code=1),
        ]))
        assert r["status"][0] != 0xFFFFFFFF and r["status"][1] != 0xFFFFFFFF
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("force_replay", [False, True, "serial"], ids=["parallel", "flow", "serial"])
def test_account_index_wide_entries(force_replay):
    """Index entries hold an id's low word and a ledger's low 16 bits: accounts whose id high
    word is nonzero or whose ledger is >= 2^16 are matched and checked through the row. Ids that
    share a low word, and ledgers that share their low 16 bits, must stay distinct."""
    p = Pair(account_capacity=64, transfer_capacity=1024, batch_events_max=256,
             force_replay=force_replay)
    try:
        acc = workload.accounts(6, seed=3, ledger=1)
        acc["id"][:, 0] = [7, 7, 7, 8, 9, 10]
        acc["id"][:, 1] = [0, 1, 2, 0, 0, 0]
        acc["ledger"] = [1, 1, 1, 65537, 65537, 1]
        acc["flags"] = 0
        p.create_accounts(acc)
        hi = 1 << 64
        r = p.create_transfers(_transfers([
            dict(id=1, debit_account_id=7, credit_account_id=7 + hi, amount=5, ledger=1, code=1),
            dict(id=2, debit_account_id=7 + 2 * hi, credit_account_id=7 + hi, amount=3, ledger=1,
                 code=1),
            dict(id=3, debit_account_id=7 + 3 * hi, credit_account_id=7, amount=1, ledger=1,
                 code=1),                                                  # debit not found
            dict(id=4, debit_account_id=8, credit_account_id=9, amount=2, ledger=65537, code=1),
            dict(id=5, debit_account_id=8, credit_account_id=10, amount=2, ledger=65537,
                 code=1),                                                  # different ledgers
            dict(id=6, debit_account_id=8, credit_account_id=9, amount=2, ledger=1, code=1),
            dict(id=7, debit_account_id=10, credit_account_id=7, amount=2, ledger=1, code=1),
        ]))
        created = r["status"] == 0xFFFFFFFF
        assert created.tolist() == [True, True, False, True, False, False, True]
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("seed", range(4))
def test_flow_replay_stress(seed):
    """Every event through the flow replay, with enough events per call for many units to run at
    once: chains, duplicates, post/void of pending transfers created earlier in the same call,
    limits and closing, over a small account set (long key chains) -- against the oracle."""
    rng = np.random.default_rng(5000 + seed)
    p = Pair(account_capacity=1 << 12, transfer_capacity=1 << 17, batch_events_max=1 << 14,
             pulse_batch_max=64, pulse_next_timestamp_init=TIMESTAMP_MAX, force_replay=True)
    try:
        n_acc = 160
        clean = workload.accounts(n_acc, seed=seed, id_offset=0, ledger=1)
        clean["flags"] = rng.choice([0, 0, 0, 2, 4, 8], size=n_acc).astype(np.uint16)
        p.create_accounts(clean, _split(n_acc, rng, 64))
        ids_seen = []
        for step in range(5):
            pend = np.array(ids_seen[-3000:], dtype=np.uint64) if ids_seen else None
            t = workload.fuzz_transfers(rng, 6000, 9000, n_acc + 1, pending_ids=pend)
            ids_seen.extend(int(x) for x in t["id"][:, 0])
            p.create_transfers(t, _split(len(t), rng, 2048))
            p.tick(int(rng.integers(1, 3)) * NS_PER_S)
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("walk", ["wave", "wave-seq", "one-lane"])
@pytest.mark.parametrize("n_acc", [200, 700], ids=["lanes", "over-lanes"])
def test_account_lanes_limits(n_acc, walk, monkeypatch):
    """Calls whose replayed events are all limit events run on the account lanes (one lane per
    limited account): debits_must_not_exceed_credits and credits_must_not_exceed_debits on both
    sides, transfers between two limited accounts (both verdicts needed), between a limited and an
    unlimited account, and funding; 700 limited accounts exceed the lanes (the flow replay runs).
    `walk`: one wave per walked owner (lanes_walk; wave-wide steps or, TBG_WALK_SEQ, event by
    event) or one lane (lanes_replay)."""
    if walk == "one-lane":
        monkeypatch.setenv("TBG_LANES_ONE_LANE", "1")
    if walk == "wave-seq":  # the walk event by event (no wave-wide steps)
        monkeypatch.setenv("TBG_WALK_SEQ", "1")
    rng = np.random.default_rng(n_acc)
    p = Pair(account_capacity=1 << 12, transfer_capacity=1 << 17, batch_events_max=1 << 15)
    try:
        acc = workload.accounts(n_acc, seed=11, ledger=2)
        # (6: both limits -- such an owner walks event by event)
        acc["flags"] = rng.choice([0, 2, 4, 6], size=n_acc, p=[0.2, 0.35, 0.35, 0.1]).astype(np.uint16)
        acc["flags"][0] = 0  # an unlimited source
        p.create_accounts(acc, _split(n_acc, rng, 512))
        fund = workload.funding_transfers(n_acc - 1, 50_000, id_offset=1 << 30)
        fund["credit_account_id"][:, 0] = np.arange(2, n_acc + 1, dtype=np.uint64)
        p.create_transfers(fund, _split(len(fund), rng, 512))
        back = fund.copy()  # and the other way, so credits_must_not_exceed_debits has room
        back["id"][:, 0] += np.uint64(1 << 20)
        back["debit_account_id"], back["credit_account_id"] = fund["credit_account_id"], fund["debit_account_id"]
        p.create_transfers(back, _split(len(back), rng, 512))
        off = 0
        for step in range(4):
            t = workload.transfers_uniform(12_000, n_acc, seed=100 + step, id_offset=off)
            off += 12_000
            t["amount"][:, 0] = rng.integers(1, 30_000, size=len(t)).astype(np.uint64)
            r = p.create_transfers(t, _split(len(t), rng, 8189))
            if step == 0:
                assert ((r["status"] == 54) | (r["status"] == 55)).any()
        p.compare_state()
    finally:
        p.close()

@pytest.mark.parametrize("additive", [True, False], ids=["additive", "keyed"])
def test_flow_additive_accounts(additive, monkeypatch):
    """Plain accounts that no replayed event reads (Replay::additive, replay.hpp) take the flow
    replay's deltas as u128 atomics without ordering keys: many concurrent units on the same few
    accounts with amounts that carry into the high word, linked chains whose deltas are undone by
    a later failure, posts (partial) and voids of non-closing pending transfers, a void of a
    closing one (its accounts keyed), and a limited account in the mix -- against the oracle, with
    and without the additive path (TBG_NO_ADDITIVE)."""
    if not additive:
        monkeypatch.setenv("TBG_NO_ADDITIVE", "1")
    rng = np.random.default_rng(77)
    p = Pair(account_capacity=64, transfer_capacity=1 << 14, batch_events_max=1 << 12,
             force_replay=True)
    try:
        acc = workload.accounts(10, seed=7, ledger=1)
        acc["flags"] = [0, 0, 0, 0, 0, 0, 0, 0, 2, 0]  # 9: debits_must_not_exceed_credits
        p.create_accounts(acc)
        big = (1 << 64) - 1
        n = 300
        first = []
        for i in range(n):
            dr, cr = rng.choice(8, size=2, replace=False) + 1
            first.append(dict(id=1000 + i, debit_account_id=int(dr), credit_account_id=int(cr),
                              amount=big - i, ledger=1, code=1, flags=2))  # pending
        first.append(dict(id=5000, debit_account_id=10, credit_account_id=1, amount=9, ledger=1,
                          code=1, flags=2 | 64))                           # pending closing_debit
        first.append(dict(id=5001, debit_account_id=1, credit_account_id=9, amount=big, ledger=1,
                          code=1))                                         # funds account 9
        p.create_transfers(_transfers(first))
        second = []
        for i in range(n):
            dr, cr = rng.choice(8, size=2, replace=False) + 1
            kind = i % 5
            if kind == 0:    # a chain whose last event fails: the first two deltas are undone
                second += [dict(id=2000 + 10 * i, debit_account_id=int(dr), credit_account_id=int(cr),
                                amount=big - 7, ledger=1, code=1, flags=1),
                           dict(id=2001 + 10 * i, debit_account_id=int(cr), credit_account_id=int(dr),
                                amount=big - 3, ledger=1, code=1, flags=1),
                           dict(id=2002 + 10 * i, debit_account_id=int(dr), credit_account_id=99,
                                amount=1, ledger=1, code=1)]
            elif kind == 1:  # void (the pending transfer is not closing)
                second.append(dict(id=2000 + 10 * i, pending_id=1000 + i, flags=8))
            elif kind == 2:  # partial post
                second.append(dict(id=2000 + 10 * i, pending_id=1000 + i, amount=big // 3, flags=4))
            elif kind == 3:  # a chain that persists
                second += [dict(id=2000 + 10 * i, debit_account_id=int(dr), credit_account_id=int(cr),
                                amount=big, ledger=1, code=1, flags=1),
                           dict(id=2001 + 10 * i, debit_account_id=int(cr), credit_account_id=int(dr),
                                amount=5, ledger=1, code=1)]
            else:            # the limited account debits
                second.append(dict(id=2000 + 10 * i, debit_account_id=9, credit_account_id=int(cr),
                                   amount=big // 50, ledger=1, code=1))
        second.append(dict(id=6000, pending_id=5000, flags=8))  # void of a closing transfer
        second.append(dict(id=6001, debit_account_id=10, credit_account_id=2, amount=1, ledger=1,
                           code=1))                              # 10 reopened by the void
        r = p.create_transfers(_transfers(second), [len(second)])
        assert (r["status"] == 0xFFFFFFFF).sum() > n // 2
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("walk", ["wave", "wave-seq", "one-lane"])
@pytest.mark.parametrize("free_owners", [True, False], ids=["free", "walked"])
def test_account_lanes_free_owners(free_owners, walk, monkeypatch):
    """Account lanes with free owners (lanes.hpp): limited accounts funded beyond every amount
    they check in the call need no lane (their sides become atomics, events left without owners
    are created), next to limited accounts that run out mid-call and still walk -- with events
    between a free and a walked owner, between two free owners, and with credits_must_not_exceed
    debits on the credit side; against the oracle, with and without free owners."""
    if not free_owners:
        monkeypatch.setenv("TBG_NO_FREE_OWNERS", "1")
    if walk == "one-lane":
        monkeypatch.setenv("TBG_LANES_ONE_LANE", "1")
    if walk == "wave-seq":  # the walk event by event (no wave-wide steps)
        monkeypatch.setenv("TBG_WALK_SEQ", "1")
    rng = np.random.default_rng(91)
    p = Pair(account_capacity=64, transfer_capacity=1 << 14, batch_events_max=1 << 12)
    try:
        acc = workload.accounts(12, seed=9, ledger=1)
        # 1-4: debits_must_not_exceed_credits (1, 2 rich; 3, 4 poor); 5, 6:
        # credits_must_not_exceed_debits (5 rich, 6 poor); 7-12 plain (7 funds everyone).
        acc["flags"] = [2, 2, 2, 2, 4, 4, 0, 0, 0, 0, 0, 0]
        p.create_accounts(acc)
        fund = [dict(id=1 + i, debit_account_id=7, credit_account_id=a, amount=amt, ledger=1,
                     code=1)
                for i, (a, amt) in enumerate([(1, 10**9), (2, 10**9), (3, 3000), (4, 5000)])]
        fund += [dict(id=10, debit_account_id=5, credit_account_id=8, amount=10**9, ledger=1,
                      code=1),
                 dict(id=11, debit_account_id=6, credit_account_id=8, amount=4000, ledger=1,
                      code=1)]
        p.create_transfers(_transfers(fund))
        for call in range(3):
            rows = []
            for i in range(1500):
                dr = int(rng.choice([1, 2, 3, 4, 9, 10]))
                cr = int(rng.choice([5, 6, 1, 3, 11, 12]))
                if cr == dr:
                    cr = 12
                rows.append(dict(id=100_000 * (call + 1) + i, debit_account_id=dr,
                                 credit_account_id=cr, amount=int(rng.integers(1, 60)), ledger=1,
                                 code=1))
            r = p.create_transfers(_transfers(rows), [len(rows)])
            assert (r["status"] == 0xFFFFFFFF).sum() > 0
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("walk", ["wave", "wave-seq", "one-lane"])
def test_account_walk_long_owner(walk, monkeypatch):
    """One walked owner with ~100k events in a single call (its funding runs out a third of the
    way), a second walked owner in another wave with a few hundred events, transfers between them
    both ways (each needs the other's verdict) and the call's LAST event shared by both: the waiting
    owner polls for as long as the long walk takes (the watchdog must count every wave's progress,
    ADVICE r1)."""
    if walk == "one-lane":
        monkeypatch.setenv("TBG_LANES_ONE_LANE", "1")
    if walk == "wave-seq":  # the walk event by event (no wave-wide steps)
        monkeypatch.setenv("TBG_WALK_SEQ", "1")
    rng = np.random.default_rng(4242)
    p = Pair(account_capacity=64, transfer_capacity=1 << 18, batch_events_max=1 << 17)
    try:
        acc = workload.accounts(8, seed=3, ledger=1)
        acc["flags"] = [0, 2, 2, 0, 0, 0, 0, 0]  # 2, 3: debits_must_not_exceed_credits
        p.create_accounts(acc)
        n = 100_000
        p.create_transfers(_transfers([
            dict(id=1, debit_account_id=1, credit_account_id=2, amount=n * 50 // 3, ledger=1,
                 code=1),
            dict(id=2, debit_account_id=1, credit_account_id=3, amount=4000, ledger=1, code=1)]))
        t = workload.transfers_uniform(n, 8, seed=5, id_offset=100)
        t["ledger"] = 1
        t["debit_account_id"][:, 0] = 2
        t["credit_account_id"][:, 0] = rng.choice([4, 5, 6, 7, 8], size=n).astype(np.uint64)
        t["amount"][:, 0] = rng.integers(1, 100, size=n).astype(np.uint64)
        few = rng.choice(n - 1, size=600, replace=False)
        t["debit_account_id"][few[:300], 0] = 3          # 3 -> 2: 2 waits for 3's verdict
        t["credit_account_id"][few[:300], 0] = 2
        t["credit_account_id"][few[300:], 0] = 3         # 2 -> 3: 3 waits for 2's verdict
        t["amount"][few, 0] = rng.integers(1, 40, size=600).astype(np.uint64)
        t["credit_account_id"][n - 1, 0] = 3             # the last event: 2 -> 3
        r = p.create_transfers(t, [8189] * (n // 8189) + [n % 8189])
        assert (r["status"] == 54).sum() > n // 2
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("force_replay", [False, True, "serial"], ids=["parallel", "flow", "serial"])
@pytest.mark.parametrize("length", [257, 8189])
def test_long_linked_chains(length, force_replay):
    """Linked chains longer than the flow replay's per-lane undo log (256 events: such a chain
    runs as a barrier on the global undo log), up to a whole 8189-event batch
    (state_machine.zig:3033-3207): a chain that persists, one whose last event fails (every
    earlier event's balance deltas, statuses and ids undone, the failing id orphaned when the
    failure is transient), one that fails in the middle on a repeated id (`exists` against the
    chain's own earlier event), and one left open by the batch end (linked_event_chain_open)."""
    p = Pair(account_capacity=64, transfer_capacity=1 << 17, batch_events_max=1 << 15,
             force_replay=force_replay)
    try:
        acc = workload.accounts(16, seed=5, ledger=1)
        acc["flags"] = 0
        acc["flags"][0] = 2  # account 1: debits_must_not_exceed_credits
        p.create_accounts(acc)
        p.create_transfers(_transfers([dict(id=1, debit_account_id=2, credit_account_id=1,
                                            amount=1000, ledger=1, code=1)]))
        rng = np.random.default_rng(length)

        def chain(first_id, n):
            rows = []
            for i in range(n):
                dr, cr = (int(x) for x in rng.choice(np.arange(2, 17), size=2, replace=False))
                rows.append(dict(id=first_id + i, debit_account_id=dr, credit_account_id=cr,
                                 amount=int(rng.integers(1, 1000)), ledger=1, code=1,
                                 flags=(1 if i < n - 1 else 0) | (2 if i % 7 == 3 else 0)))
            return rows

        a = chain(10_000, length)                        # persists
        b = chain(20_000, length)                        # last event: exceeds_credits
        b[-1].update(debit_account_id=1, amount=10**9)
        c = chain(30_000, length)                        # middle event repeats an earlier id
        c[length // 2] = dict(c[length // 3])
        d = chain(40_000, length)                        # the batch ends inside the chain
        d[-1]["flags"] |= 1
        r = p.create_transfers(_transfers(a + b + c + d), [length] * 4)
        st = r["status"]
        assert (st[:length] == 0xFFFFFFFF).all()
        assert st[2 * length - 1] == 54 and (st[length:2 * length - 1] == 1).all()
        assert st[2 * length + length // 2] == 46  # exists (its own chain's earlier event)
        assert st[4 * length - 1] == 2             # linked_event_chain_open
        # The failed chains' ids are free again (the orphaned exceeds_credits id is not).
        again = _transfers([dict(b[0], flags=0), dict(c[0], flags=0), dict(b[-1], flags=0)])
        r = p.create_transfers(again)
        assert list(r["status"]) == [0xFFFFFFFF, 0xFFFFFFFF, 68]  # 68: id_already_failed
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("registered", [False, True], ids=["pageable", "registered"])
@pytest.mark.parametrize("force_replay", [False, True, "serial"], ids=["parallel", "flow", "serial"])
def test_change_events(force_replay, registered):
    """AccountEvents (state_machine.zig:4384-4465) and get_change_events (:3395-3527) against the
    oracle: single-phase, pending, posted (partial), voided (also of closing transfers) and
    expired events, balancing amounts, rolled-back chains; then filters by timestamp range and
    limit, and an invalid filter."""
    rng = np.random.default_rng(31)
    p = Pair(account_capacity=1 << 10, transfer_capacity=1 << 15, batch_events_max=4096,
             pulse_batch_max=16, pulse_next_timestamp_init=TIMESTAMP_MAX,
             force_replay=force_replay, registered=registered)
    try:
        acc = workload.accounts(30, seed=3, ledger=1)
        acc["flags"] = rng.choice([0, 0, 2, 4, 8], size=30).astype(np.uint16)
        p.create_accounts(acc)
        ids = []
        for step in range(6):
            pend = np.array(ids[-300:], dtype=np.uint64) if ids else None
            t = workload.fuzz_transfers(rng, 400, 2000, 31, pending_ids=pend)
            ids.extend(int(x) for x in t["id"][:, 0])
            p.create_transfers(t, _split(len(t), rng, 64))
            p.tick(int(rng.integers(1, 3)) * NS_PER_S)
        # Pending transfers on plain accounts (some closing), then posts (partial) and voids.
        plain = [i + 1 for i in range(30) if int(acc["flags"][i]) in (0, 8)]
        pend_rows = [dict(id=90_000 + i, debit_account_id=plain[i % len(plain)],
                          credit_account_id=plain[(i + 1) % len(plain)], amount=100 + i,
                          ledger=1, code=1, flags=2 | (64 if i % 9 == 4 else 0))
                     for i in range(20)]
        p.create_transfers(_transfers(pend_rows))
        p.create_transfers(_transfers(
            [dict(id=91_000 + i, pending_id=90_000 + i, amount=50, flags=4) for i in range(0, 20, 3)] +
            [dict(id=92_000 + i, pending_id=90_000 + i, flags=8) for i in range(1, 20, 3)]))
        p.compare_state()
        all_events = p.change_events()
        assert len(all_events) > 100 and {0, 1, 2, 3, 4} <= set(all_events["type"].tolist())
        ts = all_events["timestamp"]
        p.change_events(timestamp_min=int(ts[10]), timestamp_max=int(ts[60]))
        p.change_events(timestamp_min=int(ts[5]), limit=7)
        p.change_events(timestamp_max=int(ts[-20]), limit=1000, limit_max=33)
        p.change_events(timestamp_min=int(ts[-1]) + 1)
        assert len(p.change_events(timestamp_min=int(ts[50]), timestamp_max=int(ts[40]))) == 0
        assert len(p.change_events(limit=0)) == 0
    finally:
        p.close()


def test_change_events_imported_before_expiries():
    """An imported batch whose timestamps precede a pulse's expiry events (the imported checks
    compare with the transfers' key range, not the events'): the account_events groove is keyed
    by timestamp, so the executor's log must come back in timestamp order."""
    p = Pair(account_capacity=64, transfer_capacity=4096, batch_events_max=256,
             pulse_next_timestamp_init=TIMESTAMP_MAX)
    try:
        acc = workload.accounts(4, seed=1, ledger=1)
        acc["flags"] = 0
        p.create_accounts(acc)
        p.create_transfers(_transfers([dict(id=1, debit_account_id=1, credit_account_id=2,
                                            amount=5, ledger=1, code=1, flags=2, timeout=1)]))
        key_max = p.prepare_timestamp
        p.tick(2 * NS_PER_S)  # the pending transfer expires (events at the pulse's timestamps)
        assert p.pulse_next() == TIMESTAMP_MAX
        imp = _transfers([dict(id=10 + i, debit_account_id=3, credit_account_id=4, amount=7,
                               ledger=1, code=1, flags=256, timestamp=key_max + 10 + i)
                          for i in range(3)])
        r = p.create_transfers(imp)
        assert (r["status"] == 0xFFFFFFFF).all()
        p.compare_state()
        ev = p.change_events()
        assert list(ev["type"]) == [1, 0, 0, 0, 4]
    finally:
        p.close()


@pytest.mark.parametrize("mode", ["parallel", "no-pv-fast", "flow"])
@pytest.mark.parametrize("seed", range(3))
def test_fast_post_void_and_chains(seed, mode, monkeypatch):
    """The parallel path's post/voids, linked chains and pulse_next_timestamp ordering against the
    oracle: post/voids of committed pending transfers drawn from a small pool (many calls post or
    void the same pending transfer several times: the earliest claimant may be FAST, the others
    replay), full / partial / excess / maxInt amounts, voids with and without amounts, mismatched
    accounts / ledgers / codes, pending transfers with timeouts of 0-3 s and some closing ones,
    posts of pending transfers created in the same call, 4-event linked chains mixing all of these
    (all-FAST chains commit in parallel, others replay), and pulses between calls."""
    if mode == "no-pv-fast":
        monkeypatch.setenv("TBG_NO_PV_FAST", "1")
    rng = np.random.default_rng(700 + seed)
    p = Pair(account_capacity=256, transfer_capacity=1 << 16, batch_events_max=1 << 13,
             force_replay=(mode == "flow"))
    try:
        n_acc = 24
        acc = workload.accounts(n_acc, seed=seed, ledger=1)
        p.create_accounts(acc)
        fund = [dict(id=1 + i, debit_account_id=1 + (i + 1) % n_acc, credit_account_id=1 + i,
                     amount=10**12, ledger=1, code=1) for i in range(n_acc)]
        p.create_transfers(_transfers(fund))
        next_id = 1000
        pool = []  # pending transfers of earlier calls: (id, amount)

        def account_pair():
            dr = int(rng.integers(1, n_acc + 1))
            cr = int(rng.integers(1, n_acc + 1))
            return dr, cr if cr != dr else 1 + dr % n_acc

        def event(in_call_pending):
            nonlocal next_id
            next_id += 1
            kind = rng.random()
            if kind < 0.45 and (pool or in_call_pending):
                if in_call_pending and (not pool or rng.random() < 0.1):
                    pid, pamt = in_call_pending[int(rng.integers(0, len(in_call_pending)))]
                else:
                    pid, pamt = pool[int(rng.integers(0, len(pool)))]
                post = rng.random() < 0.6
                r = rng.random()
                if post:
                    amount = [(1 << 128) - 1, pamt, max(pamt // 3, 1), pamt + 1][int(r * 4)]
                else:
                    amount = [0, 0, pamt, max(pamt // 2, 1)][int(r * 4)]
                ev = dict(id=next_id, pending_id=pid, amount=amount,
                          flags=4 if post else 8)
                m = rng.random()
                if m < 0.05:
                    ev["debit_account_id"] = int(rng.integers(1, n_acc + 1))
                elif m < 0.08:
                    ev["ledger"] = 2
                elif m < 0.10:
                    ev["code"] = 9
                return ev
            dr, cr = account_pair()
            amount = int(rng.integers(1, 10**6))
            if kind < 0.75:
                flags = 2
                if rng.random() < 0.03:
                    flags |= 64 if rng.random() < 0.5 else 128  # closing_debit / closing_credit
                ev = dict(id=next_id, debit_account_id=dr, credit_account_id=cr, amount=amount,
                          ledger=1, code=1, flags=flags, timeout=int(rng.integers(0, 4)))
                in_call_pending.append((next_id, amount))
                return ev
            return dict(id=next_id, debit_account_id=dr, credit_account_id=cr, amount=amount,
                        ledger=1, code=1)

        for call in range(6):
            rows, in_call = [], []
            while len(rows) < 3000:
                if rng.random() < 0.12:
                    chain = [event(in_call) for _ in range(4)]
                    for ev in chain[:-1]:
                        ev["flags"] = ev.get("flags", 0) | 1  # linked
                    rows += chain
                else:
                    rows.append(event(in_call))
            t = _transfers(rows)
            r = p.create_transfers(t, [1500, len(rows) - 1500])
            created = r["status"] == 0xFFFFFFFF
            for i, ev in enumerate(rows):
                if created[i] and (ev.get("flags", 0) & 2):
                    pool.append((ev["id"], ev["amount"]))
            pool = pool[-400:]
            p.tick(int(rng.integers(1, 3)) * NS_PER_S)
            p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("seed", range(4))
def test_doomed_debits(seed, monkeypatch):
    """The flow plan's doomed debits (group.hpp: a replayed debit of a debits_must_not_exceed_credits
    account that fails in any order gets no key on that account): limited accounts with some
    starting credit, debits above and below what the call's credits could ever cover, credits to
    them in the same call (bounding the rule), pending debits, posts / voids of their pending
    transfers (which turn the rule off for the account), linked chains holding doomed debits --
    every call against the oracle, and once more with the rule off (TBG_NO_DOOM)."""
    rng = np.random.default_rng(500 + seed)
    for doom in (True, False):
        if not doom:
            monkeypatch.setenv("TBG_NO_DOOM", "1")
        p = Pair(account_capacity=256, transfer_capacity=1 << 14, batch_events_max=4096)
        try:
            n_acc = 40
            acc = workload.accounts(n_acc, seed=seed, ledger=1)
            acc["flags"][:8] |= 2  # accounts 1..8: debits_must_not_exceed_credits
            p.create_accounts(acc)
            # starting credits of the limited accounts (from unlimited accounts 20..39)
            p.create_transfers(_transfers([dict(id=10 + i, debit_account_id=20 + i,
                                                credit_account_id=1 + i, amount=1000 * (i + 1),
                                                ledger=1, code=1) for i in range(8)]))
            pend = [dict(id=100 + i, debit_account_id=1 + i % 8, credit_account_id=30 + i % 5,
                         amount=50 + i, ledger=1, code=1, flags=2) for i in range(16)]
            p.create_transfers(_transfers(pend))
            next_id = 1000
            for step in range(5):
                rows = []
                for _ in range(600):
                    r = rng.random()
                    dr = int(rng.integers(1, n_acc + 1))
                    cr = int(rng.integers(1, n_acc + 1))
                    if cr == dr:
                        cr = dr % n_acc + 1
                    row = dict(id=next_id, debit_account_id=dr, credit_account_id=cr, ledger=1,
                               code=1, amount=int(rng.choice([10, 300, 2000, 9000, 50_000])))
                    if r < 0.35:
                        row["debit_account_id"] = int(rng.integers(1, 9))  # a limited debit
                        if row["credit_account_id"] == row["debit_account_id"]:
                            row["credit_account_id"] = 20
                    elif r < 0.45:
                        row["credit_account_id"] = int(rng.integers(1, 9))  # credit a limited one
                        if row["credit_account_id"] == row["debit_account_id"]:
                            row["debit_account_id"] = 21
                    elif r < 0.5:
                        row["flags"] = 2  # pending
                    rows.append(row)
                    next_id += 1
                # posts / voids of the limited accounts' pending transfers (some accounts only)
                if step in (1, 3):
                    for i in range(step, 16, 5):
                        rows.insert(int(rng.integers(0, len(rows))),
                                    dict(id=next_id, pending_id=100 + i,
                                         flags=4 if i % 2 else 8, amount=0))
                        next_id += 1
                else:  # a post / void forces the flow replay (no account lanes)
                    rows.insert(0, dict(id=next_id, pending_id=999_999, flags=4, amount=0))
                    next_id += 1
                # in-call duplicate ids (every claimant's credits bound the rule; an uncertain
                # pending transfer turns it off)
                if step % 2 == 0:
                    for _ in range(12):
                        a_i, b_i = rng.integers(0, len(rows), size=2)
                        rows[int(b_i)]["id"] = rows[int(a_i)]["id"]
                # linked chains ending in a limited debit
                for _ in range(30):
                    at = int(rng.integers(0, len(rows) - 4))
                    for j in range(3):
                        rows[at + j]["flags"] = rows[at + j].get("flags", 0) | 1
                p.create_transfers(_transfers(rows), [len(rows) // 2, len(rows) - len(rows) // 2])
            p.compare_state()
        finally:
            p.close()


@pytest.mark.parametrize("mode", ["parallel", "no-pv-fast", "flow"])
def test_later_post_void_claims(mode, monkeypatch):
    """Later posts / voids of a pending transfer whose first post / void in the call is a single
    FAST event fail with already_posted / already_voided without replaying (tr_commit:
    later_claim_status), also inside linked chains (the chain fails there: linked_event_failed for
    the rest); a winner inside a chain (which may roll back), a second winner and duplicate ids
    keep the ordered replay. Every call against the oracle."""
    if mode == "no-pv-fast":
        monkeypatch.setenv("TBG_NO_PV_FAST", "1")
    rng = np.random.default_rng(77)
    p = Pair(account_capacity=256, transfer_capacity=1 << 14, batch_events_max=4096,
             force_replay=mode == "flow")
    try:
        acc = workload.accounts(30, seed=5, ledger=1)
        p.create_accounts(acc)
        pend = [dict(id=100 + i, debit_account_id=1 + i % 30, credit_account_id=1 + (i + 7) % 30,
                     amount=1000 + i, ledger=1, code=1, flags=2) for i in range(300)]
        p.create_transfers(_transfers(pend))
        next_id = 10_000
        for step in range(4):
            rows = []
            for _ in range(500):
                r = rng.random()
                if r < 0.6:  # a post / void of one of a few pending transfers: many later claims
                    x = 100 + int(rng.integers(step * 70, step * 70 + 60))
                    post = rng.random() < 0.6
                    rows.append(dict(id=next_id, pending_id=x, flags=4 if post else 8,
                                     amount=(2**128 - 1) if post else 0))
                else:
                    dr, cr = rng.integers(1, 31, size=2)
                    if dr == cr:
                        cr = dr % 30 + 1
                    rows.append(dict(id=next_id, debit_account_id=int(dr), credit_account_id=int(cr),
                                     amount=int(rng.integers(1, 100)), ledger=1, code=1))
                next_id += 1
            for _ in range(40):  # chains of 2-4 events
                at = int(rng.integers(0, len(rows) - 5))
                for j in range(int(rng.integers(1, 4))):
                    rows[at + j]["flags"] = rows[at + j].get("flags", 0) | 1
            if step == 2:
                for _ in range(8):  # in-call duplicate ids
                    a_i, b_i = rng.integers(0, len(rows), size=2)
                    rows[int(b_i)]["id"] = rows[int(a_i)]["id"]
            p.create_transfers(_transfers(rows), [len(rows) // 3, len(rows) - len(rows) // 3])
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("mode", ["finish", "no-ingest-finish"])
def test_many_small_device_calls(mode, monkeypatch):
    """tbg_create_transfers_device, the body and results in HBM (a replica's per-commit path on
    device buffers): a call whose events are all FAST ends in tr_ingest's last workgroup (the
    counters, the scalars block, the call's scalar words cleared, the sequence word; the queued
    tr_commit and stage_out return at once). 300 small calls, every third one clean, each compared
    with the oracle as it returns; TBG_NO_INGEST_FINISH (tr_commit and stage_out end every call) is
    the control."""
    if mode == "no-ingest-finish":
        monkeypatch.setenv("TBG_NO_INGEST_FINISH", "1")
    rng = np.random.default_rng(37)
    p = Pair(account_capacity=1 << 12, transfer_capacity=1 << 20, batch_events_max=8189,
             device_calls=True)
    try:
        n_acc = 500
        p.create_accounts(workload.accounts(n_acc, seed=4))
        off = 0
        for call in range(300):
            n = int(rng.integers(1, 3000)) if call % 10 else 8189
            t = workload.transfers_uniform(n, n_acc, seed=call, id_offset=off)
            off += n
            if call % 3:
                bad = rng.random(n) < 0.05
                t["id"][bad] = 0
            p.create_transfers(t, _split(n, rng, 8189))
        if mode == "finish":
            assert p.stats["ingest_finished"] >= 90
        else:
            assert p.stats["ingest_finished"] == 0
        p.compare_state()
    finally:
        p.close()
