"""The routed data path of the group (include/tbg_group.h): the device router, per-shard stamped
execution, results gathered to call order -- against one unsharded oracle, call by call, and the
union of the shards' final tables and AccountEvents against the oracle's.

One process owns two executors on the box's one GPU (the group's shards; on a node, one per GPU):
the client calls are in HBM on the router's GPU (tbg_group_create_transfers_device), some come as
host buffers (tbg_group_create_transfers). Each call is expected on a path -- the device path
(interleaved ledgers and fresh ids; a linked chain on one shard; resubmitted ids on their holders;
posts / voids of pending transfers on their pending transfer's shard, with and without a timeout:
a post/void of the earliest-expiring one resets pulse_next_timestamp, resolved across the shards
after the call; a transfer between the two shards' accounts as a surrogate; events whose status
follows from themselves alone; ids repeated within the call on one shard) or the exact engine (a
linked chain across the two shards failing transiently on its second shard, an imported call
regressing across shards, an id repeated on the other shard's accounts); pending transfers expire
in sharded pulses.
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


LEDGERS = 4
PER_LEDGER = 200


def _calls(seed):
    """(kind, events, lens) ops; kind "device" / "engine": the path the call is expected on
    ("-host": passed as host buffers, "-imported": imported timestamps in a gap before the call)."""
    from tigerbeetle_amd import workload
    from tigerbeetle_amd.types import TRANSFER_DTYPE
    rng = np.random.default_rng(seed)
    acc = workload.accounts(LEDGERS * PER_LEDGER, seed=seed)
    k = np.arange(LEDGERS * PER_LEDGER)
    acc["ledger"] = 1 + k // PER_LEDGER
    acc["flags"] = rng.choice([0, 0, 0, 2], size=len(acc)).astype(np.uint16)
    ops = [("accounts", acc, [len(acc)])]
    next_id = 10_000

    def uniform(n, pending_frac=0.0):
        nonlocal next_id
        t = np.zeros(n, dtype=TRANSFER_DTYPE)
        lg = rng.integers(0, LEDGERS, size=n)
        dr = rng.integers(0, PER_LEDGER, size=n)
        cr = (dr + 1 + rng.integers(0, PER_LEDGER - 1, size=n)) % PER_LEDGER
        t["id"][:, 0] = next_id + 1 + np.arange(n)
        next_id += n
        t["debit_account_id"][:, 0] = lg * PER_LEDGER + dr + 1
        t["credit_account_id"][:, 0] = lg * PER_LEDGER + cr + 1
        t["amount"][:, 0] = rng.integers(1, 1000, size=n)
        t["ledger"] = lg + 1
        t["code"] = 1
        pend = rng.random(n) < pending_frac
        t["flags"][pend] = 2
        t["timeout"][pend] = rng.integers(0, 3, size=int(pend.sum()))
        return t

    fast1 = uniform(30_000, pending_frac=0.1)
    ops.append(("device", fast1, [8189, 8189, 8189, 30_000 - 3 * 8189]))
    cross = uniform(2_000)
    # (ledgers 1, 2 on shard 0 and 3, 4 on shard 1: the credit account two ledgers over)
    for j in (5, 77, 78, 901):
        cross["credit_account_id"][j, 0] = ((int(cross["ledger"][j]) + 1) % LEDGERS) * \
            PER_LEDGER + 8
    cross["ledger"][77] = 0        # ledger_must_not_be_zero (patched in)
    cross["timeout"][78] = 5       # timeout_reserved_for_pending_transfer (patched in)
    cross["flags"][900:902] = 1, 0  # ... in a linked chain (failing it)
    cross["debit_account_id"][900] = cross["debit_account_id"][901]
    cross["credit_account_id"][900, 0] = int(cross["debit_account_id"][901, 0]) % PER_LEDGER + 1 + \
        (int(cross["debit_account_id"][901, 0]) - 1) // PER_LEDGER * PER_LEDGER
    cross["ledger"][900] = cross["ledger"][901]
    ops.append(("device-host", cross, [2_000]))  # transfers between two shards' accounts
    haz = uniform(3_000)
    haz["flags"][10:13] |= 1  # a chain (same ledger: set its accounts)
    for j in range(10, 14):
        haz["ledger"][j] = 1
        haz["debit_account_id"][j, 0] = 1 + j
        haz["credit_account_id"][j, 0] = 50 + j
    haz["id"][100:110] = fast1["id"][200:210]  # resubmitted: exists on their holders
    untimed = fast1["id"][(fast1["flags"] == 2) & (fast1["timeout"] == 0), 0][:20]
    for j, pid in enumerate(untimed):  # posts / voids of untimed pending transfers
        e = 200 + j
        haz["pending_id"][e, 0] = pid
        haz["flags"][e] = 4 if j % 2 else 8
        haz["amount"][e] = [2**64 - 1, 2**64 - 1] if j % 2 else [0, 0]
        haz["debit_account_id"][e] = 0
        haz["credit_account_id"][e] = 0
        haz["ledger"][e] = 0
        haz["code"][e] = 0
        haz["timeout"][e] = 0
    ops.append(("device", haz, [3_000]))
    # posts / voids of pending transfers with a timeout, the earliest-expiring one first (its
    # expiry is pulse_next_timestamp: the reset fires), among new pending transfers and transfers
    timed_ids = fast1["id"][(fast1["flags"] == 2) & (fast1["timeout"] == 1), 0][:40]
    tpv = uniform(4_000, pending_frac=0.2)
    for j, pid in enumerate(timed_ids):
        e = 50 + 37 * j
        tpv["pending_id"][e, 0] = pid
        tpv["flags"][e] = 8 if j % 3 == 0 else 4
        tpv["amount"][e] = [0, 0] if j % 3 == 0 else [2**64 - 1, 2**64 - 1]
        tpv["debit_account_id"][e] = 0
        tpv["credit_account_id"][e] = 0
        tpv["ledger"][e] = 0
        tpv["code"][e] = 0
        tpv["timeout"][e] = 0
    ops.append(("device", tpv, [4_000]))
    ops.append(("tick", 2_000_000_000))
    ops.append(("device", uniform(20_000), [8189, 20_000 - 8189]))
    # events whose status follows from themselves alone, unknown accounts, posts / voids of
    # pending transfers found nowhere, ids repeated within the call on one shard: the device path
    bad = uniform(6_000)
    bad["flags"][10] |= 1 << 12                       # reserved_flag
    bad["id"][11] = 0                                 # id_must_not_be_zero
    bad["id"][12] = [2**64 - 1, 2**64 - 1]            # id_must_not_be_int_max
    bad["timestamp"][13] = 99                         # timestamp_must_be_zero
    bad["debit_account_id"][14, 0] = 555_555          # debit_account_not_found (transient)
    bad["credit_account_id"][15, 0] = 555_556         # credit_account_not_found
    bad["debit_account_id"][16, 0] = 555_557          # both unknown
    bad["credit_account_id"][16, 0] = 555_558
    bad["flags"][17] = 4                              # post of a pending transfer found nowhere
    bad["pending_id"][17, 0] = 424_242
    bad["id"][300] = bad["id"][20]                    # repeats of created ids (exists*)
    bad["debit_account_id"][300] = bad["debit_account_id"][20]
    bad["credit_account_id"][300] = bad["credit_account_id"][20]
    bad["ledger"][300] = bad["ledger"][20]
    bad["amount"][300, 0] = 1                         # exists_with_different_amount
    bad["id"][301] = bad["id"][14]                    # repeat of an orphaned id: id_already_failed
    bad["debit_account_id"][301] = bad["debit_account_id"][14]
    bad["credit_account_id"][301] = bad["credit_account_id"][14]
    bad["ledger"][301] = bad["ledger"][14]
    bad["id"][302] = bad["id"][11]                    # id 0 again
    bad["flags"][400:403] = 1, 1, 0                   # a chain with an unknown account (fails)
    for j in (400, 401, 402):
        bad["ledger"][j] = 2
        bad["debit_account_id"][j, 0] = PER_LEDGER + 3 + j % 5
        bad["credit_account_id"][j, 0] = PER_LEDGER + 10 + j % 3
    bad["credit_account_id"][401, 0] = 777_777
    ops.append(("device", bad, [3_000, 3_000]))
    rep = uniform(2_000)
    rep["id"][900] = rep["id"][100]                   # an id repeated on the other shard's accounts
    rep["ledger"][900] = 1 + (int(rep["ledger"][100]) + 1) % LEDGERS
    rep["debit_account_id"][900, 0] = (int(rep["ledger"][900]) - 1) * PER_LEDGER + 1
    rep["credit_account_id"][900, 0] = (int(rep["ledger"][900]) - 1) * PER_LEDGER + 2
    rep["debit_account_id"][100, 0] = 888_888        # (the first occurrence fails: not found)
    ops.append(("engine", rep, [2_000]))
    # a linked chain across the two shards, failing transiently on its second shard: the host
    # engine's chain protocol (probe, the first failure across shards, the orphan kept)
    xc = uniform(1_000)
    for j, lg in zip(range(300, 304), (1, 3, 3, 2)):
        xc["flags"][j] |= 1 if j < 303 else 0
        xc["ledger"][j] = lg
        xc["debit_account_id"][j, 0] = (lg - 1) * PER_LEDGER + 1 + j % 7
        xc["credit_account_id"][j, 0] = (lg - 1) * PER_LEDGER + 20 + j % 5
    xc["debit_account_id"][302, 0] = 999_999  # debit_account_not_found
    ops.append(("engine", xc, [1_000]))
    # imported calls (timestamps in a gap before the call, increasing): on the device path above
    # the floor; then with a regress across shards on the host engine
    imp = uniform(3_000)
    imp["flags"] |= 256
    ops.append(("device-imported", imp, [1_500, 1_500]))
    imp2 = uniform(500)
    imp2["flags"] |= 256
    ops.append(("engine-imported", imp2, [500]))
    ops.append(("device-host", uniform(5_000), [5_000]))
    return ops


@pytest.mark.gpu
def test_group_routed_device_path():
    """Every routed call's scatter stores each shard's slice into that shard's own buffers and
    settle reads the results from there (tbr_route_device_slices) -- the transport shards on other
    GPUs take (stores and loads across xGMI), here on one GPU."""
    from hipmem import Hip
    from test_shard import OracleShard, assert_same_state
    from tigerbeetle_amd import native, shard
    from tigerbeetle_amd.types import RESULT_DTYPE, TIMESTAMP_MAX
    opts = [native.options(4096, 1 << 18, 1 << 16, pulse_next_timestamp_init=TIMESTAMP_MAX,
                           account_events_capacity=1 << 18) for _ in range(2)]
    g = shard.Group.open_gpu(opts, ledgers=LEDGERS, events_max=1 << 16,
                             router_transfer_capacity=1 << 19, router_account_capacity=4096)
    views = [shard.GpuShard.wrap(g.lib, g.shard(s)) for s in range(2)]
    ref = OracleShard()
    hip = Hip(0)
    ts, pulses = 0, 0
    try:
        for i, op in enumerate(_calls(3)):
            if op[0] == "tick":
                ts += op[1]
            else:
                kind, ev, lens = op
                n = len(ev)
                if kind.endswith("-imported"):  # timestamps in a gap before the call
                    ev = ev.copy()
                    ev["timestamp"] = ts + 1 + np.arange(n, dtype=np.uint64)
                    if kind.startswith("engine"):
                        ev["timestamp"][[10, 11]] = ev["timestamp"][[11, 10]]  # a regress
                    ts += n
                ts += 1 + n
                batch_ts = (ts - n + np.cumsum(lens)).astype(np.uint64)
                if kind == "accounts":
                    got = g.create_accounts(ev, lens, batch_ts)
                    want = ref.create_accounts(ev, lens, batch_ts)
                    assert got.tobytes() == want.tobytes(), "accounts"
                    continue
                before = g.stats()
                if kind.endswith("-host"):
                    got = g.create_transfers(ev, lens, batch_ts)
                else:
                    got = _group_call(g, hip, ev, lens, batch_ts)
                after = g.stats()
                path = "device" if after["device_calls"] > before["device_calls"] else "engine"
                assert path == kind.split("-")[0], (i, kind, path)
                want = ref.create_transfers(ev, lens, batch_ts)
                if got.tobytes() != want.tobytes():
                    bad = np.nonzero(got != want)[0]
                    raise AssertionError(f"{kind} call: {len(bad)} results differ, first "
                                         f"{bad[:5].tolist()}: {got[bad[:3]]} vs "
                                         f"{want[bad[:3]]}")
            nxt = g.pulse_next_timestamp()
            assert nxt == ref.pulse_next_timestamp()
            if nxt <= ts:
                ts += 1 + 8190
                assert g.pulse(ts) == ref.pulse(ts)
                pulses += 1
        dumps = [v.dump() for v in views]
        assert all(len(d[1]) for d in dumps), "every shard holds transfers"
        events = [v.dump_account_events() for v in views]
        assert sum(len(e) for e in events) > 50_000
        assert_same_state(dumps, ref, events)
        st = g.stats()
        assert st["surrogates"] >= 4 and st["anywhere"] >= 8 and st["repeats"] >= 2, st
        assert pulses > 0
    finally:
        g.close()
        ref.close()
        hip.free_all()


def _group_call(g, hip, t, lens, batch_ts):
    """One tbg_group_create_transfers_device call (the call's buffers on the router's GPU)."""
    from tigerbeetle_amd.types import RESULT_DTYPE
    n = len(t)
    d_ev = hip.upload(t)
    d_ends = hip.upload(np.cumsum(lens).astype(np.uint32))
    d_ts = hip.upload(np.ascontiguousarray(batch_ts, dtype=np.uint64))
    d_res = hip.zeros(n * 16)
    g.create_transfers_device(d_ev, n, d_ends, d_ts, len(lens), d_res)
    out = hip.download(d_res, np.zeros(n, dtype=RESULT_DTYPE))
    hip.free_all()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [2, 3])
def test_group_hazard_calls_on_device(shards):
    """Calls of mixed-ledger transfers with injected failures across ledgers (bench.py's
    `hazard_call`: unknown accounts, cross-ledger accounts, id 0, reserved flags, posts of pending
    transfers found nowhere, exact repeats) stay on the device path: exact against the oracle and
    against the closed form the bench validates with; the balances match."""
    from hipmem import Hip
    from test_shard import OracleShard
    from tigerbeetle_amd import native, shard, workload
    from tigerbeetle_amd.types import TIMESTAMP_MAX
    L, P, n = shards, 5_000, 200_000
    opts = [native.options(L * P, 1 << 20, n, pulse_next_timestamp_init=TIMESTAMP_MAX)
            for _ in range(shards)]
    g = shard.Group.open_gpu(opts, ledgers=L + 1, events_max=n, router_transfer_capacity=1 << 21,
                             router_account_capacity=L * P + 16)
    ref = OracleShard()
    hip = Hip(0)
    try:
        acc = workload.group_accounts(L, P, seed=5)
        lens = [len(acc)]
        assert (g.create_accounts(acc, lens, [len(acc) + 1])["status"] == 0xFFFFFFFF).all()
        ref.create_accounts(acc, lens, [len(acc) + 1])
        ts = len(acc) + 1
        for step in range(3):
            t, kinds, src = workload.hazard_transfers(n, L, P, rate=0.002, seed=10 + step,
                                                      id_offset=step * n)
            lens = [8189] * (n // 8189) + [n % 8189]
            batch_ts = (ts + np.cumsum(np.asarray(lens) + 1)).astype(np.uint64)
            ts = int(batch_ts[-1])
            before = g.stats()
            got = _group_call(g, hip, t, lens, batch_ts)
            after = g.stats()
            assert after["device_calls"] == before["device_calls"] + 1, "device path"
            want = ref.create_transfers(t, lens, batch_ts)
            assert got.tobytes() == want.tobytes(), np.nonzero(got != want)[0][:8]
            stamps = (np.repeat(batch_ts - np.asarray(lens, np.uint64), lens) +
                      np.arange(n, dtype=np.uint64) -
                      np.repeat(np.cumsum(lens) - lens, lens).astype(np.uint64) + np.uint64(1))
            st, tts, _ = workload.hazard_expected(t, kinds, src, stamps, L)
            assert (got["status"] == st).all() and (got["timestamp"] == tts).all()
        ids = np.arange(1, L * P + 1)
        got = g.lookup_accounts(ids)
        want = ref.lookup_accounts(ids)
        assert len(got) == L * P
        assert all(got[i].tobytes() == want[int(got[i]["id"][0])].tobytes()
                   for i in range(0, L * P, 97))
    finally:
        g.close()
        ref.close()
        hip.free_all()


def test_hazard_expected_closed_form():
    """The closed form bench.py validates its hazard calls with equals the oracle's serial
    results (CPU, unsharded)."""
    from test_shard import OracleShard
    from tigerbeetle_amd import workload
    from tigerbeetle_amd.types import TIMESTAMP_MAX  # noqa: F401
    ref = OracleShard()
    try:
        L, P, n = 3, 500, 20_000
        acc = workload.group_accounts(L, P, seed=2)
        ref.create_accounts(acc, [len(acc)], [len(acc) + 1])
        t, kinds, src = workload.hazard_transfers(n, L, P, rate=0.01, seed=4)
        lens = [8189, 8189, n - 2 * 8189]
        batch_ts = (len(acc) + 1 + np.cumsum(np.asarray(lens) + 1)).astype(np.uint64)
        want = ref.create_transfers(t, lens, batch_ts)
        stamps = (np.repeat(batch_ts - np.asarray(lens, np.uint64), lens) +
                  np.arange(n, dtype=np.uint64) -
                  np.repeat(np.cumsum(lens) - lens, lens).astype(np.uint64) + np.uint64(1))
        st, tts, created = workload.hazard_expected(t, kinds, src, stamps, L)
        assert (want["status"] == st).all() and (want["timestamp"] == tts).all()
        assert (kinds >= 0).sum() == n // 100 and created.sum() == n - n // 100
    finally:
        ref.close()


@pytest.mark.gpu
def test_group_slice_capacity():
    """A call whose part for one shard exceeds that shard's batch_events_max fails with EINVAL
    before anything is scattered (its id claims released); the group stays usable and exact."""
    from hipmem import Hip
    from test_shard import OracleShard
    from tigerbeetle_amd import native, shard, workload
    from tigerbeetle_amd.types import TIMESTAMP_MAX
    opts = [native.options(4096, 1 << 16, 1000, pulse_next_timestamp_init=TIMESTAMP_MAX)
            for _ in range(2)]
    g = shard.Group.open_gpu(opts, ledgers=3, events_max=4000, router_transfer_capacity=1 << 16,
                             router_account_capacity=4096)
    ref = OracleShard()
    hip = Hip(0)
    try:
        acc = workload.group_accounts(2, 500, seed=1)
        for c in (g, ref):
            c.create_accounts(acc, [len(acc)], [len(acc) + 1])
        t, _ = workload.mixed_ledger_transfers(3000, 2, 500, seed=2, id_offset=10_000)
        t["ledger"] = 2  # every event on ledger 2's shard: 3,000 > its 1,000
        t["debit_account_id"][:, 0] = t["debit_account_id"][:, 0] % 500 + 1
        t["credit_account_id"][:, 0] = (t["debit_account_id"][:, 0]) % 500 + 1
        with pytest.raises(RuntimeError, match="-22"):
            _group_call(g, hip, t, [3000], np.asarray([5000], np.uint64))
        ok, _ = workload.mixed_ledger_transfers(1500, 2, 500, seed=3, id_offset=20_000)
        got = _group_call(g, hip, ok, [1500], np.asarray([7000], np.uint64))
        want = ref.create_transfers(ok, [1500], [7000])
        assert got.tobytes() == want.tobytes()
        # the refused call's ids were released: the same ids, resubmitted within limits, create
        t2 = t[:900].copy()
        got = _group_call(g, hip, t2, [900], np.asarray([9000], np.uint64))
        want = ref.create_transfers(t2, [900], [9000])
        assert got.tobytes() == want.tobytes() and (got["status"] == 0xFFFFFFFF).all()
    finally:
        g.close()
        ref.close()
        hip.free_all()
