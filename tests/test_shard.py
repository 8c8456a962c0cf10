"""Ledger sharding (tigerbeetle_amd/shard.py) against one unsharded executor.

The CPU oracle stands in for every shard here (test infrastructure). The router and both drivers
-- LocalShards (all shards in one process) and ShardGroup (one shard per rank over
torch.distributed gloo, world_size 2, 127.0.0.1) -- must give the unsharded oracle's results call
by call, the same pulse_next_timestamp and pulse counts, and shard tables whose union in
timestamp order is the unsharded tables byte for byte. The GPU test runs LocalShards over two HBM
executors on cuda:0.
"""
import ctypes
import multiprocessing as mp
import os
import socket
import sys
import traceback

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

from tigerbeetle_amd import shard, workload  # noqa: E402
from tigerbeetle_amd.types import (ACCOUNT_DTYPE, ACCOUNT_EVENT_DTYPE, NS_PER_S, RESULT_DTYPE,  # noqa: E402,E501
                                   TIMESTAMP_MAX, TRANSFER_DTYPE)
import oracle_binding  # noqa: E402

PBM = 8190
LEDGERS = 4
CREATED = 0xFFFFFFFF


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class OracleShard:
    """The CPU oracle behind the shard executor interface (test infrastructure only)."""

    def __init__(self, pbm=PBM):
        self.lib = oracle_binding.load()
        self.o = self.lib.tbo_open(pbm, TIMESTAMP_MAX)

    def close(self):
        if self.o:
            self.lib.tbo_close(self.o)
            self.o = None

    def _run(self, fn, events, lens, batch_ts):
        out = np.zeros(len(events), dtype=RESULT_DTYPE)
        off = 0
        for ln, ts in zip(lens, batch_ts):
            ln = int(ln)
            fn(self.o, _ptr(events[off:off + ln]), ln, int(ts), _ptr(out[off:off + ln]))
            off += ln
        return out

    def create_accounts(self, events, lens, batch_ts):
        ev = np.ascontiguousarray(events, dtype=ACCOUNT_DTYPE)
        return self._run(self.lib.tbo_create_accounts, ev, lens, batch_ts)

    def create_transfers(self, events, lens, batch_ts):
        ev = np.ascontiguousarray(events, dtype=TRANSFER_DTYPE)
        n = int(self.lib.tbo_pnt_ops(self.o, None, None, None))  # (the log starts with this call)
        z = np.zeros(max(n, 1), dtype=np.uint64)
        self.lib.tbo_pnt_ops(self.o, _ptr(z), _ptr(z.copy()), None)
        return self._run(self.lib.tbo_create_transfers, ev, lens, batch_ts)

    def pulse(self, timestamp):
        return int(self.lib.tbo_pulse(self.o, timestamp))

    def pulse_candidates(self, timestamp, max_keys):
        e = np.zeros(max(max_keys, 1), dtype=np.uint64)
        t = np.zeros(max(max_keys, 1), dtype=np.uint64)
        n = int(self.lib.tbo_pulse_candidates(self.o, timestamp, _ptr(e), _ptr(t), max_keys))
        k = min(n, max_keys)
        return n, list(zip(e[:k].tolist(), t[:k].tolist()))

    def pulse_cut(self, timestamp, cut_expires_at, cut_timestamp, pulse_next_timestamp,
                  stamps=None):
        st = None if not stamps else np.ascontiguousarray(stamps, dtype=np.uint64)
        return int(self.lib.tbo_pulse_cut(self.o, timestamp, cut_expires_at, cut_timestamp,
                                          pulse_next_timestamp, None if st is None else _ptr(st)))

    def pulse_next_timestamp(self):
        return int(self.lib.tbo_pulse_next_timestamp(self.o))

    def set_pnt_sharded(self, on):
        self.lib.tbo_pnt_sharded(self.o, 1 if on else 0)

    def pnt_ops(self):
        """The updates recorded since the last create_transfers call began: (start, pairs)."""
        start = ctypes.c_uint64()
        n = int(self.lib.tbo_pnt_ops(self.o, None, None, ctypes.byref(start)))
        ts = np.zeros(max(n, 1), dtype=np.uint64)
        ops = np.zeros(max(n, 1), dtype=np.uint64)
        self.lib.tbo_pnt_ops(self.o, _ptr(ts), _ptr(ops), ctypes.byref(start))
        return int(start.value), list(zip(ts[:n].tolist(), ops[:n].tolist()))

    def set_pulse_next_timestamp(self, value):
        self.lib.tbo_set_pulse_next_timestamp(self.o, int(value))

    def raise_key_max(self, accounts_key_max, transfers_key_max):
        self.lib.tbo_raise_key_max(self.o, accounts_key_max, transfers_key_max)

    def dump(self):
        a = np.zeros(self.lib.tbo_account_count(self.o), dtype=ACCOUNT_DTYPE)
        self.lib.tbo_dump_accounts(self.o, _ptr(a))
        n = self.lib.tbo_transfer_count(self.o)
        t = np.zeros(n, dtype=TRANSFER_DTYPE)
        s = np.zeros(n, dtype=np.uint8)
        self.lib.tbo_dump_transfers(self.o, _ptr(t))
        self.lib.tbo_dump_pending_status(self.o, _ptr(s))
        return a, t, s

    def dump_account_events(self):
        """The oracle's AccountEvents in timestamp order (the groove is keyed by timestamp)."""
        e = np.zeros(self.lib.tbo_dump_account_events(self.o, None), dtype=ACCOUNT_EVENT_DTYPE)
        self.lib.tbo_dump_account_events(self.o, _ptr(e))
        return e[np.argsort(e["timestamp"], kind="stable")]


def _split(rng, n, max_batch):
    lens = []
    while n > 0:
        b = int(min(n, rng.integers(1, max_batch + 1)))
        lens.append(b)
        n -= b
    return lens


def scenario(seed, calls=8, n_acc=48, timed_post_void=True):
    """A call sequence the router can shard: transfers and chains stay within one ledger; with
    resubmitted ids, failing chains, limit failures, missing accounts, chains cut by batch ends,
    pending transfers that expire in pulses, and post/voids of pending transfers -- with a timeout
    too (`timed_post_void`: their reset of pulse_next_timestamp is resolved across shards)."""
    rng = np.random.default_rng(seed)
    acc = workload.accounts(n_acc, seed=seed)
    ids = np.arange(1, n_acc + 1)
    acc["ledger"] = 1 + (ids - 1) % LEDGERS
    acc["flags"] = rng.choice([0, 0, 0, 2, 4], size=n_acc).astype(np.uint16)
    ops = [("accounts", acc, _split(rng, n_acc, 20))]
    dup = acc[:4].copy()
    dup["code"][1] = 9  # exists_with_different_code
    ops.append(("accounts", dup, [4]))
    pools = {lg: ids[acc["ledger"] == lg] for lg in range(1, LEDGERS + 1)}
    untimed, seen = [], []
    next_id = 1_000
    for c in range(calls):
        n = int(rng.integers(150, 350))
        t = np.zeros(n, dtype=TRANSFER_DTYPE)
        k = 0
        while k < n:
            ledger = int(rng.integers(1, LEDGERS + 1))
            span = min(n - k, int(rng.integers(2, 5)) if rng.random() < 0.12 else 1)
            for j in range(span):
                e = k + j
                r = rng.random()
                resubmit = span == 1 and bool(seen) and r < 0.05  # an id of an earlier call
                if resubmit:
                    tid = int(rng.choice(seen))
                else:
                    next_id += 1
                    tid = next_id
                t["id"][e, 0] = tid
                if span == 1 and untimed and r > 0.9:  # post / void
                    t["pending_id"][e, 0] = int(rng.choice(untimed))
                    if rng.random() < 0.6:
                        t["flags"][e] = 4
                        t["amount"][e] = [2**64 - 1, 2**64 - 1]  # the full pending amount
                    else:
                        t["flags"][e] = 8
                else:
                    dr, cr = rng.choice(pools[ledger], size=2, replace=False)
                    if rng.random() < 0.03:
                        dr = n_acc + 100  # debit_account_not_found
                    elif rng.random() < 0.04:  # accounts of two ledgers (often two shards)
                        cr = int(rng.choice(pools[1 + ledger % LEDGERS]))
                    t["debit_account_id"][e, 0] = dr
                    t["credit_account_id"][e, 0] = cr
                    t["amount"][e, 0] = int(rng.integers(1, 500)) if rng.random() < 0.9 else 10**6
                    t["ledger"][e] = ledger
                    t["code"][e] = 1
                    if not resubmit and rng.random() < 0.25:
                        t["flags"][e] = 2
                        if rng.random() < 0.5:
                            t["timeout"][e] = int(rng.integers(1, 3))
                            if timed_post_void:
                                untimed.append(tid)
                        else:
                            untimed.append(tid)
                if j < span - 1:
                    t["flags"][e] |= 1
            k += span
        seen.extend(int(x) for x in t["id"][:, 0])
        ops.append(("transfers", t, _split(rng, n, 64)))
        if c % 2 == 1:
            ops.append(("tick", int(rng.integers(1, 3)) * NS_PER_S))
        if c == calls // 2:  # an imported batch (drive stamps it), some transfers cross-ledger
            m = 40
            imp = np.zeros(m, dtype=TRANSFER_DTYPE)
            for e in range(m):
                ledger = int(rng.integers(1, LEDGERS + 1))
                dr, cr = rng.choice(pools[ledger], size=2, replace=False)
                if rng.random() < 0.1:
                    cr = int(rng.choice(pools[1 + ledger % LEDGERS]))
                next_id += 1
                imp["id"][e, 0] = next_id
                imp["debit_account_id"][e, 0] = dr
                imp["credit_account_id"][e, 0] = cr
                imp["amount"][e, 0] = int(rng.integers(1, 50))
                imp["ledger"][e] = ledger
                imp["code"][e] = 1
                imp["flags"][e] = 256  # imported
            ops.append(("imported", imp, [m]))
    return ops


def drive(cluster, ref, ops, rank0=True, pbm=PBM, cuts=None):
    """Runs `ops` through `cluster` (and `ref`, compared call by call); returns the pulses run.
    Timestamps follow the TestContext rule (prepare_ts += 1 + events, pulses when due). `cuts`
    (a list) collects the pulses that expired exactly pbm transfers (a cut across shards)."""
    ts, pulses = 0, 0
    for op in ops:
        if op[0] == "tick":
            ts += op[1]
        else:
            kind, ev, lens = op
            if kind == "imported":  # timestamps after every object so far, before the batch's
                ev = ev.copy()
                ev["timestamp"] = ts + 1 + np.arange(len(ev), dtype=np.uint64)
                kind = "transfers"
            n = len(ev)
            ts += 1 + n
            batch_ts = (ts - n + np.cumsum(lens)).astype(np.uint64)
            fn = getattr(cluster, "create_" + kind)
            got = fn(ev, lens, batch_ts) if rank0 else fn()
            if ref is not None:
                want = getattr(ref, "create_" + kind)(ev, lens, batch_ts)
                if got.tobytes() != want.tobytes():
                    bad = np.nonzero((got["status"] != want["status"]) |
                                     (got["timestamp"] != want["timestamp"]))[0]
                    raise AssertionError(f"{kind}: {len(bad)} results differ, first at "
                                         f"{bad[:8].tolist()}: {got[bad[:4]]} vs {want[bad[:4]]}")
        nxt = cluster.pulse_next_timestamp()
        if ref is not None:
            assert nxt == ref.pulse_next_timestamp()
        if nxt <= ts:
            ts += 1 + pbm
            expired = cluster.pulse(ts)
            if ref is not None:
                assert expired == ref.pulse(ts)
            if cuts is not None and expired == pbm:
                cuts.append(ts)
            pulses += 1
    return pulses


def assert_same_state(dumps, ref, events=None):
    """The union of the shards' tables in timestamp order equals the unsharded reference's; with
    `events` (each shard's AccountEvents), so does the union of the account_events logs -- an
    expiry's AccountEvent carries its position in the pulse across all shards."""
    a = np.concatenate([d[0] for d in dumps])
    t = np.concatenate([d[1] for d in dumps])
    s = np.concatenate([d[2] for d in dumps])
    oa = np.argsort(a["timestamp"], kind="stable")
    ot = np.argsort(t["timestamp"], kind="stable")
    for got, want, name in zip((a[oa], t[ot], s[ot]), ref.dump(),
                               ("accounts", "transfers", "TransferPending statuses")):
        assert got.tobytes() == want.tobytes(), f"{name} differ ({len(got)} vs {len(want)} rows)"
    if events is not None:
        e = np.concatenate(events)
        e = e[np.argsort(e["timestamp"], kind="stable")]
        want = ref.dump_account_events()
        assert e.tobytes() == want.tobytes(), f"account events differ ({len(e)} vs {len(want)})"


def _accounts(ids, ledgers):
    a = workload.accounts(len(ids), seed=1)
    a["id"][:, 0] = ids
    a["ledger"] = ledgers
    a["flags"] = 0
    return a


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


def _created(n, ts):
    r = np.zeros(n, dtype=RESULT_DTYPE)
    r["status"] = CREATED
    r["timestamp"] = ts
    return r


def test_split_runs_keep_global_timestamps():
    rng = np.random.default_rng(0)
    lens = [7, 1, 12, 5, 30]
    batch_ts = np.array([100, 150, 400, 1000, 5000], dtype=np.uint64)
    n = sum(lens)
    shard_of = rng.integers(0, 3, size=n).astype(np.int32)
    slices = shard.split_runs(shard_of, lens, batch_ts, 3)
    want = np.concatenate([int(ts) - ln + np.arange(1, ln + 1)
                           for ln, ts in zip(lens, batch_ts)])
    got = np.zeros(n, dtype=np.int64)
    for s, sl in enumerate(slices):
        assert (shard_of[sl.index] == s).all()
        off = 0
        for ln, ts in zip(sl.lens, sl.batch_ts):
            got[sl.index[off:off + ln]] = ts - ln + np.arange(1, ln + 1)
            off += ln
        assert off == len(sl.index)
    assert (got == want).all()
    assert sorted(np.concatenate([sl.index for sl in slices]).tolist()) == list(range(n))


def test_router_routes_and_refuses():
    r = shard.LedgerRouter(2, ledgers=4)  # ledgers 1, 2 -> shard 0; 3, 4 -> shard 1
    acc = _accounts([1, 2, 3, 4], [1, 1, 3, 3])
    plan = r.plan_accounts(acc, [4], [10])
    r.commit(plan, acc, _created(4, 10))
    assert r.dir.accounts == {1: 0, 2: 0, 3: 1, 4: 1}
    ok = _transfers([dict(id=10, debit_account_id=1, credit_account_id=2, amount=1, ledger=1, code=1),
                     dict(id=11, debit_account_id=3, credit_account_id=4, amount=1, ledger=3, code=1),
                     dict(id=12, debit_account_id=99, credit_account_id=4, amount=1, ledger=3,
                          code=1)])  # missing debit account: the credit account's shard
    p = r.plan_transfers(ok, [3], [20])
    assert p.shard_of.tolist() == [0, 1, 1]
    assert [sl.lens for sl in p.slices] == [[1], [2]]
    r.commit(p, ok, _created(3, 20))
    # an existing id goes to its holder, whatever accounts it names
    again = _transfers([dict(id=11, debit_account_id=1, credit_account_id=2, amount=1, ledger=1,
                             code=1)])
    assert r.plan_transfers(again, [1], [30]).shard_of.tolist() == [1]
    # accounts on two shards: a surrogate on the debit account's shard, the reference's status
    cross = _transfers([dict(id=13, debit_account_id=1, credit_account_id=3, amount=1, ledger=1,
                             code=1),
                        dict(id=14, debit_account_id=1, credit_account_id=3, amount=1, ledger=0,
                             code=1)])
    p = r.plan_transfers(cross, [2], [40])
    assert p.cross == {0: 23, 1: 19}  # accounts_must_have_the_same_ledger, ledger_must_not_be_zero
    sur = p.shard_events(cross)
    assert (sur["credit_account_id"] == sur["debit_account_id"]).all()
    got = _created(2, 40)
    got["status"] = 12  # the surrogates fail with accounts_must_be_different
    assert p.patch(got)["status"].tolist() == [23, 19]
    chain = _transfers([
        dict(id=14, debit_account_id=1, credit_account_id=2, amount=1, ledger=1, code=1, flags=1),
        dict(id=15, debit_account_id=3, credit_account_id=4, amount=1, ledger=3, code=1)])
    with pytest.raises(shard.RouteError, match="linked chain"):
        r.plan_transfers(chain, [2], [50])
    # the same events with a batch end between them are two chains (the first one left open)
    assert r.plan_transfers(chain, [1, 1], [49, 50]).shard_of.tolist() == [0, 1]
    with pytest.raises(shard.RouteError, match="imported"):  # may collide with an account
        r.plan_transfers(_transfers([dict(id=16, debit_account_id=1, credit_account_id=2,
                                          amount=1, ledger=1, code=1, flags=256,
                                          timestamp=5)]), [1], [60])
    imp = _transfers([dict(id=16, debit_account_id=1, credit_account_id=2, amount=1, ledger=1,
                           code=1, flags=256, timestamp=55),
                      dict(id=17, debit_account_id=3, credit_account_id=4, amount=1, ledger=3,
                           code=1, flags=256, timestamp=56)])
    assert r.plan_transfers(imp, [2], [60]).imported
    imp["timestamp"] = [56, 55]  # the second may regress past the first, on another shard
    with pytest.raises(shard.RouteError, match="regress"):
        r.plan_transfers(imp, [2], [60])
    timed = _transfers([dict(id=17, debit_account_id=1, credit_account_id=2, amount=5, ledger=1,
                             code=1, flags=2, timeout=1)])
    r.commit(r.plan_transfers(timed, [1], [70]), timed, _created(1, 70))
    # a post/void of a pending transfer with a timeout goes to its shard (its reset of
    # pulse_next_timestamp is resolved across shards after the call)
    pv = r.plan_transfers(_transfers([dict(id=18, pending_id=17, flags=4, amount=(1 << 128) - 1)]),
                          [1], [80])
    assert pv.shard_of.tolist() == [0] and pv.post_void
    untimed = _transfers([dict(id=19, debit_account_id=3, credit_account_id=4, amount=5,
                               ledger=3, code=1, flags=2)])
    r.commit(r.plan_transfers(untimed, [1], [90]), untimed, _created(1, 90))
    post = _transfers([dict(id=20, pending_id=19, flags=4, amount=(1 << 128) - 1)])
    assert r.plan_transfers(post, [1], [100]).shard_of.tolist() == [1]


def test_pnt_resets_fire():
    """The reset-if-equal of a post/void (:4227-4229) fires against the value over all shards in
    call order: a `min` recorded by another shard before it can prevent it."""
    R = shard.PNT_RESET
    assert shard.pnt_resets_fire([100, 50], [[], [(10, 50 | R)]])
    assert not shard.pnt_resets_fire([100, 60], [[(5, 40)], [(10, 60 | R)]])
    assert not shard.pnt_resets_fire([100, 60], [[(15, 40)], [(10, 50 | R)]])
    assert shard.pnt_resets_fire([100, 100], [[(5, 40)], [(10, 40 | R)]])


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_local_shards_match_unsharded(seed):
    shards = [OracleShard() for _ in range(3)]
    ref = OracleShard()
    try:
        cluster = shard.LocalShards(shard.LedgerRouter(3, ledgers=LEDGERS), shards, PBM)
        assert drive(cluster, ref, scenario(seed)) > 0
        dumps = [s.dump() for s in shards]
        assert all(len(d[1]) for d in dumps), "every shard holds transfers"
        assert_same_state(dumps, ref, [s.dump_account_events() for s in shards])
    finally:
        for s in shards + [ref]:
            s.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("seed", [3, 4])
def test_local_shards_pulse_cut(seed):
    """pulse_batch_max 6: pulses whose expired transfers span shards and exceed the batch take
    the global cut (the 6th key across shards) -- the same transfers, counts and
    pulse_next_timestamp as the unsharded reference."""
    pbm = 6
    shards = [OracleShard(pbm) for _ in range(3)]
    ref = OracleShard(pbm)
    try:
        cluster = shard.LocalShards(shard.LedgerRouter(3, ledgers=LEDGERS), shards, pbm)
        cuts = []
        assert drive(cluster, ref, scenario(seed, calls=10), pbm=pbm, cuts=cuts) > 0
        assert cuts, "the scenario should expire more than pulse_batch_max at once"
        assert_same_state([s.dump() for s in shards], ref,
                          [s.dump_account_events() for s in shards])
    finally:
        for s in shards + [ref]:
            s.close()


def _gloo_rank(rank, world, port, seed, q, pbm=PBM):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ex = OracleShard(pbm)
        router = shard.LedgerRouter(world, ledgers=LEDGERS) if rank == 0 else None
        group = shard.ShardGroup(ex, router, device="cpu", pulse_batch_max=pbm)
        ref = OracleShard(pbm) if rank == 0 else None
        cuts = []
        pulses = drive(group, ref, scenario(seed, calls=10 if pbm < PBM else 8),
                       rank0=rank == 0, pbm=pbm, cuts=cuts)
        if rank == 0 and pbm < PBM:
            assert cuts, "the scenario should expire more than pulse_batch_max at once"
        dumps = [None] * world
        dist.all_gather_object(dumps, ex.dump())
        events = [None] * world
        dist.all_gather_object(events, ex.dump_account_events())
        if rank == 0:
            assert all(len(d[1]) for d in dumps), "every shard holds transfers"
            assert_same_state(dumps, ref, events)
        # A refused call fails on every rank and leaves the group usable.
        chain = _transfers([
            dict(id=10**9, debit_account_id=1, credit_account_id=5, amount=1, ledger=1, code=1,
                 flags=1),
            dict(id=10**9 + 1, debit_account_id=3, credit_account_id=7, amount=1, ledger=3,
                 code=1)])
        try:
            if rank == 0:
                group.create_transfers(chain, [2], np.array([10**15], dtype=np.uint64))
            else:
                group.create_transfers()
            raise AssertionError("the cross-shard chain was not refused")
        except shard.RouteError:
            pass
        assert group.pulse_next_timestamp() > 0
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, None, pulses))
    except BaseException:  # noqa: BLE001 -- reported to the parent
        q.put((rank, traceback.format_exc(), 0))


@pytest.mark.parametrize("pbm", [PBM, 6], ids=["pbm8190", "pbm6-cuts"])
def test_shard_group_gloo_world2(pbm):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_rank, args=(r, 2, port, 5, q, pbm)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(2):
            rank, err, pulses = q.get(timeout=240)
            out[rank] = (err, pulses)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, (err, _) in sorted(out.items()):
        assert err is None, f"rank {rank}:\n{err}"
    assert out[0][1] > 0


@pytest.mark.gpu
def test_local_shards_gpu():
    """Two HBM executors on cuda:0 behind the router, against the unsharded oracle."""
    shards = [shard.GpuShard(1 << 10, 1 << 14, batch_events_max=4096,
                             account_events_capacity=1 << 15) for _ in range(2)]
    ref = OracleShard()
    try:
        cluster = shard.LocalShards(shard.LedgerRouter(2, ledgers=LEDGERS), shards, PBM)
        assert drive(cluster, ref, scenario(11)) > 0
        assert_same_state([s.dump() for s in shards], ref,
                          [s.dump_account_events() for s in shards])
    finally:
        for s in shards:
            s.close()
        ref.close()


@pytest.mark.gpu
def test_local_shards_gpu_pulse_cut():
    """Two HBM executors with pulse_batch_max 6: the global pulse cut through tbg_pulse_candidates
    / tbg_pulse_cut, against the unsharded oracle."""
    pbm = 6
    shards = [shard.GpuShard(1 << 10, 1 << 14, batch_events_max=4096, pulse_batch_max=pbm,
                             account_events_capacity=1 << 15) for _ in range(2)]
    ref = OracleShard(pbm)
    try:
        cluster = shard.LocalShards(shard.LedgerRouter(2, ledgers=LEDGERS), shards, pbm)
        cuts = []
        assert drive(cluster, ref, scenario(12, calls=10), pbm=pbm, cuts=cuts) > 0
        assert cuts
        assert_same_state([s.dump() for s in shards], ref,
                          [s.dump_account_events() for s in shards])
    finally:
        for s in shards:
            s.close()
        ref.close()
