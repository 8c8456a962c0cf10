"""Ledger sharding (include/tbg_group.h: the C++ group and its exact engine, csrc/engine.cpp)
against one unsharded executor.

The CPU oracle stands in for every shard here (test infrastructure, bound through the shard
executor interface, tbo_shard_ops_fill). The group must give the unsharded oracle's results call
by call, the same pulse_next_timestamp and pulse counts, and shard tables whose union in
timestamp order is the unsharded tables byte for byte. The GPU tests run the group over two or
three HBM executors on cuda:0.
"""
import ctypes
import os
import sys

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
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        ts = np.ascontiguousarray(batch_ts, dtype=np.uint64)
        fn(self.o, _ptr(events), _ptr(ln), _ptr(ts), len(ln), _ptr(out))
        return out

    def create_accounts(self, events, lens, batch_ts):
        ev = np.ascontiguousarray(events, dtype=ACCOUNT_DTYPE)
        return self._run(self.lib.tbo_create_accounts_batches, ev, lens, batch_ts)

    def create_transfers(self, events, lens, batch_ts):
        ev = np.ascontiguousarray(events, dtype=TRANSFER_DTYPE)
        return self._run(self.lib.tbo_create_transfers_batches, ev, lens, batch_ts)

    def _stamped(self, fn, events, stamps, batch_timestamp, options):
        out = np.zeros(len(events), dtype=RESULT_DTYPE)
        st = np.ascontiguousarray(stamps, dtype=np.uint64)
        fn(self.o, _ptr(events), len(events), _ptr(st), int(batch_timestamp), int(options),
           _ptr(out))
        return out

    def create_accounts_stamped(self, events, stamps, batch_timestamp=0, options=0):
        ev = np.ascontiguousarray(events, dtype=ACCOUNT_DTYPE)
        return self._stamped(self.lib.tbo_create_accounts_stamped, ev, stamps, batch_timestamp,
                             options)

    def create_transfers_stamped(self, events, stamps, batch_timestamp=0, options=0):
        ev = np.ascontiguousarray(events, dtype=TRANSFER_DTYPE)
        return self._stamped(self.lib.tbo_create_transfers_stamped, ev, stamps, batch_timestamp,
                             options)

    def forget_orphans(self, ids):
        a = shard._u128_array(list(ids))
        return int(self.lib.tbo_forget_orphans(self.o, _ptr(a), len(a)))

    def timestamps_exist(self, transfers, ts):
        ts = np.ascontiguousarray(ts, dtype=np.uint64)
        out = np.zeros(len(ts), dtype=np.uint8)
        self.lib.tbo_timestamps_exist(self.o, int(bool(transfers)), _ptr(ts), len(ts), _ptr(out))
        return out.astype(bool)

    def key_max(self):
        a, t = ctypes.c_uint64(), ctypes.c_uint64()
        self.lib.tbo_key_max(self.o, ctypes.byref(a), ctypes.byref(t))
        return int(a.value), int(t.value)

    def _lookup(self, fn, ids, dtype):
        ids = list(ids)
        if not ids:
            return {}
        a = shard._u128_array(ids)
        out = np.zeros(len(ids), dtype=dtype)
        n = int(fn(self.o, _ptr(a), len(ids), _ptr(out)))
        return {int(r["id"][0]) | (int(r["id"][1]) << 64): r for r in out[:n]}

    def lookup_accounts(self, ids):
        return self._lookup(self.lib.tbo_lookup_accounts, ids, ACCOUNT_DTYPE)

    def lookup_transfers(self, ids):
        return self._lookup(self.lib.tbo_lookup_transfers, ids, TRANSFER_DTYPE)

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


def cross_scenario(seed, calls=10, n_acc=60):
    """A call sequence full of what no shard can execute alone (module doc of shard.py): linked
    chains across ledgers (shards) that succeed or fail at every position -- transiently
    (exceeds_credits, accounts / pending transfers not found) or not (ledger mismatch, id 0,
    exists, surrogates for transfers between shards) --, chains left open across shards at batch
    ends, timed pending transfers and their posts / voids inside such chains, ids repeated on
    another shard's accounts within a call (first occurrence created, failed transiently or not),
    account chains across ledgers, imported batches whose timestamps regress across shards,
    collide with the other groove's objects on other shards, advance past the batch, or mismatch
    the batch's imported flag."""
    rng = np.random.default_rng(seed)
    acc = workload.accounts(n_acc, seed=seed)
    ids = np.arange(1, n_acc + 1)
    acc["ledger"] = 1 + (ids - 1) % LEDGERS
    acc["flags"] = rng.choice([0, 0, 2, 4], size=n_acc).astype(np.uint16)
    pools = {lg: ids[acc["ledger"] == lg] for lg in range(1, LEDGERS + 1)}
    ops = [("accounts", acc, _split(rng, n_acc, 24))]
    # an account chain across ledgers with a failure (and one without)
    ach = workload.accounts(6, seed=seed + 1, id_offset=5_000)
    ach["ledger"] = [1, 3, 4, 2, 3, 1]
    ach["flags"] = [1, 1, 1, 0, 1, 0]
    ach["code"][4] = 0  # code_must_not_be_zero: the first chain of two survives, the second fails
    ops.append(("accounts", ach, [6]))
    seen, pend, failed_ids = [], [], []
    next_id = [100_000]

    def fresh():
        next_id[0] += 1
        return next_id[0]

    def plain(t, e, ledger, amount=None):
        dr, cr = rng.choice(pools[ledger], size=2, replace=False)
        t["debit_account_id"][e, 0] = dr
        t["credit_account_id"][e, 0] = cr
        t["amount"][e, 0] = int(rng.integers(1, 300)) if amount is None else amount
        t["ledger"][e] = ledger
        t["code"][e] = 1

    for c in range(calls):
        n = int(rng.integers(60, 140))
        t = np.zeros(n, dtype=TRANSFER_DTYPE)
        k = 0
        while k < n:
            span = min(n - k, int(rng.integers(2, 7)) if rng.random() < 0.45 else 1)
            for j in range(span):
                e = k + j
                ledger = int(rng.integers(1, LEDGERS + 1))
                r = rng.random()
                t["id"][e, 0] = fresh()
                if r < 0.06 and seen:  # an id of an earlier call: exists / id_already_failed
                    t["id"][e, 0] = int(rng.choice(seen + failed_ids))
                    plain(t, e, ledger)
                elif r < 0.12 and e > 0:  # an id of this call, on any ledger
                    t["id"][e, 0] = int(t["id"][int(rng.integers(0, e)), 0])
                    plain(t, e, ledger)
                elif r < 0.18 and pend:  # post / void (maybe of a transfer gone)
                    t["pending_id"][e, 0] = int(rng.choice(pend)) if rng.random() < 0.9 \
                        else 9_999_999
                    t["flags"][e] = 4 if rng.random() < 0.6 else 8
                    if t["flags"][e] == 4:
                        t["amount"][e] = [2**64 - 1, 2**64 - 1]
                elif r < 0.22:  # accounts of two ledgers (two shards, mostly)
                    plain(t, e, ledger)
                    t["credit_account_id"][e, 0] = int(rng.choice(pools[1 + ledger % LEDGERS]))
                elif r < 0.25:
                    plain(t, e, ledger)
                    t["debit_account_id"][e, 0] = 77_777  # debit_account_not_found (transient)
                elif r < 0.28:
                    plain(t, e, ledger)
                    t["ledger"][e] = 1 + ledger % LEDGERS  # not the accounts' ledger
                elif r < 0.30:
                    t["id"][e] = 0
                    plain(t, e, ledger)
                elif r < 0.36:
                    plain(t, e, ledger, amount=10**7)  # exceeds_credits on a limited account
                else:
                    plain(t, e, ledger)
                    if rng.random() < 0.3:
                        t["flags"][e] = 2
                        if rng.random() < 0.6:
                            t["timeout"][e] = int(rng.integers(1, 4))
                        pend.append(int(t["id"][e, 0]))
                if j < span - 1:
                    t["flags"][e] |= 1
            k += span
        if rng.random() < 0.5:
            t["flags"][n - 1] |= 1  # a chain left open at the call's last batch end
        seen.extend(int(x) for x in t["id"][:, 0] if x)
        failed_ids.extend(int(x) for x in t["id"][rng.integers(0, n, size=3), 0] if x)
        ops.append(("transfers", t, _split(rng, n, 40)))
        if c % 3 == 1:
            ops.append(("tick", int(rng.integers(1, 3)) * NS_PER_S))
        if c % 3 == 2:
            ops.extend(_imported_ops(rng, pools, fresh, seed + c))
    return ops


def _imported_ops(rng, pools, fresh, seed):
    """Imported calls (drive's "imported2"): new accounts on every ledger (their timestamps
    collide with the latest transfers), then transfers whose timestamps regress across shards,
    collide with those accounts' timestamps, advance past the batch, or mismatch the batch's
    imported flag."""
    m = 8
    a = workload.accounts(m, seed=seed, id_offset=int(fresh()) * 10)
    a["ledger"] = 1 + np.arange(m) % LEDGERS
    a["flags"] = 16
    a["flags"][int(rng.integers(0, m))] |= 1  # a chain across ledgers (two events)

    def fix_acc(ev, lo, ref):
        ev["timestamp"] = lo + np.arange(len(ev), dtype=np.uint64)
        if ref is not None and rng.random() < 0.7:  # a transfer's timestamp (a later one)
            tr = ref.dump()[1]
            if len(tr):
                j = int(rng.integers(0, len(ev)))
                ev["timestamp"][j] = int(tr["timestamp"][-1 - int(rng.integers(0, min(3, len(tr))))])
        if rng.random() < 0.5:
            ev["timestamp"] = ev["timestamp"][rng.permutation(len(ev))]

    n = 24
    t = np.zeros(n, dtype=TRANSFER_DTYPE)
    for e in range(n):
        ledger = 1 + e % LEDGERS
        dr, cr = rng.choice(pools[ledger], size=2, replace=False)
        t["id"][e, 0] = fresh()
        t["debit_account_id"][e, 0] = dr
        t["credit_account_id"][e, 0] = cr
        t["amount"][e, 0] = int(rng.integers(1, 50))
        t["ledger"][e] = ledger
        t["code"][e] = 1
        t["flags"][e] = 256 | (1 if rng.random() < 0.2 else 0)

    def fix_tr(ev, lo, ref):
        ts = lo + np.arange(len(ev), dtype=np.uint64)
        swap = rng.integers(0, len(ev), size=(4, 2))
        for x, y in swap:
            ts[[x, y]] = ts[[y, x]]
        ev["timestamp"] = ts
        if ref is not None:
            accs = ref.dump()[0]
            j = int(rng.integers(0, len(ev)))
            ev["timestamp"][j] = int(accs["timestamp"][-1 - int(rng.integers(0, 4))])
        ev["timestamp"][int(rng.integers(0, len(ev)))] = (1 << 62)  # must_not_advance
        x = int(rng.integers(1, len(ev)))
        ev["flags"][x] &= ~np.uint16(256)  # imported_event_expected

    return [("imported2", "accounts", a, [m], fix_acc),
            ("imported2", "transfers", t, [12, 12], fix_tr)]


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


def drive(cluster, ref, ops, pbm=PBM, cuts=None, clock=None):
    """Runs `ops` through `cluster` (and `ref`, compared call by call); returns the pulses run.
    Timestamps follow the TestContext rule (prepare_ts += 1 + events, pulses when due). `cuts`
    (a list) collects the pulses that expired exactly pbm transfers (a cut across shards).
    `clock` (a one-element list): the timestamp to start from, and where the last one is left."""
    ts, pulses = (clock[0] if clock else 0), 0
    for op in ops:
        if op[0] == "tick":
            ts += op[1]
        else:
            if op[0] == "imported2":  # timestamps chosen by the op in a gap before the call
                _, kind, ev, lens, fix = op
                lo = ts + 1
                ts += len(ev)
                ev = ev.copy()
                fix(ev, lo, ref)
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
            got = fn(ev, lens, batch_ts)
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
    if clock is not None:
        clock[0] = ts
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


def oracle_group(shards, pbm=PBM, **kw):
    """The C++ group over oracle shards (tbg_group_open_shards)."""
    ops = shard.ShardOps()
    oracle_binding.load().tbo_shard_ops_fill(ctypes.byref(ops))
    return shard.Group.open_shards(ops, [s.o for s in shards], ledgers=LEDGERS,
                                   pulse_batch_max=pbm, **kw)


def gpu_group(n, pbm=PBM, account_capacity=1 << 12, transfer_capacity=1 << 16,
              batch_events_max=4096, account_events_capacity=1 << 16, **kw):
    """The C++ group over `n` HBM executors on cuda:0, and GpuShard views of them (dumps)."""
    from tigerbeetle_amd import native
    opts = [native.options(account_capacity, transfer_capacity, batch_events_max,
                           pulse_batch_max=pbm, account_events_capacity=account_events_capacity)
            for _ in range(n)]
    kw.setdefault("events_max", batch_events_max)
    kw.setdefault("router_transfer_capacity", 1 << 20)
    g = shard.Group.open_gpu(opts, ledgers=LEDGERS, pulse_batch_max=pbm, **kw)
    views = [shard.GpuShard.wrap(g.lib, g.shard(s)) for s in range(n)]
    return g, views


def test_planner_places_and_segments():
    shards = [OracleShard() for _ in range(2)]
    try:
        g = oracle_group(shards)  # ledgers 1, 2 -> shard 0; 3, 4 -> shard 1
        g.record_accounts([1, 2, 3, 4], [0, 0, 1, 1])
        ok = _transfers([dict(id=10, debit_account_id=1, credit_account_id=2, amount=1, ledger=1,
                              code=1),
                         dict(id=11, debit_account_id=3, credit_account_id=4, amount=1, ledger=3,
                              code=1),
                         dict(id=12, debit_account_id=99, credit_account_id=4, amount=1,
                              ledger=3, code=1)])  # missing debit account: the credit's shard
        assert g.plan(True, ok, [3], [20]) == [(0, 3, False, [0, 1, 1])]
        # an existing id goes to its holder, whatever accounts it names
        g.record_transfers([11], [1])
        again = _transfers([dict(id=11, debit_account_id=1, credit_account_id=2, amount=1,
                                 ledger=1, code=1)])
        assert g.plan(True, again, [1], [30]) == [(0, 1, False, [1])]
        # a linked chain across shards: a segment of its own, between the segments around it
        chain = _transfers([
            dict(id=20, debit_account_id=1, credit_account_id=2, amount=1, ledger=1, code=1),
            dict(id=21, debit_account_id=1, credit_account_id=2, amount=1, ledger=1, code=1,
                 flags=1),
            dict(id=22, debit_account_id=3, credit_account_id=4, amount=1, ledger=3, code=1),
            dict(id=23, debit_account_id=3, credit_account_id=4, amount=1, ledger=3, code=1)])
        assert g.plan(True, chain, [4], [50]) == [(0, 1, False, [0]), (1, 3, True, [0, 1]),
                                                  (3, 4, False, [1])]
        # the same events with a batch end between them: two chains (the first one left open)
        assert g.plan(True, chain, [2, 2], [49, 50]) == [(0, 4, False, [0, 0, 1, 1])]
        # an id repeated on another shard's accounts: the repeat waits for the first one's outcome
        rep = _transfers([dict(id=30, debit_account_id=1, credit_account_id=2, amount=1, ledger=1,
                               code=1),
                          dict(id=30, debit_account_id=3, credit_account_id=4, amount=1, ledger=3,
                               code=1)])
        assert g.plan(True, rep, [2], [60]) == [(0, 1, False, [0]), (1, 2, False, [1])]
        # ... but within one chain it runs where the first one did (the chain reaches it only if
        # the first occurrence created the id: create_transfer_exists decides it there)
        rep["flags"][0] = 1
        assert g.plan(True, rep, [2], [60]) == [(0, 2, False, [0, 0])]
        # imported events that may regress past another shard's: a new segment
        imp = _transfers([dict(id=40, debit_account_id=1, credit_account_id=2, amount=1, ledger=1,
                               code=1, flags=256, timestamp=55),
                          dict(id=41, debit_account_id=3, credit_account_id=4, amount=1, ledger=3,
                               code=1, flags=256, timestamp=56)])
        assert len(g.plan(True, imp, [2], [70])) == 1
        imp["timestamp"] = [56, 55]
        assert len(g.plan(True, imp, [2], [70])) == 2
        g.close()
    finally:
        for s in shards:
            s.close()


def test_surrogates_and_batch_statuses():
    """Transfers between two shards' accounts get the reference's status (the surrogate's
    accounts_must_be_different patched), and an imported-flag mismatch the batch's status
    (execute_create :3052-3064) -- against the unsharded oracle."""
    shards = [OracleShard() for _ in range(2)]
    ref = OracleShard()
    try:
        g = oracle_group(shards)
        acc = _accounts([1, 2, 3, 4], [1, 1, 3, 3])
        for c in (g, ref):
            c.create_accounts(acc, [4], [10])
        cross = _transfers([dict(id=13, debit_account_id=1, credit_account_id=3, amount=1,
                                 ledger=1, code=1),
                            dict(id=14, debit_account_id=1, credit_account_id=3, amount=1,
                                 ledger=0, code=1),
                            dict(id=15, debit_account_id=1, credit_account_id=3, amount=1,
                                 ledger=1, code=1, flags=256, timestamp=5),
                            dict(id=16, debit_account_id=1, credit_account_id=2, amount=1,
                                 ledger=1, code=1)])
        got = g.create_transfers(cross, [4], [40])
        want = ref.create_transfers(cross, [4], [40])
        assert got.tobytes() == want.tobytes()
        assert got["status"].tolist() == [23, 19, 57, CREATED]
        g.close()
    finally:
        for s in shards + [ref]:
            s.close()


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_local_shards_match_unsharded(seed):
    shards = [OracleShard() for _ in range(3)]
    ref = OracleShard()
    try:
        g = oracle_group(shards)
        assert drive(g, ref, scenario(seed)) > 0
        dumps = [s.dump() for s in shards]
        assert all(len(d[1]) for d in dumps), "every shard holds transfers"
        assert_same_state(dumps, ref, [s.dump_account_events() for s in shards])
        g.close()
    finally:
        for s in shards + [ref]:
            s.close()


@pytest.mark.parametrize("seed", list(range(8)))
def test_local_shards_cross_shard_calls(seed):
    """cross_scenario through three shards: every call no shard could execute alone, executed
    exactly -- results call by call, pulse_next_timestamp, pulses and the final tables and
    AccountEvents against the unsharded oracle."""
    shards = [OracleShard() for _ in range(3)]
    ref = OracleShard()
    try:
        g = oracle_group(shards)
        drive(g, ref, cross_scenario(seed))
        assert g.stats()["chain_segments"] > 0
        assert_same_state([s.dump() for s in shards], ref,
                          [s.dump_account_events() for s in shards])
        g.close()
    finally:
        for s in shards + [ref]:
            s.close()


@pytest.mark.parametrize("seed", [3, 4])
def test_local_shards_pulse_cut(seed):
    """pulse_batch_max 6: pulses whose expired transfers span shards and exceed the batch take
    the global cut (the 6th key across shards) -- the same transfers, counts and
    pulse_next_timestamp as the unsharded reference."""
    pbm = 6
    shards = [OracleShard(pbm) for _ in range(3)]
    ref = OracleShard(pbm)
    try:
        g = oracle_group(shards, pbm)
        cuts = []
        assert drive(g, ref, scenario(seed, calls=10), pbm=pbm, cuts=cuts) > 0
        assert cuts, "the scenario should expire more than pulse_batch_max at once"
        assert_same_state([s.dump() for s in shards], ref,
                          [s.dump_account_events() for s in shards])
        g.close()
    finally:
        for s in shards + [ref]:
            s.close()


def test_group_lookups_and_errors():
    """Lookups across shards in request order (found objects only); an invalid call fails without
    touching the shards, and the group stays usable."""
    shards = [OracleShard() for _ in range(2)]
    ref = OracleShard()
    try:
        g = oracle_group(shards)
        drive(g, ref, scenario(9, calls=2))
        ids = [5, 9999, 1, 3, 1]
        got = g.lookup_accounts(ids)
        want = ref.lookup_accounts(ids)
        assert [int(r["id"][0]) for r in got] == [5, 1, 3, 1]
        assert all(got[i].tobytes() == want[int(got[i]["id"][0])].tobytes()
                   for i in range(len(got)))
        tids = [1001, 1002, 77, 1003]
        got = g.lookup_transfers(tids)
        want = ref.lookup_transfers(tids)
        assert [int(r["id"][0]) for r in got] == sorted(want, key=tids.index)
        with pytest.raises(ValueError):
            g.create_transfers(np.zeros(2, dtype=TRANSFER_DTYPE), [3], [10**15])
        assert g.pulse_next_timestamp() == ref.pulse_next_timestamp()
        g.close()
    finally:
        for s in shards + [ref]:
            s.close()


@pytest.mark.gpu
def test_local_shards_gpu():
    """Two HBM executors on cuda:0 behind the group, against the unsharded oracle."""
    g, views = gpu_group(2, account_capacity=1 << 10, transfer_capacity=1 << 14)
    ref = OracleShard()
    try:
        assert drive(g, ref, scenario(11)) > 0
        assert_same_state([v.dump() for v in views], ref,
                          [v.dump_account_events() for v in views])
        assert g.stats()["device_calls"] > 0
    finally:
        g.close()
        ref.close()


@pytest.mark.gpu
def test_local_shards_gpu_pulse_cut():
    """Two HBM executors with pulse_batch_max 6: the global pulse cut through tbg_pulse_candidates
    / tbg_pulse_cut, against the unsharded oracle."""
    pbm = 6
    g, views = gpu_group(2, pbm=pbm, account_capacity=1 << 10, transfer_capacity=1 << 14)
    ref = OracleShard(pbm)
    try:
        cuts = []
        assert drive(g, ref, scenario(12, calls=10), pbm=pbm, cuts=cuts) > 0
        assert cuts
        assert_same_state([v.dump() for v in views], ref,
                          [v.dump_account_events() for v in views])
    finally:
        g.close()
        ref.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_local_shards_gpu_cross_shard(seed):
    """cross_scenario through three HBM executors on cuda:0 (the device path where it places a
    call, else the exact engine: stamped calls, TBG_ONE_CHAIN probes and commits,
    tbg_forget_orphans, tbg_timestamps_exist, tbg_key_max), against the unsharded oracle."""
    g, views = gpu_group(3)
    ref = OracleShard()
    try:
        drive(g, ref, cross_scenario(seed))
        st = g.stats()
        assert st["chain_segments"] > 0, st
        assert_same_state([v.dump() for v in views], ref,
                          [v.dump_account_events() for v in views])
    finally:
        g.close()
        ref.close()


def window_scenario(seed, n=150_000, n_acc=2_000, wide=False):
    """Large sharded calls (each shard's part >= 65,536 events over <= 2^14 accounts: the balance
    window path, pnt_resolve on every sharded call): plain transfers (the one-pass AccountEvents
    window), then a call with timed pending transfers (their pulse_next_timestamp minimums resolved
    across shards; AccountEvents from the general path), then plain transfers again, with ticks so
    that pulses expire some of the pending ones. `wide`: the plain calls' amounts log-uniform below
    2^63 (the window's wide layout and the wide one-pass AccountEvents, events.hpp ae_wide_*)."""
    rng = np.random.default_rng(seed)
    acc = workload.accounts(n_acc, seed=seed)
    ids = np.arange(1, n_acc + 1)
    acc["ledger"] = 1 + (ids - 1) % LEDGERS
    acc["flags"] = 0
    pools = {lg: ids[acc["ledger"] == lg] for lg in range(1, LEDGERS + 1)}
    ops = [("accounts", acc, [n_acc])]
    next_id = 10_000_000
    for c, pending in enumerate((0.0, 0.2, 0.0)):
        t = np.zeros(n, dtype=TRANSFER_DTYPE)
        ledger = rng.integers(1, LEDGERS + 1, size=n)
        for lg in range(1, LEDGERS + 1):
            sel = np.nonzero(ledger == lg)[0]
            pair = rng.choice(len(pools[lg]), size=(len(sel), 2))
            pair[:, 1] = (pair[:, 0] + 1 + pair[:, 1] % (len(pools[lg]) - 1)) % len(pools[lg])
            t["debit_account_id"][sel, 0] = pools[lg][pair[:, 0]]
            t["credit_account_id"][sel, 0] = pools[lg][pair[:, 1]]
        t["id"][:, 0] = next_id + np.arange(n)
        next_id += n
        t["amount"][:, 0] = rng.integers(1, 1_000, size=n)
        if wide and not pending:
            t["amount"][:, 0] = workload._amounts(rng, n, amounts="wide")
        t["ledger"] = ledger
        t["code"] = 1
        if pending:
            p = rng.random(n) < pending
            t["flags"][p] = 2
            t["timeout"][p] = rng.integers(1, 4, size=int(p.sum()))
        ops.append(("transfers", t, [8189] * (n // 8189) + ([n % 8189] if n % 8189 else [])))
        ops.append(("tick", 2 * NS_PER_S))
    return ops


@pytest.mark.gpu
@pytest.mark.parametrize("amounts", ["exp", "wide"])
def test_local_shards_gpu_window_calls(amounts):
    """window_scenario through two HBM executors: every shard's part of a call takes the balance
    window and pnt_resolve (sharded calls record every pulse_next_timestamp update); results,
    tables and AccountEvents against the unsharded oracle (pnt_resolve's scratch must
    not be the balance items the AccountEvents window reads). `wide`: amounts below 2^63."""
    g, views = gpu_group(2, transfer_capacity=1 << 19, batch_events_max=1 << 18,
                         account_events_capacity=1 << 20)
    ref = OracleShard()
    try:
        drive(g, ref, window_scenario(3, wide=amounts == "wide"))
        assert_same_state([v.dump() for v in views], ref,
                          [v.dump_account_events() for v in views])
    finally:
        g.close()
        ref.close()


def test_local_shards_batch_cap():
    """A shard's runs of a call whose ledgers interleave event by event become many short batches:
    the engine splits them over sub-calls of at most batch_count_max batches, results and state
    unchanged."""
    shards = [OracleShard() for _ in range(2)]
    ref = OracleShard()
    try:
        g = oracle_group(shards, batch_count_max=64, events_max=1 << 16)
        drive(g, ref, window_scenario(4, n=20_000, n_acc=200))
        assert_same_state([s.dump() for s in shards], ref,
                          [s.dump_account_events() for s in shards])
        g.close()
    finally:
        for s in shards + [ref]:
            s.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 6])
def test_group_checkpoint_gpu(seed, tmp_path):
    """tbg_group_checkpoint / tbg_group_open_checkpoint: half of a cross-shard scenario, every
    shard's image written, the group closed and reopened from the images (the router's
    directories rebuilt from the shards' accounts and transfer ids, orphaned ids included), the
    other half -- results, pulses, tables and AccountEvents against the unsharded oracle, which
    runs straight through."""
    from tigerbeetle_amd import native
    n = 2
    opts = [native.options(1 << 12, 1 << 16, 4096, pulse_batch_max=PBM,
                           account_events_capacity=1 << 16) for _ in range(n)]
    kw = dict(ledgers=LEDGERS, pulse_batch_max=PBM, events_max=4096,
              router_transfer_capacity=1 << 20)
    ops = cross_scenario(seed, calls=12)
    half = len(ops) // 2
    ref = OracleShard()
    g = shard.Group.open_gpu(opts, **kw)
    try:
        clock = [0]
        drive(g, ref, ops[:half], clock=clock)
        paths = [str(tmp_path / f"shard{s}.img") for s in range(n)]
        g.checkpoint(paths)
        g.close()
        g = shard.Group.open_gpu_checkpoint(opts, paths, **kw)
        drive(g, ref, ops[half:], clock=clock)
        views = [shard.GpuShard.wrap(g.lib, g.shard(s)) for s in range(n)]
        assert_same_state([v.dump() for v in views], ref, [v.dump_account_events() for v in views])
    finally:
        g.close()
        ref.close()
