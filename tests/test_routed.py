"""The routed data path (tigerbeetle_amd/routed.py): the device router, per-shard stamped
execution, results gathered to call order -- against one unsharded oracle, call by call, and the
union of the shards' final tables against the oracle's.

Two ranks on the box's one GPU, over gloo (host staging; RCCL needs one GPU per rank): rank 0
holds the client calls in HBM and the device router; each rank owns two of four ledgers. The
calls take the device path -- interleaved ledgers and fresh ids; a linked chain on one shard,
resubmitted ids (on their holders), posts / voids of pending transfers (on their pending
transfer's shard), with and without a timeout: a post/void of the earliest-expiring one resets
pulse_next_timestamp, resolved across the shards after the call -- except the one the device
router must hand to the exact host router (a transfer between two shards' accounts); pending
transfers expire in sharded pulses. Every shard
records AccountEvents, and the union of the shards' logs must be the oracle's (the ADVICE item:
the appends a device call leaves on the executor's stream read the call's buffers).
"""
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

pytestmark = pytest.mark.gpu

LEDGERS = 4
PER_LEDGER = 200


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _calls(seed):
    """(kind, events, lens) ops; kind "fast" calls are expected on the device path."""
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
    ops.append(("fast", fast1, [8189, 8189, 8189, 30_000 - 3 * 8189]))
    cross = uniform(2_000)
    # (ledgers 1, 2 on shard 0 and 3, 4 on shard 1: the credit account two ledgers over)
    cross["credit_account_id"][5, 0] = ((int(cross["ledger"][5]) + 1) % LEDGERS) * PER_LEDGER + 8
    ops.append(("host", cross, [2_000]))  # a transfer between two shards' accounts
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
    ops.append(("fast", haz, [3_000]))
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
    ops.append(("fast", tpv, [4_000]))
    ops.append(("tick", 2_000_000_000))
    ops.append(("fast", uniform(20_000), [8189, 20_000 - 8189]))
    # a linked chain across the two shards, failing transiently on its second shard: the host
    # engine's chain protocol (probe, the first failure across shards, the orphan kept)
    xc = uniform(1_000)
    for j, lg in zip(range(300, 304), (1, 3, 3, 2)):
        xc["flags"][j] |= 1 if j < 303 else 0
        xc["ledger"][j] = lg
        xc["debit_account_id"][j, 0] = (lg - 1) * PER_LEDGER + 1 + j % 7
        xc["credit_account_id"][j, 0] = (lg - 1) * PER_LEDGER + 20 + j % 5
    xc["debit_account_id"][302, 0] = 999_999  # debit_account_not_found
    ops.append(("host", xc, [1_000]))
    # imported calls (timestamps in a gap before the call, increasing): on the device path above
    # the floor; then with a regress across shards on the host engine
    imp = uniform(3_000)
    imp["flags"] |= 256
    ops.append(("fast-imported", imp, [1_500, 1_500]))
    imp2 = uniform(500)
    imp2["flags"] |= 256
    ops.append(("host-imported", imp2, [500]))
    ops.append(("fast", uniform(5_000), [5_000]))
    return ops


def _rank(rank, world, port, seed, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from test_shard import OracleShard, assert_same_state
        from tigerbeetle_amd import native
        from tigerbeetle_amd.routed import RoutedShards
        from tigerbeetle_amd.types import RESULT_DTYPE, TIMESTAMP_MAX
        o = native.TbgOptions()
        o.account_capacity = 4096
        o.transfer_capacity = 1 << 18
        o.batch_events_max = 1 << 16
        o.batch_count_max = 4096
        o.pulse_batch_max = 8190
        o.device = 0
        o.pulse_next_timestamp_init = TIMESTAMP_MAX
        o.account_events_capacity = 1 << 18
        rs = RoutedShards(o, events_max=1 << 16, router_transfer_capacity=1 << 19,
                          router_account_capacity=4096, ledgers=LEDGERS)
        ref = OracleShard() if rank == 0 else None
        ts, pulses = 0, 0
        for op in _calls(seed):
            if op[0] == "tick":
                ts += op[1]
            else:
                kind, ev, lens = op
                n = len(ev)
                if kind.endswith("-imported"):  # timestamps in a gap before the call
                    ev = ev.copy()
                    ev["timestamp"] = ts + 1 + np.arange(n, dtype=np.uint64)
                    if kind.startswith("host"):
                        ev["timestamp"][[10, 11]] = ev["timestamp"][[11, 10]]  # a regress
                    ts += n
                    kind = kind.split("-")[0]
                ts += 1 + n
                batch_ts = (ts - n + np.cumsum(lens)).astype(np.uint64)
                if kind == "accounts":
                    got = rs.create_accounts(ev, lens, batch_ts) if rank == 0 \
                        else rs.create_accounts()
                    if rank == 0:
                        want = ref.create_accounts(ev, lens, batch_ts)
                        assert got.tobytes() == want.tobytes(), "accounts"
                else:
                    if rank == 0:
                        dev = torch.device("cuda", 0)
                        d_ev = torch.from_numpy(ev.view(np.uint8).copy()).to(dev)
                        d_ends = torch.from_numpy(np.cumsum(lens).astype(np.int32)).to(dev)
                        d_ts = torch.from_numpy(batch_ts.view(np.int64).copy()).to(dev)
                        d_res = torch.zeros(n * 16, dtype=torch.uint8, device=dev)
                        torch.cuda.synchronize()
                        mode = rs.create_transfers(d_ev.data_ptr(), n, d_ends.data_ptr(),
                                                   d_ts.data_ptr(), len(lens), d_res.data_ptr(),
                                                   host_call=(ev, lens, batch_ts))
                        assert mode == (0 if kind == "fast" else 1), (kind, mode)
                        got = d_res.cpu().numpy().view(RESULT_DTYPE)
                        want = ref.create_transfers(ev, lens, batch_ts)
                        if got.tobytes() != want.tobytes():
                            bad = np.nonzero(got != want)[0]
                            raise AssertionError(f"{kind} call: {len(bad)} results differ, first "
                                                 f"{bad[:5].tolist()}: {got[bad[:3]]} vs "
                                                 f"{want[bad[:3]]}")
                    else:
                        rs.create_transfers()
            nxt = rs.pulse_next_timestamp()
            if rank == 0:
                assert nxt == ref.pulse_next_timestamp()
            if nxt <= ts:
                ts += 1 + 8190
                expired = rs.pulse(ts)
                if rank == 0:
                    assert expired == ref.pulse(ts)
                pulses += 1
        dumps = [None] * world
        dist.all_gather_object(dumps, rs.shard.dump())
        events = [None] * world
        dist.all_gather_object(events, rs.shard.dump_account_events())
        if rank == 0:
            assert all(len(d[1]) for d in dumps), "every shard holds transfers"
            assert_same_state(dumps, ref)
            got = np.concatenate(events)
            got = got[np.argsort(got["timestamp"], kind="stable")]
            want = ref.dump_account_events()
            assert len(got) > 50_000 and got.tobytes() == want.tobytes(), \
                f"account events differ ({len(got)} vs {len(want)})"
            assert rs.fast_calls == 6 and rs.host_calls == 3, (rs.fast_calls, rs.host_calls)
            assert pulses > 0
        rs.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, None))
    except BaseException:  # noqa: BLE001 -- reported to the parent
        q.put((rank, traceback.format_exc()))


def test_routed_shards_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, 3, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    try:
        for _ in range(2):
            rank, err = q.get(timeout=240)
            out[rank] = err
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    for rank, err in sorted(out.items()):
        assert err is None, f"rank {rank}:\n{err}"
