"""The exact engine over shards in other processes (tigerbeetle_amd/remote.py): world size 2 over
gloo on the CPU, one oracle shard per rank (test infrastructure, bound through tbo_shard_ops_fill).

Rank 0 owns the group (tbg_group_open_shards over the transport's callbacks) and drives a
cross-shard or a pulse-cut scenario against an unsharded oracle, call by call; rank 1 serves its
shard's operations. Afterwards both ranks' tables, gathered, must be the unsharded tables byte for
byte (test_shard.assert_same_state).
"""
import datetime
import os
import socket
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, case, seed, gpu=False):
    import ctypes

    import torch.distributed as dist

    import oracle_binding
    import test_shard as ts
    from tigerbeetle_amd import remote, shard

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=120))
    try:
        pbm = 6 if case == "pulse_cut" else ts.PBM
        ops = shard.ShardOps()
        if gpu:  # this rank's executor: a HIP executor on cuda:0 (every rank shares the one GPU)
            from tigerbeetle_amd import native
            lib = native.load()
            ctx = lib.tbg_open(ctypes.byref(native.options(
                1 << 12, 1 << 16, 4096, pulse_batch_max=pbm, account_events_capacity=1 << 16)))
            assert ctx, "tbg_open"
            mine = shard.GpuShard.wrap(lib, ctx)
            lib.tbg_group_hip_shard_ops(ctypes.byref(ops))
            self_ptr = ctx
        else:
            mine = ts.OracleShard(pbm)
            oracle_binding.load().tbo_shard_ops_fill(ctypes.byref(ops))
            self_ptr = mine.o
        rs = remote.RemoteShards(ops, self_ptr, ledgers=ts.LEDGERS, pulse_batch_max=pbm)
        if rank == 0:
            ref = ts.OracleShard(pbm)
            g = rs.group
            if case == "pulse_cut":
                cuts = []
                assert ts.drive(g, ref, ts.scenario(seed, calls=10), pbm=pbm, cuts=cuts) > 0
                assert cuts, "the scenario should expire more than pulse_batch_max at once"
            else:
                ts.drive(g, ref, ts.cross_scenario(seed))
                stats = g.stats()
                assert stats["engine_calls"] == stats["calls"] and stats["chain_segments"] > 0
            rs.close()
        else:
            rs.serve()
        dumps = [None] * world
        events = [None] * world
        dist.all_gather_object(dumps, mine.dump())
        dist.all_gather_object(events, mine.dump_account_events())
        if rank == 0:
            assert all(len(d[1]) for d in dumps), "every rank's shard holds transfers"
            ts.assert_same_state(dumps, ref, events)
            ref.close()
        if gpu:
            lib.tbg_close(ctx)
        else:
            mine.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,seed", [("cross", 0), ("cross", 5), ("pulse_cut", 3)])
def test_remote_shards_gloo_world2(case, seed):
    import torch.multiprocessing as mp
    mp.spawn(_rank, args=(2, _port(), case, seed), nprocs=2, join=True)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [2])
def test_remote_hip_shards_gloo_world2(seed):
    """The same transport over HIP executors (tbg_group_hip_shard_ops): each rank opens its own
    executor on cuda:0, rank 0's group reaches rank 1's over gloo."""
    import torch.multiprocessing as mp
    mp.spawn(_rank, args=(2, _port(), "cross", seed, True), nprocs=2, join=True)
