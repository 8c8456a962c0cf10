"""The reference's table tests through the StateMachine mirror bound to an executor group.

tb_sm_open over tbg_group_executor (include/tbg_group.h): the StateMachine over N shards, as a
replica over a node's GPUs would run it. Two shards, ledger 1 on shard 0 and
ledger 2 on shard 1 (the tables' ledgers), so every table that names both ledgers crosses shards:
transfers between them (accounts_must_have_the_same_ledger through the router's surrogate),
linked chains across them (the exact engine's chain protocol), pulses and lookups over both. The
replies must be byte-identical to the reference's expected replies -- the same tables as
test_oracle_tables.py / test_gpu_tables.py.

CPU: the group over two oracle shards (the exact engine only; the scans and get_change_events,
which merge the shards' scans, need HIP shards and are skipped). GPU: over two HBM executors on
cuda:0 (the device path and the exact engine), every table.
"""
import ctypes

import pytest

import tablerun
from tigerbeetle_amd import native, shard
from tigerbeetle_amd.types import TIMESTAMP_MAX

SCANS = ("get_account_balances", "get_account_transfers", "get_change_events", "query_")


def group_handle(gpu: bool):
    lib = native.load()
    opts = tablerun.sm_options()
    kw = dict(ledgers=2, events_max=256, batch_count_max=64,
              pulse_batch_max=tablerun.TEST_PULSE_BATCH_MAX, router_account_capacity=4096,
              router_transfer_capacity=1 << 16)
    if gpu:
        shard_opts = [native.options(4096, 4096, 256, batch_count_max=64,
                                     pulse_batch_max=tablerun.TEST_PULSE_BATCH_MAX,
                                     pulse_next_timestamp_init=TIMESTAMP_MAX,
                                     account_events_capacity=8192) for _ in range(2)]
        g = shard.Group.open_gpu(shard_opts, **kw)
        shards = [g.shard(s) for s in range(2)]
        oracles = []

        def set_one(s, i, dp, dpo, cp, cpo):
            U = native.U128.of
            return lib.tbg_debug_set_account_balances(s, U(i), U(dp), U(dpo), U(cp), U(cpo))
    else:
        import oracle_binding
        from test_shard import OracleShard
        oracles = [OracleShard(tablerun.TEST_PULSE_BATCH_MAX) for _ in range(2)]
        ops = shard.ShardOps()
        olib = oracle_binding.load()
        olib.tbo_shard_ops_fill(ctypes.byref(ops))
        g = shard.Group.open_shards(ops, [o.o for o in oracles], **kw)
        shards = [o.o for o in oracles]

        def set_one(s, i, dp, dpo, cp, cpo):
            U = native.U128.of
            return olib.tbo_set_account_balances(s, U(i), U(dp), U(dpo), U(cp), U(cpo))
    ex = g.executor()
    sm = lib.tb_sm_open(ctypes.byref(opts), ctypes.byref(ex))
    assert sm, "tb_sm_open failed"

    def set_balances(i, dp, dpo, cp, cpo):
        # (the test harness' setup action: the account lives on one shard)
        return 0 if any(set_one(s, i, dp, dpo, cp, cpo) == 0 for s in shards) else -1

    def close():
        lib.tb_sm_close(h.sm)
        g.close()
        for o in oracles:
            o.close()

    h = tablerun.StateMachineHandle(lib, sm, set_balances, close)
    h.group = g
    return h


@pytest.mark.parametrize("table", tablerun.table_files())
def test_group_table_oracle_shards(table):
    if table.startswith(SCANS):
        pytest.skip("scans over a group merge the HIP shards' scans")
    rows = tablerun.load_table(f"{tablerun.TABLE_DIR}/{table}")
    h = group_handle(False)
    try:
        tablerun.run_table(h, rows, table)
    finally:
        h.close()


@pytest.mark.gpu
@pytest.mark.parametrize("table", tablerun.table_files())
def test_group_table_gpu(table):
    rows = tablerun.load_table(f"{tablerun.TABLE_DIR}/{table}")
    h = group_handle(True)
    try:
        tablerun.run_table(h, rows, table)
    finally:
        h.close()
