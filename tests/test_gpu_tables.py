"""The HIP executor against the reference's table tests, through the StateMachine mirror.

Same tables and expected replies as test_oracle_tables.py, with tb_sm_open_gpu: the replies of the
MI355X executor must be byte-identical to the reference's expected replies. Run twice: with the
parallel path enabled, and with every event forced through the ordered replay.
"""
import ctypes

import pytest

import tablerun
from tigerbeetle_amd import native
from tigerbeetle_amd.types import TIMESTAMP_MAX

pytestmark = pytest.mark.gpu


def gpu_handle(force_replay: bool, durability=None, tmp_path=None):
    """durability: None, "compact" (tbg_compact after every commit) or "checkpoint" (compact,
    checkpoint, close, and reopen from the image after every commit)."""
    lib = native.load()
    o = native.TbgOptions()
    o.account_capacity = 4096
    o.transfer_capacity = 4096
    o.batch_events_max = 256
    o.batch_count_max = 64
    o.pulse_batch_max = tablerun.TEST_PULSE_BATCH_MAX
    o.device = 0
    o.pulse_next_timestamp_init = TIMESTAMP_MAX
    o.account_events_capacity = 8192  # get_change_events reads the account_events groove
    opts = tablerun.sm_options()
    sm = lib.tb_sm_open_gpu(ctypes.byref(opts), ctypes.byref(o))
    assert sm, "tb_sm_open_gpu failed"

    def debug_modes(g):
        if force_replay:
            lib.tbg_debug_force_replay(g, 1)
        if force_replay == "serial":  # (and the appends on the call's stream: both append paths)
            lib.tbg_debug_serial_replay(g, 1)
            lib.tbg_debug_ae_sync(g, 1)

    debug_modes(lib.tb_sm_executor_gpu(sm))
    h = None

    def set_balances(i, dp, dpo, cp, cpo):
        U = native.U128.of
        return lib.tbg_debug_set_account_balances(lib.tb_sm_executor_gpu(h.sm), U(i), U(dp),
                                                  U(dpo), U(cp), U(cpo))

    def after_commit():
        assert lib.tbg_compact(lib.tb_sm_executor_gpu(h.sm)) >= 0
        if durability == "checkpoint":
            path = str(tmp_path / "sm.tbgckpt").encode()
            assert lib.tb_sm_checkpoint(h.sm, path) == 0
            ts = (lib.tb_sm_get_prepare_timestamp(h.sm), lib.tb_sm_get_commit_timestamp(h.sm),
                  lib.tb_sm_get_prefetch_timestamp(h.sm))
            lib.tb_sm_close(h.sm)
            h.sm = lib.tb_sm_open_gpu_checkpoint(ctypes.byref(opts), ctypes.byref(o), path)
            assert h.sm, "tb_sm_open_gpu_checkpoint failed"
            lib.tb_sm_set_prepare_timestamp(h.sm, ts[0])
            lib.tb_sm_set_commit_timestamp(h.sm, ts[1])
            lib.tb_sm_set_prefetch_timestamp(h.sm, ts[2])
            debug_modes(lib.tb_sm_executor_gpu(h.sm))

    h = tablerun.StateMachineHandle(lib, sm, set_balances, lambda: lib.tb_sm_close(h.sm),
                                    after_commit if durability else None)
    return h


@pytest.mark.parametrize("force_replay", [False, True, "serial"], ids=["parallel", "flow", "serial"])
@pytest.mark.parametrize("table", tablerun.table_files())
def test_gpu_table(table, force_replay):
    rows = tablerun.load_table(f"{tablerun.TABLE_DIR}/{table}")
    h = gpu_handle(force_replay)
    try:
        tablerun.run_table(h, rows, table)
    finally:
        h.close()


@pytest.mark.parametrize("version", ["sparse", "unbatched"])
@pytest.mark.parametrize("table", tablerun.table_files())
def test_gpu_table_deprecated_encodings(table, version):
    """The reference runs every table in each client encoding (check, state_machine_tests.zig
    :607-619): the sparse create results and the unbatched bodies through the HIP executor."""
    rows = tablerun.load_table(f"{tablerun.TABLE_DIR}/{table}")
    h = gpu_handle(False)
    try:
        tablerun.run_table(h, rows, table, version)
    finally:
        h.close()


@pytest.mark.parametrize("durability", ["compact", "checkpoint"])
@pytest.mark.parametrize("table", tablerun.table_files())
def test_gpu_table_durability(table, durability, tmp_path):
    """Every table with the transfer store compacted after every commit, and with the tables
    checkpointed, closed and reopened from the image after every commit (StateMachine.compact /
    checkpoint / open, tb_sm_compact / tb_sm_checkpoint / tb_sm_open_gpu_checkpoint): the replies
    must still be the reference's, byte for byte."""
    rows = tablerun.load_table(f"{tablerun.TABLE_DIR}/{table}")
    h = gpu_handle(False, durability, tmp_path)
    try:
        tablerun.run_table(h, rows, table)
    finally:
        h.close()
