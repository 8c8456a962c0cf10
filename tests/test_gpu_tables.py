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


def gpu_handle(force_replay: bool):
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
    sm = lib.tb_sm_open_gpu(ctypes.byref(tablerun.sm_options()), ctypes.byref(o))
    assert sm, "tb_sm_open_gpu failed"
    g = lib.tb_sm_executor_gpu(sm)
    if force_replay:
        lib.tbg_debug_force_replay(g, 1)
    if force_replay == "serial":
        lib.tbg_debug_serial_replay(g, 1)

    def set_balances(i, dp, dpo, cp, cpo):
        U = native.U128.of
        return lib.tbg_debug_set_account_balances(g, U(i), U(dp), U(dpo), U(cp), U(cpo))

    return tablerun.StateMachineHandle(lib, sm, set_balances, lambda: lib.tb_sm_close(sm))


@pytest.mark.parametrize("force_replay", [False, True, "serial"], ids=["parallel", "flow", "serial"])
@pytest.mark.parametrize("table", tablerun.table_files())
def test_gpu_table(table, force_replay):
    rows = tablerun.load_table(f"{tablerun.TABLE_DIR}/{table}")
    h = gpu_handle(force_replay)
    try:
        tablerun.run_table(h, rows, table)
    finally:
        h.close()
