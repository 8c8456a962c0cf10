"""The CPU oracle against the reference's own table tests (src/state_machine_tests.zig).

Every table is replayed through the StateMachine mirror (tb_sm_*, libtbg.so) bound to the oracle
executor, under the reference's unit-test configuration, and each commit's reply must equal the
expected reply byte for byte. This pins the oracle to the reference.
"""
import ctypes

import pytest

import oracle_binding
import tablerun
from tigerbeetle_amd import native
from tigerbeetle_amd.types import TIMESTAMP_MAX


def oracle_handle():
    lib = native.load()
    olib = oracle_binding.load()
    ctx = olib.tbo_open(tablerun.TEST_PULSE_BATCH_MAX, TIMESTAMP_MAX)
    ex = native.Executor()
    olib.tbo_executor_fill(ctx, ctypes.byref(ex))
    sm = lib.tb_sm_open(ctypes.byref(tablerun.sm_options()), ctypes.byref(ex))
    assert sm

    def set_balances(i, dp, dpo, cp, cpo):
        U = native.U128.of
        return olib.tbo_set_account_balances(ctx, U(i), U(dp), U(dpo), U(cp), U(cpo))

    def close():
        lib.tb_sm_close(sm)
        olib.tbo_close(ctx)

    return tablerun.StateMachineHandle(lib, sm, set_balances, close)


@pytest.mark.parametrize("version", list(tablerun.VERSIONS))
@pytest.mark.parametrize("table", tablerun.table_files())
def test_oracle_table(table, version):
    """check(): every table in each client encoding (state_machine_tests.zig:607-619)."""
    rows = tablerun.load_table(f"{tablerun.TABLE_DIR}/{table}")
    h = oracle_handle()
    try:
        tablerun.run_table(h, rows, table, version)
    finally:
        h.close()


def test_tables_cover_every_create_transfer_status():
    seen, seen_accounts = set(), set()
    for table in tablerun.table_files():
        for row in tablerun.load_table(f"{tablerun.TABLE_DIR}/{table}"):
            if row["kind"] == "transfer":
                seen.add(row["status"].name)
            if row["kind"] == "account":
                seen_accounts.add(row["status"].name)
    from tigerbeetle_amd.types import CreateTransferStatus
    expected = {s.name for s in CreateTransferStatus} - {"deprecated_18"}
    # The reference tables exercise linked_event_chain_open on create_accounts only (the same
    # execute_create code path); create_transfers chain_open is covered by the fuzz parity tests.
    assert expected - seen == {"linked_event_chain_open"}
    assert "linked_event_chain_open" in seen_accounts


def test_negative_control_detects_a_wrong_expectation():
    """A corrupted expected status must fail the comparison (the runner really compares)."""
    table = "create_transfers_lookup_transfers__1.txt"
    rows = tablerun.load_table(f"{tablerun.TABLE_DIR}/{table}")
    from tigerbeetle_amd.types import CreateTransferStatus
    for row in rows:
        if row["kind"] == "transfer" and row["status"] == CreateTransferStatus.exceeds_credits:
            row["status"] = CreateTransferStatus.exceeds_debits
            break
    h = oracle_handle()
    try:
        with pytest.raises(tablerun.TableMismatch):
            tablerun.run_table(h, rows, table)
    finally:
        h.close()
