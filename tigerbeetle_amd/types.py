"""Host-side mirror of the extern layouts in src/tigerbeetle.zig (see include/tb_types.h).

u128 fields are two little-endian u64 words ``[lo, hi]``; the numpy record image is byte-identical
to the reference's ``Account`` / ``Transfer`` / ``Create*Result`` (128 / 128 / 16 bytes).
"""
import enum

import numpy as np

U128_MAX = (1 << 128) - 1
U64_MAX = (1 << 64) - 1
TIMESTAMP_MIN = 1
TIMESTAMP_MAX = (1 << 63) - 1  # src/lsm/timestamp_range.zig
NS_PER_S = 1_000_000_000
STATUS_CREATED = 0xFFFFFFFF

_u128 = ("<u8", (2,))

# src/tigerbeetle.zig:10-43
ACCOUNT_DTYPE = np.dtype([
    ("id",) + _u128,
    ("debits_pending",) + _u128,
    ("debits_posted",) + _u128,
    ("credits_pending",) + _u128,
    ("credits_posted",) + _u128,
    ("user_data_128",) + _u128,
    ("user_data_64", "<u8"),
    ("user_data_32", "<u4"),
    ("reserved", "<u4"),
    ("ledger", "<u4"),
    ("code", "<u2"),
    ("flags", "<u2"),
    ("timestamp", "<u8"),
])

# src/tigerbeetle.zig:85-116
TRANSFER_DTYPE = np.dtype([
    ("id",) + _u128,
    ("debit_account_id",) + _u128,
    ("credit_account_id",) + _u128,
    ("amount",) + _u128,
    ("pending_id",) + _u128,
    ("user_data_128",) + _u128,
    ("user_data_64", "<u8"),
    ("user_data_32", "<u4"),
    ("timeout", "<u4"),
    ("ledger", "<u4"),
    ("code", "<u2"),
    ("flags", "<u2"),
    ("timestamp", "<u8"),
])

# src/state_machine.zig:104-220 (AccountEvent)
ACCOUNT_EVENT_DTYPE = np.dtype([
    ("dr_account_id",) + _u128, ("dr_debits_pending",) + _u128, ("dr_debits_posted",) + _u128,
    ("dr_credits_pending",) + _u128, ("dr_credits_posted",) + _u128,
    ("cr_account_id",) + _u128, ("cr_debits_pending",) + _u128, ("cr_debits_posted",) + _u128,
    ("cr_credits_pending",) + _u128, ("cr_credits_posted",) + _u128,
    ("timestamp", "<u8"), ("dr_account_timestamp", "<u8"), ("cr_account_timestamp", "<u8"),
    ("dr_account_flags", "<u2"), ("cr_account_flags", "<u2"), ("transfer_flags", "<u2"),
    ("transfer_pending_flags", "<u2"), ("transfer_pending_id",) + _u128,
    ("amount_requested",) + _u128, ("amount",) + _u128, ("ledger", "<u4"),
    ("transfer_pending_status", "u1"), ("reserved", "u1", (11,)),
])

# src/tigerbeetle.zig:622-670 (ChangeEvent)
CHANGE_EVENT_DTYPE = np.dtype([
    ("transfer_id",) + _u128, ("transfer_amount",) + _u128, ("transfer_pending_id",) + _u128,
    ("transfer_user_data_128",) + _u128, ("transfer_user_data_64", "<u8"),
    ("transfer_user_data_32", "<u4"), ("transfer_timeout", "<u4"), ("transfer_code", "<u2"),
    ("transfer_flags", "<u2"), ("ledger", "<u4"), ("type", "u1"), ("reserved", "u1", (39,)),
    ("debit_account_id",) + _u128, ("debit_account_debits_pending",) + _u128,
    ("debit_account_debits_posted",) + _u128, ("debit_account_credits_pending",) + _u128,
    ("debit_account_credits_posted",) + _u128, ("debit_account_user_data_128",) + _u128,
    ("debit_account_user_data_64", "<u8"), ("debit_account_user_data_32", "<u4"),
    ("debit_account_code", "<u2"), ("debit_account_flags", "<u2"),
    ("credit_account_id",) + _u128, ("credit_account_debits_pending",) + _u128,
    ("credit_account_debits_posted",) + _u128, ("credit_account_credits_pending",) + _u128,
    ("credit_account_credits_posted",) + _u128, ("credit_account_user_data_128",) + _u128,
    ("credit_account_user_data_64", "<u8"), ("credit_account_user_data_32", "<u4"),
    ("credit_account_code", "<u2"), ("credit_account_flags", "<u2"),
    ("timestamp", "<u8"), ("transfer_timestamp", "<u8"), ("debit_account_timestamp", "<u8"),
    ("credit_account_timestamp", "<u8"),
])

# src/tigerbeetle.zig:672-682 (ChangeEventsFilter)
CHANGE_EVENTS_FILTER_DTYPE = np.dtype([("timestamp_min", "<u8"), ("timestamp_max", "<u8"),
                                       ("limit", "<u4"), ("reserved", "u1", (44,))])

# src/tigerbeetle.zig:563-611 (AccountFilter; flags: debits 1, credits 2, reversed 4)
ACCOUNT_FILTER_DTYPE = np.dtype([
    ("account_id", "<u8", (2,)), ("user_data_128", "<u8", (2,)), ("user_data_64", "<u8"),
    ("user_data_32", "<u4"), ("code", "<u2"), ("reserved", "u1", (58,)),
    ("timestamp_min", "<u8"), ("timestamp_max", "<u8"), ("limit", "<u4"), ("flags", "<u4"),
])
# src/tigerbeetle.zig:517-561 (QueryFilter; flags: reversed 1)
QUERY_FILTER_DTYPE = np.dtype([
    ("user_data_128", "<u8", (2,)), ("user_data_64", "<u8"), ("user_data_32", "<u4"),
    ("ledger", "<u4"), ("code", "<u2"), ("reserved", "u1", (6,)), ("timestamp_min", "<u8"),
    ("timestamp_max", "<u8"), ("limit", "<u4"), ("flags", "<u4"),
])
# src/tigerbeetle.zig:70-84 (AccountBalance)
ACCOUNT_BALANCE_DTYPE = np.dtype([
    ("debits_pending", "<u8", (2,)), ("debits_posted", "<u8", (2,)),
    ("credits_pending", "<u8", (2,)), ("credits_posted", "<u8", (2,)), ("timestamp", "<u8"),
    ("reserved", "u1", (56,)),
])

# src/tigerbeetle.zig:471-493
RESULT_DTYPE = np.dtype([("timestamp", "<u8"), ("status", "<u4"), ("reserved", "<u4")])

assert ACCOUNT_DTYPE.itemsize == 128
assert TRANSFER_DTYPE.itemsize == 128
assert RESULT_DTYPE.itemsize == 16
assert ACCOUNT_EVENT_DTYPE.itemsize == 256
assert CHANGE_EVENT_DTYPE.itemsize == 384
assert CHANGE_EVENT_DTYPE.fields["debit_account_id"][1] == 128
assert CHANGE_EVENT_DTYPE.fields["timestamp"][1] == 352
assert CHANGE_EVENTS_FILTER_DTYPE.itemsize == 64


class AccountFlags(enum.IntFlag):
    """src/tigerbeetle.zig:45-68"""
    linked = 1 << 0
    debits_must_not_exceed_credits = 1 << 1
    credits_must_not_exceed_debits = 1 << 2
    history = 1 << 3
    imported = 1 << 4
    closed = 1 << 5


class TransferFlags(enum.IntFlag):
    """src/tigerbeetle.zig:132-148"""
    linked = 1 << 0
    pending = 1 << 1
    post_pending_transfer = 1 << 2
    void_pending_transfer = 1 << 3
    balancing_debit = 1 << 4
    balancing_credit = 1 << 5
    closing_debit = 1 << 6
    closing_credit = 1 << 7
    imported = 1 << 8


class CreateAccountStatus(enum.IntEnum):
    """src/tigerbeetle.zig:153-215"""
    created = 0xFFFFFFFF
    linked_event_failed = 1
    linked_event_chain_open = 2
    imported_event_expected = 22
    imported_event_not_expected = 23
    timestamp_must_be_zero = 3
    imported_event_timestamp_out_of_range = 24
    imported_event_timestamp_must_not_advance = 25
    reserved_field = 4
    reserved_flag = 5
    id_must_not_be_zero = 6
    id_must_not_be_int_max = 7
    exists_with_different_flags = 15
    exists_with_different_user_data_128 = 16
    exists_with_different_user_data_64 = 17
    exists_with_different_user_data_32 = 18
    exists_with_different_ledger = 19
    exists_with_different_code = 20
    exists = 21
    flags_are_mutually_exclusive = 8
    debits_pending_must_be_zero = 9
    debits_posted_must_be_zero = 10
    credits_pending_must_be_zero = 11
    credits_posted_must_be_zero = 12
    ledger_must_not_be_zero = 13
    code_must_not_be_zero = 14
    imported_event_timestamp_must_not_regress = 26


class CreateTransferStatus(enum.IntEnum):
    """src/tigerbeetle.zig:220-320"""
    created = 0xFFFFFFFF
    linked_event_failed = 1
    linked_event_chain_open = 2
    imported_event_expected = 56
    imported_event_not_expected = 57
    timestamp_must_be_zero = 3
    imported_event_timestamp_out_of_range = 58
    imported_event_timestamp_must_not_advance = 59
    reserved_flag = 4
    id_must_not_be_zero = 5
    id_must_not_be_int_max = 6
    exists_with_different_flags = 36
    exists_with_different_pending_id = 40
    exists_with_different_timeout = 44
    exists_with_different_debit_account_id = 37
    exists_with_different_credit_account_id = 38
    exists_with_different_amount = 39
    exists_with_different_user_data_128 = 41
    exists_with_different_user_data_64 = 42
    exists_with_different_user_data_32 = 43
    exists_with_different_ledger = 67
    exists_with_different_code = 45
    exists = 46
    id_already_failed = 68
    flags_are_mutually_exclusive = 7
    debit_account_id_must_not_be_zero = 8
    debit_account_id_must_not_be_int_max = 9
    credit_account_id_must_not_be_zero = 10
    credit_account_id_must_not_be_int_max = 11
    accounts_must_be_different = 12
    pending_id_must_be_zero = 13
    pending_id_must_not_be_zero = 14
    pending_id_must_not_be_int_max = 15
    pending_id_must_be_different = 16
    timeout_reserved_for_pending_transfer = 17
    closing_transfer_must_be_pending = 64
    ledger_must_not_be_zero = 19
    code_must_not_be_zero = 20
    debit_account_not_found = 21
    credit_account_not_found = 22
    accounts_must_have_the_same_ledger = 23
    transfer_must_have_the_same_ledger_as_accounts = 24
    pending_transfer_not_found = 25
    pending_transfer_not_pending = 26
    pending_transfer_has_different_debit_account_id = 27
    pending_transfer_has_different_credit_account_id = 28
    pending_transfer_has_different_ledger = 29
    pending_transfer_has_different_code = 30
    exceeds_pending_transfer_amount = 31
    pending_transfer_has_different_amount = 32
    pending_transfer_already_posted = 33
    pending_transfer_already_voided = 34
    pending_transfer_expired = 35
    imported_event_timestamp_must_not_regress = 60
    imported_event_timestamp_must_postdate_debit_account = 61
    imported_event_timestamp_must_postdate_credit_account = 62
    imported_event_timeout_must_be_zero = 63
    debit_account_already_closed = 65
    credit_account_already_closed = 66
    overflows_debits_pending = 47
    overflows_credits_pending = 48
    overflows_debits_posted = 49
    overflows_credits_posted = 50
    overflows_debits = 51
    overflows_credits = 52
    overflows_timeout = 53
    exceeds_credits = 54
    exceeds_debits = 55
    deprecated_18 = 18


TRANSIENT_TRANSFER_STATUSES = frozenset({
    CreateTransferStatus.debit_account_not_found,
    CreateTransferStatus.credit_account_not_found,
    CreateTransferStatus.pending_transfer_not_found,
    CreateTransferStatus.exceeds_credits,
    CreateTransferStatus.exceeds_debits,
    CreateTransferStatus.debit_account_already_closed,
    CreateTransferStatus.credit_account_already_closed,
})  # src/tigerbeetle.zig:322-399


class Operation(enum.IntEnum):
    """The operations of this path (src/tigerbeetle.zig:685-1004; vsr_operations_reserved = 128)."""
    pulse = 128
    get_change_events = 137
    create_accounts = 146
    create_transfers = 147
    lookup_accounts = 140
    lookup_transfers = 141
    get_account_transfers = 142
    get_account_balances = 143
    query_accounts = 144
    query_transfers = 145


def u128_split(x: int):
    return (x & U64_MAX, (x >> 64) & U64_MAX)


def u128_join(pair) -> int:
    return int(pair[0]) | (int(pair[1]) << 64)


def u128_array_to_int(a: np.ndarray):
    """(n, 2) u64 -> list of Python ints."""
    return [int(lo) | (int(hi) << 64) for lo, hi in a.reshape(-1, 2)]
