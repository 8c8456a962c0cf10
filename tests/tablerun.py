"""Table-test runner: the reference's state-machine table DSL and TestContext, restated in Python.

Follows src/testing/table.zig (row DSL) and src/state_machine_tests.zig:37-1086 (TestContext,
TestAction, check_version for the dense `create_*` operation encoding). Each table row is an input
event with its expected result; `commit <op>` submits the accumulated batch through a StateMachine
(tb_sm_*, include/tb_state_machine.h) and compares the reply byte-for-byte with the expected reply
derived by the harness rules (:704-735, :757-811).

The StateMachine under test is bound to an executor: the CPU oracle (oracle/liboracle.so) or the
HIP executor (libtbg.so). get_change_events (the account_events groove read back as
ChangeEvents, :2396-2434, :3395-3527) is checked with the reference's own `match` rules
(TestGetChangeEventsResult, :502-599). The scans -- get_account_transfers, get_account_balances,
query_accounts, query_transfers (TestAccountFilter / TestQueryFilter, :468-494, :863-1002) -- are
submitted multi-batch encoded, one filter per commit, and their replies compared byte for byte.
"""
import ctypes
import os
import struct
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tigerbeetle_amd import native  # noqa: E402
from tigerbeetle_amd.types import (  # noqa: E402
    ACCOUNT_DTYPE, CHANGE_EVENT_DTYPE, CHANGE_EVENTS_FILTER_DTYPE, RESULT_DTYPE, TRANSFER_DTYPE,
    CreateAccountStatus, CreateTransferStatus, Operation, TIMESTAMP_MAX, U128_MAX, NS_PER_S,
    ACCOUNT_BALANCE_DTYPE, ACCOUNT_FILTER_DTYPE, QUERY_FILTER_DTYPE)

TABLE_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "tables")

# The reference's unit-test configuration (config.zig test_min + state_machine_tests.zig:123):
# message_size_max = 4096 -> message_body_size_max = 3840; batch_size_limit = 30 * 128.
TEST_MESSAGE_BODY_SIZE_MAX = 4096 - 256
TEST_BATCH_SIZE_LIMIT = 30 * 128
# batch_max.create_transfers = max(event_max) over the create_transfers encodings
# = message_body_size_max / 128 (the unbatched encoding) = 30.
TEST_PULSE_BATCH_MAX = TEST_MESSAGE_BODY_SIZE_MAX // 128

SKIPPED_OPS = set()

# TestContext.Operation.versions (state_machine_tests.zig:59-95): every table runs once per client
# encoding -- the dense multi-batch operations, the sparse create results (multi-batch), and the
# deprecated unbatched bodies. Per table operation: (operation number, event size, result size,
# multi-batch encoded).
VERSIONS = {
    "dense": {
        "create_accounts": (146, 128, 16, True), "create_transfers": (147, 128, 16, True),
        "lookup_accounts": (140, 16, 128, True), "lookup_transfers": (141, 16, 128, True),
        "get_account_transfers": (142, 128, 128, True),
        "get_account_balances": (143, 128, 128, True),
        "query_accounts": (144, 64, 128, True), "query_transfers": (145, 64, 128, True),
    },
    "sparse": {
        "create_accounts": (138, 128, 8, True), "create_transfers": (139, 128, 8, True),
        "lookup_accounts": (140, 16, 128, True), "lookup_transfers": (141, 16, 128, True),
        "get_account_transfers": (142, 128, 128, True),
        "get_account_balances": (143, 128, 128, True),
        "query_accounts": (144, 64, 128, True), "query_transfers": (145, 64, 128, True),
    },
    "unbatched": {
        "create_accounts": (129, 128, 8, False), "create_transfers": (130, 128, 8, False),
        "lookup_accounts": (131, 16, 128, False), "lookup_transfers": (132, 16, 128, False),
        "get_account_transfers": (133, 128, 128, False),
        "get_account_balances": (134, 128, 128, False),
        "query_accounts": (135, 64, 128, False), "query_transfers": (136, 64, 128, False),
    },
}
SCAN_OPS = ("get_account_transfers", "get_account_balances", "query_accounts", "query_transfers")


# ---- row DSL (src/testing/table.zig) --------------------------------------------------------

class Tokens:
    def __init__(self, toks):
        self.toks = toks
        self.i = 0

    def next(self):
        t = self.toks[self.i]
        self.i += 1
        return t

    def peek(self):
        return self.toks[self.i] if self.i < len(self.toks) else None

    def eat(self, t):
        if self.peek() == t:
            self.i += 1
            return True
        return False


def parse_uint(tok: str, bits: int) -> int:
    off = 1 if tok[0].isalpha() else 0
    body = tok[off:]
    mx = (1 << bits) - 1
    if body.startswith("-"):
        return mx - int(body[1:])
    v = int(body)
    assert 0 <= v <= mx, tok
    return v


def parse_int(tok: str) -> int:
    off = 1 if tok[0].isalpha() else 0
    return int(tok[off:])


# Field specs: (name, kind, default). kind: ("u", bits) | ("flag", NAME) | ("status",)
ACCOUNT_FIELDS = [
    ("id", ("u", 128), None), ("debits_pending", ("u", 128), 0), ("debits_posted", ("u", 128), 0),
    ("credits_pending", ("u", 128), 0), ("credits_posted", ("u", 128), 0),
    ("user_data_128", ("u", 128), 0), ("user_data_64", ("u", 64), 0),
    ("user_data_32", ("u", 32), 0), ("reserved", ("u", 1), 0), ("ledger", ("u", 32), None),
    ("code", ("u", 16), None), ("LNK", ("flag", "LNK"), 0), ("D<C", ("flag", "D<C"), 0),
    ("C<D", ("flag", "C<D"), 0), ("HIST", ("flag", "HIST"), 0), ("IMP", ("flag", "IMP"), 0),
    ("CLSD", ("flag", "CLSD"), 0), ("padding", ("u", 10), 0), ("timestamp", ("u", 64), 0),
]
ACCOUNT_FLAG_BITS = {"LNK": 0, "D<C": 1, "C<D": 2, "HIST": 3, "IMP": 4, "CLSD": 5}

TRANSFER_FIELDS = [
    ("id", ("u", 128), None), ("debit_account_id", ("u", 128), None),
    ("credit_account_id", ("u", 128), None), ("amount", ("u", 128), 0),
    ("pending_id", ("u", 128), 0), ("user_data_128", ("u", 128), 0),
    ("user_data_64", ("u", 64), 0), ("user_data_32", ("u", 32), 0), ("timeout", ("u", 32), 0),
    ("ledger", ("u", 32), None), ("code", ("u", 16), None), ("LNK", ("flag", "LNK"), 0),
    ("PEN", ("flag", "PEN"), 0), ("POS", ("flag", "POS"), 0), ("VOI", ("flag", "VOI"), 0),
    ("BDR", ("flag", "BDR"), 0), ("BCR", ("flag", "BCR"), 0), ("IMP", ("flag", "IMP"), 0),
    ("CDR", ("flag", "CDR"), 0), ("CCR", ("flag", "CCR"), 0), ("padding", ("u", 5), 0),
    ("timestamp", ("u", 64), 0),
]
TRANSFER_FLAG_BITS = {"LNK": 0, "PEN": 1, "POS": 2, "VOI": 3, "BDR": 4, "BCR": 5, "CDR": 6,
                      "CCR": 7, "IMP": 8}


def parse_fields(tokens: Tokens, spec):
    out = {}
    for name, kind, default in spec:
        if default is not None and tokens.eat("_"):
            out[name] = default
            continue
        tok = tokens.next()
        if kind[0] == "u":
            out[name] = parse_uint(tok, kind[1])
        elif kind[0] == "flag":
            assert tok == kind[1], (tok, kind)
            out[name] = 1
    return out


def parse_row(line: str):
    toks = line.split()
    if not toks:
        return None
    t = Tokens(toks)
    kind = t.next()
    row = {"kind": kind}
    if kind == "account":
        row.update(parse_fields(t, ACCOUNT_FIELDS))
        row["status"] = CreateAccountStatus[t.next()]
    elif kind == "transfer":
        row.update(parse_fields(t, TRANSFER_FIELDS))
        row["status"] = CreateTransferStatus[t.next()]
    elif kind == "setup":
        row["account"] = parse_uint(t.next(), 128)
        for f in ("debits_pending", "debits_posted", "credits_pending", "credits_posted"):
            row[f] = parse_uint(t.next(), 128)
    elif kind == "tick":
        row["value"] = parse_int(t.next())
        row["unit"] = t.next()
        assert row["unit"] in ("nanoseconds", "seconds")
    elif kind == "commit":
        row["operation"] = t.next()
    elif kind == "lookup_account":
        row["id"] = parse_uint(t.next(), 128)
        if t.eat("_"):
            row["data"] = None
        else:
            d = {}
            for f in ("debits_pending", "debits_posted", "credits_pending", "credits_posted"):
                d[f] = parse_uint(t.next(), 128)
            if t.eat("_"):
                d["closed"] = False
            else:
                assert t.next() == "CLSD"
                d["closed"] = True
            row["data"] = d
    elif kind == "lookup_transfer":
        row["id"] = parse_uint(t.next(), 128)
        variant = t.next()
        tok = t.next()
        if variant == "exists":
            row["data"] = ("exists", tok in ("1", "true", "T"))
        elif variant == "amount":
            row["data"] = ("amount", parse_uint(tok, 128))
        elif variant == "timestamp":
            row["data"] = ("timestamp", parse_uint(tok, 64))
        else:
            raise ValueError(line)
    elif kind == "get_change_events":
        # TestGetChangeEventsFilter (:496-500): optional transfer ids for the timestamp bounds
        row["min"] = None if t.eat("_") else parse_uint(t.next(), 128)
        row["max"] = None if t.eat("_") else parse_uint(t.next(), 128)
        row["limit"] = parse_uint(t.next(), 32)
    elif kind == "get_change_events_result":
        # TestGetChangeEventsResult (:502-517)
        row["event_type"] = None if t.eat("_") else t.next()
        row["timestamp_transfer"] = None if t.eat("_") else parse_uint(t.next(), 128)
        row["amount"] = parse_uint(t.next(), 128)
        row["pending_id"] = None if t.eat("_") else parse_uint(t.next(), 128)
        for side in ("dr", "cr"):
            b = {"account_id": parse_uint(t.next(), 128)}
            for f in ("debits_pending", "debits_posted", "credits_pending", "credits_posted"):
                b[f] = parse_uint(t.next(), 128)
            b["closed"] = False if t.eat("_") else (t.next() == "CLSD")
            row[side] = b
    elif kind in ("get_account_balances", "get_account_transfers"):
        # TestAccountFilter (:468-482)
        row["account_id"] = parse_uint(t.next(), 128)
        for f, bits in (("user_data_128", 128), ("user_data_64", 64), ("user_data_32", 32),
                        ("code", 16)):
            row[f] = 0 if t.eat("_") else parse_uint(t.next(), bits)
        row["min"] = None if t.eat("_") else parse_uint(t.next(), 128)
        row["max"] = None if t.eat("_") else parse_uint(t.next(), 128)
        row["limit"] = parse_uint(t.next(), 32)
        for flag in ("DR", "CR", "REV"):
            row[flag] = not t.eat("_")
            if row[flag]:
                assert t.next() == flag, line
    elif kind in ("query_accounts", "query_transfers"):
        # TestQueryFilter (:484-494)
        for f, bits in (("user_data_128", 128), ("user_data_64", 64), ("user_data_32", 32),
                        ("ledger", 32), ("code", 16)):
            row[f] = parse_uint(t.next(), bits)
        row["min"] = None if t.eat("_") else parse_uint(t.next(), 128)
        row["max"] = None if t.eat("_") else parse_uint(t.next(), 128)
        row["limit"] = parse_uint(t.next(), 32)
        row["REV"] = not t.eat("_")
        if row["REV"]:
            assert t.next() == "REV", line
    elif kind == "get_account_balances_result":
        row["transfer_id"] = parse_uint(t.next(), 128)
        for f in ("debits_pending", "debits_posted", "credits_pending", "credits_posted"):
            row[f] = parse_uint(t.next(), 128)
    elif kind in ("get_account_transfers_result", "query_transfers_result"):
        row["id"] = parse_uint(t.next(), 128)
    elif kind == "query_accounts_result":
        row["id"] = parse_uint(t.next(), 128)
        if t.eat("_"):
            row["data"] = None
        else:
            d = {}
            for f in ("debits_pending", "debits_posted", "credits_pending", "credits_posted"):
                d[f] = parse_uint(t.next(), 128)
            d["closed"] = False if t.eat("_") else (t.next() == "CLSD")
            row["data"] = d
    elif kind.split("_result")[0] in SKIPPED_OPS or kind in SKIPPED_OPS:
        row["kind"] = "skip"
        row["op"] = kind
        return row
    else:
        raise ValueError(f"unknown row: {line}")
    rest = t.peek()
    assert rest is None or rest == "//", line
    return row


def load_table(path: str):
    rows = []
    for line in open(path):
        line = line.rstrip("\n")
        if line.startswith("#"):
            continue
        r = parse_row(line)
        if r is not None:
            rows.append(r)
    return rows


def table_files():
    return sorted(f for f in os.listdir(TABLE_DIR) if f.endswith(".txt"))


# ---- event images -----------------------------------------------------------------------------

def _set_u128(rec, name, v):
    rec[name][0] = v & 0xFFFFFFFFFFFFFFFF
    rec[name][1] = v >> 64


def account_event(r) -> np.ndarray:
    a = np.zeros(1, dtype=ACCOUNT_DTYPE)[0]
    for f in ("id", "debits_pending", "debits_posted", "credits_pending", "credits_posted",
              "user_data_128"):
        _set_u128(a, f, r[f])
    a["user_data_64"] = r["user_data_64"]
    a["user_data_32"] = r["user_data_32"]
    a["reserved"] = r["reserved"]
    a["ledger"] = r["ledger"]
    a["code"] = r["code"]
    flags = r["padding"] << 6
    for name, bit in ACCOUNT_FLAG_BITS.items():
        if r[name]:
            flags |= 1 << bit
    a["flags"] = flags
    a["timestamp"] = r["timestamp"]
    return a


def transfer_event(r) -> np.ndarray:
    t = np.zeros(1, dtype=TRANSFER_DTYPE)[0]
    for f in ("id", "debit_account_id", "credit_account_id", "amount", "pending_id",
              "user_data_128"):
        _set_u128(t, f, r[f])
    t["user_data_64"] = r["user_data_64"]
    t["user_data_32"] = r["user_data_32"]
    t["timeout"] = r["timeout"]
    t["ledger"] = r["ledger"]
    t["code"] = r["code"]
    flags = r["padding"] << 9
    for name, bit in TRANSFER_FLAG_BITS.items():
        if r[name]:
            flags |= 1 << bit
    t["flags"] = flags
    t["timestamp"] = r["timestamp"]
    return t


def u128_of(rec, name) -> int:
    return int(rec[name][0]) | (int(rec[name][1]) << 64)


# ---- StateMachine harness (TestContext, state_machine_tests.zig:37-285) ------------------------

class StateMachineHandle:
    """A tb_sm bound to an executor, plus the executor's `setup` hook."""

    def __init__(self, lib, sm, set_balances, close, after_commit=None):
        self.lib = lib
        self.sm = sm
        self.set_balances = set_balances
        self._close = close
        # Optional hook run after every commit; it may replace self.sm (checkpoint + reopen).
        self.after_commit = after_commit
        self.output = ctypes.create_string_buffer(TEST_MESSAGE_BODY_SIZE_MAX + 256)

    def close(self):
        self._close()


def encode_multi_batch(lib, payload: bytes, element_size: int) -> bytes:
    n = len(payload) // element_size
    trailer = lib.tb_multi_batch_trailer_total_size(element_size, 1)
    buf = ctypes.create_string_buffer(len(payload) + trailer + 2)
    ctypes.memmove(buf, payload, len(payload))
    counts = (ctypes.c_uint16 * 1)(n)
    size = lib.tb_multi_batch_encode_trailer(buf, len(payload), element_size, counts, 1)
    assert size > 0
    return buf.raw[:size]


def decode_multi_batch_single(lib, body: bytes, element_size: int) -> bytes:
    counts = (ctypes.c_uint16 * 8)()
    payload = ctypes.c_uint32(0)
    nb = lib.tb_multi_batch_decode(body, len(body), element_size, counts, 8,
                                   ctypes.byref(payload))
    assert nb == 1, nb
    return body[:payload.value]


class TableContext:
    def __init__(self, handle: StateMachineHandle):
        self.h = handle
        self.lib = handle.lib
        self.sm = handle.sm
        self.op = 1
        self._cb = native.PREFETCH_CALLBACK(lambda ctx: None)

    # TestContext.prepare (:230-241)
    def prepare(self, operation: int, body: bytes):
        lib, sm = self.lib, self.sm
        lib.tb_sm_set_commit_timestamp(sm, lib.tb_sm_get_prepare_timestamp(sm))
        lib.tb_sm_set_prepare_timestamp(sm, lib.tb_sm_get_prepare_timestamp(sm) + 1)
        lib.tb_sm_prepare(sm, operation, body, len(body))

    # TestContext.execute (:258-285)
    def execute(self, operation: int, body: bytes) -> bytes:
        lib, sm = self.lib, self.sm
        timestamp = lib.tb_sm_get_prepare_timestamp(sm)
        lib.tb_sm_set_prefetch_timestamp(sm, timestamp)
        lib.tb_sm_prefetch(sm, self._cb, None, self.op, self.op, operation, body, len(body))
        size = lib.tb_sm_commit(sm, 1, 0, self.op, timestamp, operation, body, len(body),
                                self.h.output)
        assert size >= 0, f"commit failed: {size}"
        return self.h.output.raw[:size]

    # TestContext.pulse (:243-256)
    def pulse(self):
        lib, sm = self.lib, self.sm
        if lib.tb_sm_pulse_needed(sm, lib.tb_sm_get_prepare_timestamp(sm)):
            self.prepare(Operation.pulse, b"")
            size = self.execute(Operation.pulse, b"")
            assert len(size) == 0
            self.op += 1

    def submit_query(self, operation: int, body: bytes) -> bytes:
        """A non-multi-batch operation (get_change_events): the body is the filter itself."""
        assert self.lib.tb_sm_input_valid(self.sm, operation, body, len(body)) == 1
        self.prepare(operation, body)
        pulse_needed = self.lib.tb_sm_pulse_needed(self.sm,
                                                   self.lib.tb_sm_get_prepare_timestamp(self.sm))
        reply = self.execute(operation, body)
        if pulse_needed:
            self.pulse()
        return reply

    # TestContext.submit (:178-228)
    def submit(self, operation: int, payload: bytes, element_size: int, result_size: int,
               multi_batch: bool = True) -> bytes:
        body = encode_multi_batch(self.lib, payload, element_size) if multi_batch else payload
        assert self.lib.tb_sm_input_valid(self.sm, operation, body, len(body)) == 1
        self.prepare(operation, body)
        pulse_needed = self.lib.tb_sm_pulse_needed(self.sm,
                                                   self.lib.tb_sm_get_prepare_timestamp(self.sm))
        reply = self.execute(operation, body)
        if pulse_needed:
            self.pulse()
        if not multi_batch:
            return reply
        return decode_multi_batch_single(self.lib, reply, result_size)


class TableMismatch(AssertionError):
    pass


def run_table(handle: StateMachineHandle, rows, label="", version="dense"):
    """check_version (state_machine_tests.zig:620-1086) for one client encoding (VERSIONS)."""
    ops = VERSIONS[version]
    dense = version == "dense"
    ctx = TableContext(handle)
    lib, sm = ctx.lib, ctx.sm
    accounts = {}
    transfers = {}
    linked_events_failed = {}
    request = []
    reply = []
    operation = None
    commits = 0

    for row in rows:
        kind = row["kind"]
        if kind == "skip":
            operation = "skip"
            continue
        if kind == "setup":
            assert operation is None
            rc = handle.set_balances(row["account"], row["debits_pending"], row["debits_posted"],
                                     row["credits_pending"], row["credits_posted"])
            assert rc == 0, f"setup of unknown account {row['account']}"
        elif kind == "tick":
            interval = abs(row["value"]) * (1 if row["unit"] == "nanoseconds" else NS_PER_S)
            pts = lib.tb_sm_get_prepare_timestamp(sm)
            pts += interval if row["value"] > 0 else TIMESTAMP_MAX - interval
            lib.tb_sm_set_prepare_timestamp(sm, pts & 0xFFFFFFFFFFFFFFFF)
            ctx.pulse()
        elif kind == "account":
            assert operation in (None, "create_accounts")
            operation = "create_accounts"
            event = account_event(row)
            request.append(event.tobytes())
            timestamp_commit = lib.tb_sm_get_prepare_timestamp(sm) + 1 + len(request)
            if event["timestamp"] == 0:
                event["timestamp"] = timestamp_commit
            status = row["status"]
            if status == CreateAccountStatus.created:
                accounts[row["id"]] = event.copy()
            if status in (CreateAccountStatus.created, CreateAccountStatus.linked_event_failed):
                ts = int(event["timestamp"])
            elif status == CreateAccountStatus.exists:
                ts = int(accounts[row["id"]]["timestamp"]) if row["id"] in accounts \
                    else linked_events_failed[row["id"]]
            else:
                ts = timestamp_commit
            if dense:
                reply.append(struct.pack("<QII", ts, int(status), 0))
            elif status != CreateAccountStatus.created:  # CreateAccountErrorResult (:738-746)
                reply.append(struct.pack("<II", len(request) - 1, int(status)))
            if row["LNK"]:
                if status == CreateAccountStatus.linked_event_failed:
                    assert row["id"] not in linked_events_failed
                    linked_events_failed[row["id"]] = int(event["timestamp"])
            else:
                linked_events_failed.clear()
        elif kind == "transfer":
            assert operation in (None, "create_transfers")
            operation = "create_transfers"
            event = transfer_event(row)
            request.append(event.tobytes())
            timestamp_commit = lib.tb_sm_get_prepare_timestamp(sm) + 1 + len(request)
            if row["timestamp"] == 0:
                event["timestamp"] = timestamp_commit
            status = row["status"]
            if status == CreateTransferStatus.created:
                if row["pending_id"] != 0:
                    p = transfers[row["pending_id"]]
                    for f in ("debit_account_id", "credit_account_id", "user_data_128"):
                        if u128_of(event, f) == 0:
                            event[f] = p[f]
                    for f in ("ledger", "code", "user_data_64", "user_data_32"):
                        if int(event[f]) == 0:
                            event[f] = p[f]
                    if int(event["flags"]) & (1 << 3) and u128_of(event, "amount") == 0:
                        event["amount"] = p["amount"]
                transfers[row["id"]] = event.copy()
            if status in (CreateTransferStatus.created, CreateTransferStatus.linked_event_failed):
                ts = int(event["timestamp"])
            elif status == CreateTransferStatus.exists:
                ts = int(transfers[row["id"]]["timestamp"]) if row["id"] in transfers \
                    else linked_events_failed[row["id"]]
            else:
                ts = timestamp_commit
            if dense:
                reply.append(struct.pack("<QII", ts, int(status), 0))
            elif status != CreateTransferStatus.created:  # CreateTransferErrorResult (:812-820)
                reply.append(struct.pack("<II", len(request) - 1, int(status)))
            if row["LNK"]:
                if status == CreateTransferStatus.linked_event_failed:
                    assert row["id"] not in linked_events_failed
                    linked_events_failed[row["id"]] = int(event["timestamp"])
            else:
                linked_events_failed.clear()
        elif kind == "lookup_account":
            assert operation in (None, "lookup_accounts")
            operation = "lookup_accounts"
            request.append(struct.pack("<QQ", row["id"] & 0xFFFFFFFFFFFFFFFF, row["id"] >> 64))
            d = row["data"]
            if d is not None:
                a = accounts[row["id"]].copy()
                for f in ("debits_pending", "debits_posted", "credits_pending", "credits_posted"):
                    _set_u128(a, f, d[f])
                flags = int(a["flags"]) & ~(1 << 5)
                if d["closed"]:
                    flags |= 1 << 5
                a["flags"] = flags
                reply.append(a.tobytes())
        elif kind == "lookup_transfer":
            assert operation in (None, "lookup_transfers")
            operation = "lookup_transfers"
            request.append(struct.pack("<QQ", row["id"] & 0xFFFFFFFFFFFFFFFF, row["id"] >> 64))
            variant, value = row["data"]
            if variant == "exists":
                if value:
                    reply.append(transfers[row["id"]].tobytes())
            else:
                t = transfers[row["id"]].copy()
                if variant == "amount":
                    _set_u128(t, "amount", value)
                else:
                    t["timestamp"] = value
                reply.append(t.tobytes())
        elif kind == "get_change_events":
            assert operation is None
            operation = "get_change_events"
            f = np.zeros(1, dtype=CHANGE_EVENTS_FILTER_DTYPE)
            f["timestamp_min"] = 0 if row["min"] is None else int(transfers[row["min"]]["timestamp"])
            f["timestamp_max"] = 0 if row["max"] is None else int(transfers[row["max"]]["timestamp"])
            f["limit"] = row["limit"]
            request.append(f.tobytes())
        elif kind == "get_change_events_result":
            assert operation == "get_change_events"
            reply.append(row)
        elif kind in ("get_account_balances", "get_account_transfers"):
            assert operation is None
            operation = kind
            f = np.zeros(1, dtype=ACCOUNT_FILTER_DTYPE)[0]
            _set_u128(f, "account_id", row["account_id"])
            _set_u128(f, "user_data_128", row["user_data_128"])
            f["user_data_64"] = row["user_data_64"]
            f["user_data_32"] = row["user_data_32"]
            f["code"] = row["code"]
            f["timestamp_min"] = 0 if row["min"] is None else int(transfers[row["min"]]["timestamp"])
            f["timestamp_max"] = 0 if row["max"] is None else int(transfers[row["max"]]["timestamp"])
            f["limit"] = row["limit"]
            f["flags"] = (1 if row["DR"] else 0) | (2 if row["CR"] else 0) | \
                (4 if row["REV"] else 0)
            request.append(f.tobytes())
        elif kind in ("query_accounts", "query_transfers"):
            assert operation is None
            operation = kind
            objects = accounts if kind == "query_accounts" else transfers
            f = np.zeros(1, dtype=QUERY_FILTER_DTYPE)[0]
            _set_u128(f, "user_data_128", row["user_data_128"])
            for k in ("user_data_64", "user_data_32", "ledger", "code"):
                f[k] = row[k]
            f["timestamp_min"] = 0 if row["min"] is None else int(objects[row["min"]]["timestamp"])
            f["timestamp_max"] = 0 if row["max"] is None else int(objects[row["max"]]["timestamp"])
            f["limit"] = row["limit"]
            f["flags"] = 1 if row["REV"] else 0
            request.append(f.tobytes())
        elif kind == "get_account_balances_result":
            assert operation == "get_account_balances"
            b = np.zeros(1, dtype=ACCOUNT_BALANCE_DTYPE)[0]
            for k in ("debits_pending", "debits_posted", "credits_pending", "credits_posted"):
                _set_u128(b, k, row[k])
            b["timestamp"] = transfers[row["transfer_id"]]["timestamp"]
            reply.append(b.tobytes())
        elif kind in ("get_account_transfers_result", "query_transfers_result"):
            assert operation == kind[:-len("_result")]
            reply.append(transfers[row["id"]].tobytes())
        elif kind == "query_accounts_result":
            assert operation == "query_accounts"
            a = accounts[row["id"]].copy()
            d = row["data"]
            if d is not None:
                for k in ("debits_pending", "debits_posted", "credits_pending", "credits_posted"):
                    _set_u128(a, k, d[k])
                a["flags"] = (int(a["flags"]) & ~(1 << 5)) | ((1 << 5) if d["closed"] else 0)
            reply.append(a.tobytes())
        elif kind == "commit":
            op_name = row["operation"]
            if op_name == "get_change_events":
                assert operation == "get_change_events" and len(request) == 1
                commits += 1
                actual = ctx.submit_query(Operation.get_change_events, request[0])
                events = np.frombuffer(actual, dtype=CHANGE_EVENT_DTYPE)
                if len(events) != len(reply):
                    raise TableMismatch(f"{label}: commit #{commits} (get_change_events): "
                                        f"{len(events)} events, expected {len(reply)}")
                for i, (ev, want) in enumerate(zip(events, reply)):
                    why = change_event_mismatch(want, ev, accounts, transfers)
                    if why:
                        raise TableMismatch(f"{label}: commit #{commits} (get_change_events) "
                                            f"event {i}: {why}\n  actual={ev}")
                request.clear()
                reply.clear()
                operation = None
                if handle.after_commit:
                    handle.after_commit()
                    ctx.sm = sm = handle.sm
                continue
            if operation == "skip" or op_name in SKIPPED_OPS:
                request.clear()
                reply.clear()
                operation = None
                continue
            assert operation in (None, op_name), (operation, op_name)
            commits += 1
            payload = b"".join(request)
            if op_name not in ops:
                raise ValueError(op_name)
            if op_name in SCAN_OPS:
                assert len(request) == 1
            code, event_size, result_size, multi_batch = ops[op_name]
            actual = ctx.submit(code, payload, event_size, result_size, multi_batch)
            expected = b"".join(reply)
            if actual != expected:
                raise TableMismatch(describe_mismatch(f"{label} [{version}]", commits, op_name,
                                                      expected, actual, result_size))
            request.clear()
            reply.clear()
            operation = None
            if handle.after_commit:
                handle.after_commit()
                ctx.sm = sm = handle.sm
        else:
            raise ValueError(kind)
    assert operation is None and not request and not reply
    return commits


_CHANGE_TYPES = {None: 0, "PEN": 1, "POS": 2, "VOI": 3, "EXP": 4}


def _match_transfer(ev, t):
    """TestGetChangeEventsResult.match_transfer (state_machine_tests.zig:582-598)."""
    if int(ev["transfer_timestamp"]) != int(t["timestamp"]):
        return "transfer_timestamp"
    if u128_of(ev, "transfer_id") != u128_of(t, "id"):
        return "transfer_id"
    if u128_of(ev, "transfer_amount") != u128_of(t, "amount") and u128_of(t, "amount") != U128_MAX:
        return "transfer_amount"
    if u128_of(ev, "transfer_pending_id") != u128_of(t, "pending_id"):
        return "transfer_pending_id"
    if u128_of(ev, "transfer_user_data_128") != u128_of(t, "user_data_128"):
        return "transfer_user_data_128"
    for a, b in (("transfer_user_data_64", "user_data_64"), ("transfer_user_data_32", "user_data_32"),
                 ("transfer_code", "code"), ("ledger", "ledger"), ("transfer_flags", "flags")):
        if int(ev[a]) != int(t[b]):
            return a
    return None


def change_event_mismatch(want, ev, accounts, transfers):
    """TestGetChangeEventsResult.match (state_machine_tests.zig:519-580); None when it matches."""
    if want["timestamp_transfer"] is not None:
        t = transfers[want["timestamp_transfer"]]
        if int(ev["type"]) == 4:
            return "expired event for a transfer timestamp"
        if int(ev["timestamp"]) != int(t["timestamp"]):
            return "timestamp"
        why = _match_transfer(ev, t)
        if why:
            return why
    if int(ev["type"]) != _CHANGE_TYPES[want["event_type"]]:
        return "type"
    if u128_of(ev, "transfer_amount") != want["amount"]:
        return "amount"
    if want["pending_id"] is not None:
        typ = int(ev["type"])
        if typ in (0, 1):
            return "pending id on a single-phase / pending event"
        if typ in (2, 3):
            if u128_of(ev, "transfer_pending_id") != want["pending_id"]:
                return "transfer_pending_id"
        else:
            t = transfers[want["pending_id"]]
            if int(t["timeout"]) == 0:
                return "expired transfer without timeout"
            if int(ev["timestamp"]) < int(t["timestamp"]) + int(t["timeout"]) * NS_PER_S:
                return "expired before its expiry"
            why = _match_transfer(ev, t)
            if why:
                return why
    for side, prefix in (("dr", "debit_account_"), ("cr", "credit_account_")):
        b = want[side]
        a = accounts[b["account_id"]]
        if int(a["ledger"]) != int(ev["ledger"]):
            return f"{side} ledger"
        if u128_of(ev, prefix + "id") != b["account_id"]:
            return f"{side} account id"
        if int(a["timestamp"]) != int(ev[prefix + "timestamp"]):
            return f"{side} account timestamp"
        for f in ("debits_pending", "debits_posted", "credits_pending", "credits_posted"):
            if u128_of(ev, prefix + f) != b[f]:
                return f"{side} {f}"
        if bool(int(ev[prefix + "flags"]) & (1 << 5)) != b["closed"]:
            return f"{side} closed"
    return None


def describe_mismatch(label, commit_index, op_name, expected: bytes, actual: bytes,
                      result_size=16) -> str:
    lines = [f"{label}: commit #{commit_index} ({op_name}) reply mismatch "
             f"(expected {len(expected)} B, actual {len(actual)} B)"]
    if op_name.startswith("create") and result_size == 8:
        e = np.frombuffer(expected, dtype=np.uint32).reshape(-1, 2)
        a = np.frombuffer(actual, dtype=np.uint32).reshape(-1, 2)
        lines.append(f"expected {e.tolist()}\nactual   {a.tolist()}")
    elif op_name.startswith("create"):
        e = np.frombuffer(expected, dtype=RESULT_DTYPE)
        a = np.frombuffer(actual, dtype=RESULT_DTYPE)
        enum_t = CreateAccountStatus if op_name == "create_accounts" else CreateTransferStatus
        for i in range(max(len(e), len(a))):
            es = (int(e[i]["timestamp"]), enum_t(int(e[i]["status"])).name) if i < len(e) else None
            as_ = (int(a[i]["timestamp"]), enum_t(int(a[i]["status"])).name) if i < len(a) else None
            mark = "   " if es == as_ else ">>>"
            lines.append(f"{mark} [{i}] expected={es} actual={as_}")
    else:
        dt = {"lookup_accounts": ACCOUNT_DTYPE, "query_accounts": ACCOUNT_DTYPE,
              "get_account_balances": ACCOUNT_BALANCE_DTYPE}.get(op_name, TRANSFER_DTYPE)
        e = np.frombuffer(expected, dtype=dt)
        a = np.frombuffer(actual, dtype=dt)
        for i in range(max(len(e), len(a))):
            ei = e[i] if i < len(e) else None
            ai = a[i] if i < len(a) else None
            mark = "   " if (ei is not None and ai is not None and ei.tobytes() == ai.tobytes()) \
                else ">>>"
            lines.append(f"{mark} [{i}] expected={ei}\n        actual={ai}")
    return "\n".join(lines)


def sm_options():
    o = native.SmOptions()
    o.batch_size_limit = TEST_BATCH_SIZE_LIMIT
    o.message_body_size_max = TEST_MESSAGE_BODY_SIZE_MAX
    o.pulse_batch_max = TEST_PULSE_BATCH_MAX
    return o
