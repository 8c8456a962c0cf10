"""The StateMachine contract's sizing and validation, restated from the reference's own tests.

- "StateMachine: batch_elements_max" (src/state_machine_tests.zig:2911-2948)
- "StateMachine: input_valid" (:2950-3048): every operation but pulse, with 0, 1, event_max and
  event_max + 1 events, multi-batch encoded or not as the operation is
- "StateMachine: query multi-batch input_valid" (:3050-3219): multi-batch query filters are valid
  while the sum of their limits fits one reply
- "sum_overflows" (src/state_machine.zig:5144-5166): the executor's overflow predicate, on the
  host and once on the device

All under the reference's unit-test configuration (message_body_size_max 3840, batch_size_limit
30 x 128), through tb_sm (tb_state_machine.h) bound to the CPU oracle executor, and once bound to
the HIP executor (tb_sm_open_gpu).
"""
import ctypes

import numpy as np
import pytest

import tablerun
from test_oracle_tables import oracle_handle
from tigerbeetle_amd import native
from tigerbeetle_amd.types import ACCOUNT_FILTER_DTYPE, QUERY_FILTER_DTYPE

MBSM = tablerun.TEST_MESSAGE_BODY_SIZE_MAX
BSL = tablerun.TEST_BATCH_SIZE_LIMIT
U32_MAX = 0xFFFFFFFF

# Operation (src/tigerbeetle.zig:685-849): number -> (event size, result size, batchable,
# multi-batch). Pulse is skipped by the reference's test.
OPERATIONS = {
    "deprecated_create_accounts_unbatched": (129, 128, 8, True, False),
    "deprecated_create_transfers_unbatched": (130, 128, 8, True, False),
    "deprecated_lookup_accounts_unbatched": (131, 16, 128, True, False),
    "deprecated_lookup_transfers_unbatched": (132, 16, 128, True, False),
    "deprecated_get_account_transfers_unbatched": (133, 128, 128, False, False),
    "deprecated_get_account_balances_unbatched": (134, 128, 128, False, False),
    "deprecated_query_accounts_unbatched": (135, 64, 128, False, False),
    "deprecated_query_transfers_unbatched": (136, 64, 128, False, False),
    "get_change_events": (137, 64, 384, False, False),
    "deprecated_create_accounts_sparse": (138, 128, 8, True, True),
    "deprecated_create_transfers_sparse": (139, 128, 8, True, True),
    "lookup_accounts": (140, 16, 128, True, True),
    "lookup_transfers": (141, 16, 128, True, True),
    "get_account_transfers": (142, 128, 128, False, True),
    "get_account_balances": (143, 128, 128, False, True),
    "query_accounts": (144, 64, 128, False, True),
    "query_transfers": (145, 64, 128, False, True),
    "create_accounts": (146, 128, 16, True, True),
    "create_transfers": (147, 128, 16, True, True),
}
OP = {name: v[0] for name, v in OPERATIONS.items()}


def encode(lib, batches, element_size):
    """MultiBatchEncoder: `batches` (byte strings, one per batch) and the trailer."""
    payload = b"".join(batches)
    counts = (ctypes.c_uint16 * len(batches))(*[len(b) // element_size for b in batches])
    buf = ctypes.create_string_buffer(len(payload) + 2 * MBSM)
    ctypes.memmove(buf, payload, len(payload))
    size = lib.tb_multi_batch_encode_trailer(buf, len(payload), element_size, counts,
                                             len(batches))
    assert size > 0
    return buf.raw[:size]


def build_input(lib, name, event_count):
    """build_input (:2961-2981): event_count zeroed events, one batch if multi-batch."""
    _, event_size, _, _, multi_batch = OPERATIONS[name]
    payload = bytes(event_count * event_size)
    return encode(lib, [payload], event_size) if multi_batch else payload


def valid(lib, sm, name, body):
    return lib.tb_sm_input_valid(sm, OP[name], body, len(body)) == 1


def check_batch_elements_max(lib, sm):
    events_max = MBSM // 128
    for name in ("deprecated_create_accounts_unbatched", "deprecated_lookup_accounts_unbatched",
                 "deprecated_create_transfers_unbatched", "deprecated_lookup_transfers_unbatched"):
        assert lib.tb_sm_event_max(sm, OP[name], MBSM) == events_max, name
    # multi-batch encoded: one element's room is taken by the trailer
    for name in ("create_accounts", "create_transfers", "lookup_accounts", "lookup_transfers"):
        assert lib.tb_sm_event_max(sm, OP[name], MBSM) == events_max - 1, name


def check_input_valid(lib, sm):
    checked = 0
    for name, (op, event_size, _, batchable, _) in OPERATIONS.items():
        event_min, event_max = (1, 1) if not batchable else (0, lib.tb_sm_event_max(sm, op, BSL))
        assert event_min <= event_max
        assert valid(lib, sm, name, build_input(lib, name, 0)) == (event_min == 0), name
        assert valid(lib, sm, name, build_input(lib, name, 1)), name
        assert valid(lib, sm, name, build_input(lib, name, event_max)), name
        too_much_data = build_input(lib, name, event_max + 1)
        if len(too_much_data) < MBSM:
            assert not valid(lib, sm, name, too_much_data), name
        checked += 1
    assert checked == 19


def filters(name, limits):
    """One zeroed AccountFilter / QueryFilter per batch with the given limit (:3066-3136)."""
    _, event_size, _, _, _ = OPERATIONS[name]
    dt = ACCOUNT_FILTER_DTYPE if event_size == 128 else QUERY_FILTER_DTYPE
    off = dt.fields["limit"][1]
    out = []
    for limit in limits:
        f = bytearray(event_size)
        f[off:off + 4] = int(limit).to_bytes(4, "little")
        out.append(bytes(f))
    return out


def check_query_multi_batch(lib, sm):
    for name in ("get_account_transfers", "get_account_balances", "query_accounts",
                 "query_transfers"):
        op, event_size = OP[name], OPERATIONS[name][1]
        batch_max = lib.tb_sm_result_max(sm, op, BSL)

        def body(limits):
            if not limits:
                return encode(lib, [b""], event_size)  # body_encoder.add(0)
            return encode(lib, filters(name, limits), event_size)

        for limits in ([0], [0, 0], [1], [1, 1, 1], [batch_max], [0, batch_max],
                       [0, 1, batch_max - 1], [1, 1, batch_max - 2],
                       [batch_max // 2, -(-batch_max // 2)], [U32_MAX]):
            assert valid(lib, sm, name, body(limits)), (name, limits)
        for limits in ([], [1, batch_max], [1, U32_MAX], [batch_max, batch_max],
                       [batch_max // 2, -(-batch_max // 2), 1]):
            assert not valid(lib, sm, name, body(limits)), (name, limits)


SUM_OVERFLOWS_CASES = [  # sum_overflows_test (:5151-5161): (a, b, overflows) per Int width
    ("max", "0", False), ("max-1", "1", False), ("1", "max-1", False),
    ("max", "1", True), ("1", "max", True), ("max", "max", True),
]


def sum_overflows_vectors(bits):
    m = (1 << bits) - 1
    val = {"max": m, "max-1": m - 1, "0": 0, "1": 1}
    a = np.zeros((len(SUM_OVERFLOWS_CASES), 2), dtype=np.uint64)
    b = np.zeros_like(a)
    want = []
    for i, (x, y, o) in enumerate(SUM_OVERFLOWS_CASES):
        for arr, v in ((a, val[x]), (b, val[y])):
            arr[i, 0] = v & 0xFFFFFFFFFFFFFFFF
            arr[i, 1] = v >> 64
        want.append(o)
    return a, b, np.asarray(want, dtype=np.uint8)


def check_sum_overflows(lib, g):
    for bits in (64, 128):
        a, b, want = sum_overflows_vectors(bits)
        out = np.full(len(want), 7, dtype=np.uint8)
        rc = lib.tbg_sum_overflows(g, bits, a.ctypes.data_as(ctypes.c_void_p),
                                   b.ctypes.data_as(ctypes.c_void_p), len(want),
                                   out.ctypes.data_as(ctypes.c_void_p))
        assert rc == 0 and (out == want).all(), (bits, out, want)


@pytest.fixture
def oracle_sm():
    h = oracle_handle()
    yield h.lib, h.sm
    h.close()


def test_batch_elements_max(oracle_sm):
    check_batch_elements_max(*oracle_sm)


def test_input_valid(oracle_sm):
    check_input_valid(*oracle_sm)


def test_query_multi_batch_input_valid(oracle_sm):
    check_query_multi_batch(*oracle_sm)


def test_input_valid_rejects_malformed_bodies(oracle_sm):
    """Beyond the reference's cases: bodies the decoder refuses (MultiBatchDecoder.init,
    multi_batch.zig:135-230) and sizes past batch_size_limit are invalid, not errors."""
    lib, sm = oracle_sm
    good = build_input(lib, "create_transfers", 3)
    assert valid(lib, sm, "create_transfers", good)
    assert not valid(lib, sm, "create_transfers", good[:-2])          # truncated postamble
    assert not valid(lib, sm, "create_transfers", good[:128] + good[256:])  # payload != counts
    assert not valid(lib, sm, "create_transfers", bytes(BSL + 128))   # > batch_size_limit
    assert not valid(lib, sm, "create_transfers", b"")                # no postamble at all
    assert lib.tb_sm_input_valid(sm, 128, b"x", 1) == 0               # pulse takes no body
    assert lib.tb_sm_input_valid(sm, 128, b"", 0) == 1                # pulse: empty body
    assert lib.tb_sm_input_valid(sm, 127, b"", 0) == 0                # not an operation
    assert not valid(lib, sm, "deprecated_create_transfers_unbatched", bytes(129))


def test_sum_overflows_host():
    check_sum_overflows(native.load(), None)


@pytest.mark.gpu
def test_contract_through_the_gpu_state_machine():
    """The same sizing and validation with the HIP executor bound (tb_sm_open_gpu), and the
    device's overflow predicate evaluated by a kernel."""
    lib = native.load()
    o = native.TbgOptions()
    o.account_capacity = 64
    o.transfer_capacity = 64
    o.batch_events_max = 64
    o.batch_count_max = 64
    o.pulse_batch_max = tablerun.TEST_PULSE_BATCH_MAX
    o.device = 0
    o.pulse_next_timestamp_init = 1 << 63
    sm = lib.tb_sm_open_gpu(ctypes.byref(tablerun.sm_options()), ctypes.byref(o))
    assert sm
    try:
        check_batch_elements_max(lib, sm)
        check_input_valid(lib, sm)
        check_query_multi_batch(lib, sm)
        check_sum_overflows(lib, lib.tb_sm_executor_gpu(sm))
    finally:
        lib.tb_sm_close(sm)
