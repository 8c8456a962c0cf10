"""ctypes binding of the CPU oracle (oracle/liboracle.so). TEST INFRASTRUCTURE ONLY."""
import ctypes
import os

from tigerbeetle_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

vp = ctypes.c_void_p
U128 = native.U128

_SIGS = [
    ("tbo_open", vp, [ctypes.c_uint32, ctypes.c_uint64]),
    ("tbo_close", None, [vp]),
    ("tbo_create_accounts", None, [vp, vp, ctypes.c_uint32, ctypes.c_uint64, vp]),
    ("tbo_create_transfers", None, [vp, vp, ctypes.c_uint32, ctypes.c_uint64, vp]),
    ("tbo_create_accounts_batches", None, [vp, vp, vp, vp, ctypes.c_uint32, vp]),
    ("tbo_create_transfers_batches", None, [vp, vp, vp, vp, ctypes.c_uint32, vp]),
    ("tbo_create_accounts_stamped", None, [vp, vp, ctypes.c_uint32, vp, ctypes.c_uint64,
                                           ctypes.c_uint32, vp]),
    ("tbo_create_transfers_stamped", None, [vp, vp, ctypes.c_uint32, vp, ctypes.c_uint64,
                                            ctypes.c_uint32, vp]),
    ("tbo_forget_orphans", ctypes.c_uint64, [vp, vp, ctypes.c_uint32]),
    ("tbo_key_max", None, [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]),
    ("tbo_timestamps_exist", ctypes.c_uint64, [vp, ctypes.c_int, vp, ctypes.c_uint32, vp]),
    ("tbo_pulse", ctypes.c_uint32, [vp, ctypes.c_uint64]),
    ("tbo_pulse_candidates", ctypes.c_uint64, [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint32]),
    ("tbo_pulse_cut", ctypes.c_uint32, [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                        ctypes.c_uint64, vp]),
    ("tbo_pulse_needed", ctypes.c_int, [vp, ctypes.c_uint64]),
    ("tbo_pulse_next_timestamp", ctypes.c_uint64, [vp]),
    ("tbo_lookup_accounts", ctypes.c_uint32, [vp, vp, ctypes.c_uint32, vp]),
    ("tbo_lookup_transfers", ctypes.c_uint32, [vp, vp, ctypes.c_uint32, vp]),
    ("tbo_set_account_balances", ctypes.c_int, [vp, U128, U128, U128, U128, U128]),
    ("tbo_account_count", ctypes.c_uint64, [vp]),
    ("tbo_transfer_count", ctypes.c_uint64, [vp]),
    ("tbo_dump_accounts", ctypes.c_uint64, [vp, vp]),
    ("tbo_dump_transfers", ctypes.c_uint64, [vp, vp]),
    ("tbo_dump_pending_status", ctypes.c_uint64, [vp, vp]),
    ("tbo_dump_account_events", ctypes.c_uint64, [vp, vp]),
    ("tbo_raise_key_max", None, [vp, ctypes.c_uint64, ctypes.c_uint64]),
    ("tbo_pnt_sharded", None, [vp, ctypes.c_int]),
    ("tbo_pnt_ops", ctypes.c_uint64, [vp, vp, vp, ctypes.POINTER(ctypes.c_uint64)]),
    ("tbo_set_pulse_next_timestamp", None, [vp, ctypes.c_uint64]),
    ("tbo_get_change_events", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbo_get_account_transfers", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbo_get_account_balances", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbo_query_accounts", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbo_query_transfers", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbo_executor_fill", None, [vp, ctypes.POINTER(native.Executor)]),
    ("tbo_shard_ops_fill", None, [vp]),
]

_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_PATH):
            raise OSError(f"oracle not built: {ORACLE_PATH} (make -C oracle)")
        lib = ctypes.CDLL(ORACLE_PATH)
        for name, res, args in _SIGS:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib
