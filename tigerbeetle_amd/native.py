"""ctypes bindings of the product library libtbg.so (include/tbg.h, include/tb_state_machine.h).

The library is built in-tree by ``__graft_entry__.build()`` (or ``make -C tigerbeetle_amd/csrc``)
into ``tigerbeetle_amd/lib/libtbg.so``. There is no fallback: if the library is missing, importing
the product path raises.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libtbg.so")

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_u16p = ctypes.POINTER(ctypes.c_uint16)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
vp = ctypes.c_void_p


class U128(ctypes.Structure):
    _fields_ = [("lo", ctypes.c_uint64), ("hi", ctypes.c_uint64)]

    @classmethod
    def of(cls, x: int):
        return cls(x & 0xFFFFFFFFFFFFFFFF, (x >> 64) & 0xFFFFFFFFFFFFFFFF)


class TbgOptions(ctypes.Structure):
    _fields_ = [
        ("account_capacity", ctypes.c_uint64),
        ("transfer_capacity", ctypes.c_uint64),
        ("batch_events_max", ctypes.c_uint32),
        ("batch_count_max", ctypes.c_uint32),
        ("pulse_batch_max", ctypes.c_uint32),
        ("device", ctypes.c_uint32),
        ("pulse_next_timestamp_init", ctypes.c_uint64),
        ("account_events_capacity", ctypes.c_uint64),
    ]


def options(account_capacity, transfer_capacity, batch_events_max=1 << 16, batch_count_max=4096,
            pulse_batch_max=8190, device=0, pulse_next_timestamp_init=(1 << 63) - 1,
            account_events_capacity=0) -> TbgOptions:
    o = TbgOptions()
    o.account_capacity = account_capacity
    o.transfer_capacity = transfer_capacity
    o.batch_events_max = batch_events_max
    o.batch_count_max = batch_count_max
    o.pulse_batch_max = pulse_batch_max
    o.device = device
    o.pulse_next_timestamp_init = pulse_next_timestamp_init
    o.account_events_capacity = account_events_capacity
    return o


class TbgStats(ctypes.Structure):
    _fields_ = [
        ("events", ctypes.c_uint64),
        ("fast", ctypes.c_uint64),
        ("replayed", ctypes.c_uint64),
        ("static_fail", ctypes.c_uint64),
        ("ae_window", ctypes.c_uint64),
        ("ingest_finished", ctypes.c_uint64),
    ]


class SmOptions(ctypes.Structure):
    _fields_ = [
        ("batch_size_limit", ctypes.c_uint32),
        ("message_body_size_max", ctypes.c_uint32),
        ("pulse_batch_max", ctypes.c_uint32),
    ]


# tb_executor (tb_state_machine.h): a vtable of C function pointers.
class Executor(ctypes.Structure):
    _fields_ = [
        ("self", vp),
        ("create_accounts", vp),
        ("create_transfers", vp),
        ("pulse", vp),
        ("pulse_next_timestamp", vp),
        ("lookup_accounts", vp),
        ("lookup_transfers", vp),
        ("get_change_events", vp),
        ("get_account_transfers", vp),
        ("get_account_balances", vp),
        ("query_accounts", vp),
        ("query_transfers", vp),
    ]


PREFETCH_CALLBACK = ctypes.CFUNCTYPE(None, vp)

# Exported symbols: (name, restype, argtypes). tests/test_abi.py checks each one against the
# declarations in include/*.h.
SIGNATURES = [
    ("tbg_open", vp, [ctypes.POINTER(TbgOptions)]),
    ("tbg_close", None, [vp]),
    ("tbg_last_error", ctypes.c_char_p, [vp]),
    ("tbg_create_accounts", ctypes.c_int, [vp, vp, ctypes.c_uint32, c_u32p, c_u64p,
                                          ctypes.c_uint32, vp]),
    ("tbg_create_transfers", ctypes.c_int, [vp, vp, ctypes.c_uint32, c_u32p, c_u64p,
                                           ctypes.c_uint32, vp]),
    ("tbg_create_accounts_device", ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, vp,
                                                 ctypes.c_uint32, vp, vp]),
    ("tbg_create_transfers_device", ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, vp,
                                                  ctypes.c_uint32, vp, vp]),
    ("tbg_create_transfers_stamped_device", ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, vp, vp]),
    ("tbg_create_transfers_stamped", ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, ctypes.c_uint64,
                                                   ctypes.c_uint32, vp]),
    ("tbg_create_accounts_stamped", ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, ctypes.c_uint64,
                                                  ctypes.c_uint32, vp]),
    ("tbg_forget_orphans", ctypes.c_int64, [vp, vp, ctypes.c_uint32]),
    ("tbg_timestamps_exist", ctypes.c_int64, [vp, ctypes.c_int, vp, ctypes.c_uint32, vp]),
    ("tbg_register_host", ctypes.c_int, [vp, vp, ctypes.c_uint64]),
    ("tbg_unregister_host", ctypes.c_int, [vp, vp]),
    ("tbg_synchronize", ctypes.c_int, [vp]),
    ("tbg_pulse", ctypes.c_int64, [vp, ctypes.c_uint64]),
    ("tbg_pulse_candidates", ctypes.c_int64, [vp, ctypes.c_uint64, vp, vp, ctypes.c_uint32]),
    ("tbg_pulse_cut", ctypes.c_int64, [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                       ctypes.c_uint64, vp]),
    ("tbg_pulse_next_timestamp", ctypes.c_uint64, [vp]),
    ("tbg_raise_key_max", ctypes.c_int, [vp, ctypes.c_uint64, ctypes.c_uint64]),
    ("tbg_key_max", ctypes.c_int, [vp, c_u64p, c_u64p]),
    ("tbg_set_pnt_sharded", ctypes.c_int, [vp, ctypes.c_int]),
    ("tbg_pnt_ops", ctypes.c_int64, [vp, vp, vp, ctypes.c_uint64, c_u64p]),
    ("tbg_set_pulse_next_timestamp", ctypes.c_int, [vp, ctypes.c_uint64]),
    ("tbg_lookup_accounts", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbg_lookup_transfers", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbg_dump_accounts", ctypes.c_int64, [vp, vp]),
    ("tbg_dump_transfers", ctypes.c_int64, [vp, vp, vp]),
    ("tbg_dump_transfer_ids", ctypes.c_int64, [vp, vp]),
    ("tbg_dump_account_events", ctypes.c_int64, [vp, vp]),
    ("tbg_get_change_events", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbg_compact", ctypes.c_int64, [vp]),
    ("tbg_checkpoint", ctypes.c_int, [vp, ctypes.c_char_p]),
    ("tbg_open_checkpoint", vp, [ctypes.POINTER(TbgOptions), ctypes.c_char_p]),
    ("tbg_get_account_transfers", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbg_get_account_balances", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbg_query_accounts", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbg_query_transfers", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbg_debug_set_account_balances", ctypes.c_int, [vp, U128, U128, U128, U128, U128]),
    ("tbg_last_stats", ctypes.c_int, [vp, ctypes.POINTER(TbgStats)]),
    ("tbg_sum_overflows", ctypes.c_int, [vp, ctypes.c_uint32, vp, vp, ctypes.c_uint32, vp]),
    ("tbg_debug_force_replay", ctypes.c_int, [vp, ctypes.c_int]),
    ("tbg_debug_serial_replay", ctypes.c_int, [vp, ctypes.c_int]),
    ("tbg_debug_ae_sync", ctypes.c_int, [vp, ctypes.c_int]),
    ("tbg_profile", ctypes.c_int, [vp, ctypes.c_int]),
    ("tbg_profile_read", ctypes.c_int, [vp, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
                                       ctypes.POINTER(ctypes.c_double), c_u64p]),
    ("tbr_open", vp, [ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                      ctypes.c_uint32]),
    ("tbr_close", None, [vp]),
    ("tbr_record_accounts", ctypes.c_int, [vp, vp, vp, ctypes.c_uint32]),
    ("tbr_record_transfers", ctypes.c_int, [vp, vp, vp, ctypes.c_uint32]),
    ("tbr_account_shards", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbr_transfer_shards", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbr_route_device", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp, vp, ctypes.c_uint32, vp, vp,
                                          vp, vp]),
    ("tbr_settle_device", ctypes.c_int, [vp, vp, vp, ctypes.c_uint32, vp, c_u64p]),
    ("tbr_set_imported_floor", ctypes.c_int, [vp, ctypes.c_uint64]),
    ("tbr_route_stats", ctypes.c_int, [vp, c_u64p]),
    ("tbr_route_device_slices", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp, vp, ctypes.c_uint32,
                                                 vp, vp, vp]),
    ("tbg_group_open", vp, [vp, vp]),
    ("tbg_group_open_shards", vp, [vp, vp, vp]),
    ("tbg_group_close", None, [vp]),
    ("tbg_group_hip_shard_ops", None, [vp]),
    ("tbg_group_checkpoint", ctypes.c_int, [vp, vp]),
    ("tbg_group_open_checkpoint", vp, [vp, vp, vp]),
    ("tbg_group_last_error", ctypes.c_char_p, [vp]),
    ("tbg_group_shard", vp, [vp, ctypes.c_uint32]),
    ("tbg_group_create_accounts", ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, vp,
                                                ctypes.c_uint32, vp]),
    ("tbg_group_create_transfers", ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, vp,
                                                 ctypes.c_uint32, vp]),
    ("tbg_group_create_transfers_device", ctypes.c_int, [vp, vp, ctypes.c_uint32, vp, vp,
                                                        ctypes.c_uint32, vp]),
    ("tbg_group_pulse", ctypes.c_int64, [vp, ctypes.c_uint64]),
    ("tbg_group_pulse_next_timestamp", ctypes.c_uint64, [vp]),
    ("tbg_group_lookup_accounts", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbg_group_lookup_transfers", ctypes.c_int64, [vp, vp, ctypes.c_uint32, vp]),
    ("tbg_group_executor", None, [vp, ctypes.POINTER(Executor)]),
    ("tbg_group_stats_read", ctypes.c_int, [vp, vp]),
    ("tbg_group_plan", ctypes.c_int64, [vp, ctypes.c_int, vp, ctypes.c_uint32, vp, vp,
                                        ctypes.c_uint32, vp, vp, vp, ctypes.c_uint32]),
    ("tbg_group_record_accounts", ctypes.c_int, [vp, vp, vp, ctypes.c_uint32]),
    ("tbg_group_record_transfers", ctypes.c_int, [vp, vp, vp, ctypes.c_uint32]),
    ("tb_sm_open", vp, [ctypes.POINTER(SmOptions), ctypes.POINTER(Executor)]),
    ("tb_sm_open_gpu", vp, [ctypes.POINTER(SmOptions), ctypes.POINTER(TbgOptions)]),
    ("tb_sm_open_gpu_checkpoint", vp, [ctypes.POINTER(SmOptions), ctypes.POINTER(TbgOptions),
                                       ctypes.c_char_p]),
    ("tb_sm_close", None, [vp]),
    ("tb_sm_compact", ctypes.c_int, [vp, ctypes.c_uint64]),
    ("tb_sm_checkpoint", ctypes.c_int, [vp, ctypes.c_char_p]),
    ("tb_sm_executor_gpu", vp, [vp]),
    ("tb_sm_register_buffer", ctypes.c_int, [vp, vp, ctypes.c_uint64]),
    ("tb_sm_input_valid", ctypes.c_int, [vp, ctypes.c_uint8, vp, ctypes.c_uint32]),
    ("tb_sm_event_max", ctypes.c_uint32, [vp, ctypes.c_uint8, ctypes.c_uint32]),
    ("tb_sm_result_max", ctypes.c_uint32, [vp, ctypes.c_uint8, ctypes.c_uint32]),
    ("tb_sm_prepare", None, [vp, ctypes.c_uint8, vp, ctypes.c_uint32]),
    ("tb_sm_pulse_needed", ctypes.c_int, [vp, ctypes.c_uint64]),
    ("tb_sm_prefetch", None, [vp, PREFETCH_CALLBACK, vp, ctypes.c_uint64, ctypes.c_uint64,
                              ctypes.c_uint8, vp, ctypes.c_uint32]),
    ("tb_sm_commit", ctypes.c_int64, [vp, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_uint64, ctypes.c_uint8, vp, ctypes.c_uint32, vp]),
    ("tb_sm_get_prepare_timestamp", ctypes.c_uint64, [vp]),
    ("tb_sm_get_commit_timestamp", ctypes.c_uint64, [vp]),
    ("tb_sm_get_prefetch_timestamp", ctypes.c_uint64, [vp]),
    ("tb_sm_set_prepare_timestamp", None, [vp, ctypes.c_uint64]),
    ("tb_sm_set_commit_timestamp", None, [vp, ctypes.c_uint64]),
    ("tb_sm_set_prefetch_timestamp", None, [vp, ctypes.c_uint64]),
    ("tb_multi_batch_encode_trailer", ctypes.c_int64, [vp, ctypes.c_uint32, ctypes.c_uint32,
                                                      c_u16p, ctypes.c_uint32]),
    ("tb_multi_batch_decode", ctypes.c_int64, [vp, ctypes.c_uint32, ctypes.c_uint32, c_u16p,
                                              ctypes.c_uint32, c_u32p]),
    ("tb_multi_batch_trailer_total_size", ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32]),
]

_lib = None


def load(path: str = None):
    """Load libtbg.so (once). Raises OSError if it is missing: there is no fallback path."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    # (TBG_LIB: an alternative build of the same library, for same-box A/B measurements)
    p = path or os.environ.get("TBG_LIB") or LIB_PATH
    if not os.path.exists(p):
        raise OSError(f"libtbg.so not built: {p} (run __graft_entry__.build())")
    lib = ctypes.CDLL(p)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path is None:
        _lib = lib
    return lib
