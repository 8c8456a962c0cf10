"""Ledger sharding of the commit path across GPUs: a thin ctypes wrapper of the
executor group, include/tbg_group.h.

The group -- the device router, the per-shard transport and the exact engine (placement,
segments, the chain protocol for linked chains across shards, imported events across shards,
pulse_next_timestamp and pulses across shards) -- is C++ in libtbg.so
(tigerbeetle_amd/csrc/shards.cpp, engine.cpp); one process owns every shard, as the reference's
one replica process owns its one StateMachine (src/vsr/replica.zig:144-152). This module only
marshals numpy arrays:

* `Group.open_gpu(...)` -- N HIP executors (devices may repeat: several shards on one GPU), the
  device router on the router's GPU;
* `Group.open_shards(ops, selves)` -- a group over executors the caller binds through the shard
  executor interface (`tbg_shard_ops`): the tests bind the CPU oracle;
* `GpuShard` -- one HIP executor (tbg.h) with the same numpy interface, for tests and the bench.
"""
import ctypes
import os

import numpy as np

from . import native
from .types import ACCOUNT_DTYPE, RESULT_DTYPE, TRANSFER_DTYPE

vp = ctypes.c_void_p


def _u128_array(ids) -> np.ndarray:
    ids = list(ids)
    a = np.zeros((len(ids), 2), dtype=np.uint64)
    if ids:
        a[:, 0] = [int(i) & 0xFFFFFFFFFFFFFFFF for i in ids]
        a[:, 1] = [int(i) >> 64 for i in ids]
    return a


def _ptr(a):
    return a.ctypes.data_as(vp)


class GroupOptions(ctypes.Structure):
    _fields_ = [
        ("shards", ctypes.c_uint32),
        ("ledgers", ctypes.c_uint32),
        ("events_max", ctypes.c_uint32),
        ("batch_count_max", ctypes.c_uint32),
        ("pulse_batch_max", ctypes.c_uint32),
        ("router_device", ctypes.c_uint32),
        ("router_account_capacity", ctypes.c_uint64),
        ("router_transfer_capacity", ctypes.c_uint64),
    ]


class GroupStats(ctypes.Structure):
    _fields_ = [(name, ctypes.c_uint64) for name in (
        "calls", "device_calls", "engine_calls", "segments", "chain_segments", "surrogates",
        "anywhere", "repeats", "route_ns", "execute_ns", "settle_ns", "engine_ns")]


class ShardOps(ctypes.Structure):
    """tbg_shard_ops: one C function pointer per shard operation."""
    _fields_ = [(name, vp) for name in (
        "create_accounts", "create_transfers", "create_accounts_stamped",
        "create_transfers_stamped", "forget_orphans", "timestamps_exist", "key_max",
        "raise_key_max", "set_pnt_sharded", "pnt_ops", "pulse_next_timestamp",
        "set_pulse_next_timestamp", "pulse_candidates", "pulse_cut", "lookup_accounts",
        "lookup_transfers")]


def group_options(shards, ledgers=64, events_max=1 << 16, batch_count_max=4096,
                  pulse_batch_max=8190, router_device=0, router_account_capacity=1 << 16,
                  router_transfer_capacity=1 << 20):
    o = GroupOptions()
    o.shards = shards
    o.ledgers = ledgers
    o.events_max = events_max
    o.batch_count_max = batch_count_max
    o.pulse_batch_max = pulse_batch_max
    o.router_device = router_device
    o.router_account_capacity = router_account_capacity
    o.router_transfer_capacity = router_transfer_capacity
    return o


class Group:
    """A tbg_group (include/tbg_group.h) with numpy calls: the client interface of the sharded
    commit path (create_accounts / create_transfers over a multi-batch call, pulses, lookups)."""

    def __init__(self, lib, g, options, owner=None):
        if not g:
            raise RuntimeError("tbg_group_open failed")
        self.lib = lib
        self.g = g
        self.options = options
        self.shards = options.shards
        self._owner = owner  # (keeps the caller's ops table alive)

    @classmethod
    def open_gpu(cls, shard_options, **kw):
        """N HIP executors: `shard_options` is a list of native.TbgOptions (one per shard, its
        `device` and capacities); keywords as group_options."""
        lib = native.load()
        o = group_options(len(shard_options), **kw)
        arr = (native.TbgOptions * len(shard_options))(*shard_options)
        return cls(lib, lib.tbg_group_open(ctypes.byref(o), arr), o)

    @classmethod
    def open_gpu_checkpoint(cls, shard_options, paths, **kw):
        """open_gpu from the shards' checkpoint images (tbg_group_open_checkpoint: the router's
        directories rebuilt from the shards' tables)."""
        lib = native.load()
        o = group_options(len(shard_options), **kw)
        arr = (native.TbgOptions * len(shard_options))(*shard_options)
        cp = (ctypes.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
        return cls(lib, lib.tbg_group_open_checkpoint(ctypes.byref(o), arr, cp), o)

    def checkpoint(self, paths):
        """Every shard's image to paths[s] (tbg_group_checkpoint)."""
        cp = (ctypes.c_char_p * len(paths))(*[os.fsencode(p) for p in paths])
        return self._check(self.lib.tbg_group_checkpoint(self.g, cp), "checkpoint")

    @classmethod
    def open_shards(cls, ops: ShardOps, selves, **kw):
        """A group over the caller's executors `selves` (pointers) bound through `ops`."""
        lib = native.load()
        o = group_options(len(selves), **kw)
        arr = (vp * len(selves))(*selves)
        return cls(lib, lib.tbg_group_open_shards(ctypes.byref(o), ctypes.byref(ops), arr), o,
                   owner=(ops, arr))

    def close(self):
        if self.g:
            self.lib.tbg_group_close(self.g)
            self.g = None

    def _check(self, rc, what):
        if rc < 0:
            raise RuntimeError(f"{what}: {rc} {self.lib.tbg_group_last_error(self.g).decode()}")
        return rc

    def shard(self, s):
        """Shard s's executor pointer (a tbg_ctx* for open_gpu)."""
        return self.lib.tbg_group_shard(self.g, s)

    def _create(self, fn, dtype, events, lens, batch_ts):
        ev = np.ascontiguousarray(events, dtype=dtype)
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        ts = np.ascontiguousarray(batch_ts, dtype=np.uint64)
        if int(ln.sum()) != len(ev):
            raise ValueError("batch lengths do not cover the events")
        out = np.zeros(len(ev), dtype=RESULT_DTYPE)
        self._check(fn(self.g, _ptr(ev), len(ev), _ptr(ln), _ptr(ts), len(ln), _ptr(out)),
                    fn.__name__)
        return out

    def create_accounts(self, events, lens, batch_ts):
        return self._create(self.lib.tbg_group_create_accounts, ACCOUNT_DTYPE, events, lens,
                            batch_ts)

    def create_transfers(self, events, lens, batch_ts):
        return self._create(self.lib.tbg_group_create_transfers, TRANSFER_DTYPE, events, lens,
                            batch_ts)

    def create_transfers_device(self, d_events, n, d_batch_ends, d_batch_ts, n_batches,
                                d_results):
        """Device pointers on the router's GPU; synchronous."""
        return self._check(self.lib.tbg_group_create_transfers_device(
            self.g, d_events, n, d_batch_ends, d_batch_ts, n_batches, d_results),
            "tbg_group_create_transfers_device")

    def pulse(self, timestamp):
        return self._check(self.lib.tbg_group_pulse(self.g, int(timestamp)), "tbg_group_pulse")

    def pulse_next_timestamp(self):
        return int(self.lib.tbg_group_pulse_next_timestamp(self.g))

    def _lookup(self, fn, ids, dtype):
        a = _u128_array(ids)
        out = np.zeros(len(a), dtype=dtype)
        n = self._check(fn(self.g, _ptr(a), len(a), _ptr(out)), fn.__name__)
        return out[:n]

    def lookup_accounts(self, ids):
        return self._lookup(self.lib.tbg_group_lookup_accounts, ids, ACCOUNT_DTYPE)

    def lookup_transfers(self, ids):
        return self._lookup(self.lib.tbg_group_lookup_transfers, ids, TRANSFER_DTYPE)

    def stats(self):
        s = GroupStats()
        self._check(self.lib.tbg_group_stats_read(self.g, ctypes.byref(s)), "stats")
        return {name: int(getattr(s, name)) for name, _ in GroupStats._fields_}

    def executor(self):
        """The group as a tb_executor (tb_sm_open binds it: the StateMachine over N GPUs)."""
        ex = native.Executor()
        self.lib.tbg_group_executor(self.g, ctypes.byref(ex))
        return ex

    def plan(self, transfers, events, lens, batch_ts, max_segments=4096):
        """Test hook: the exact engine's segments for a call against the current directories, as
        [(start, end, chain, [shard of each event])]."""
        ev = np.ascontiguousarray(events, dtype=TRANSFER_DTYPE if transfers else ACCOUNT_DTYPE)
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        ts = np.ascontiguousarray(batch_ts, dtype=np.uint64)
        ends = np.zeros(max_segments, dtype=np.uint32)
        flags = np.zeros(max_segments, dtype=np.uint8)
        place = np.zeros(max(len(ev), 1), dtype=np.int32)
        m = self._check(self.lib.tbg_group_plan(self.g, int(bool(transfers)), _ptr(ev), len(ev),
                                                _ptr(ln), _ptr(ts), len(ln), _ptr(ends),
                                                _ptr(flags), _ptr(place), max_segments),
                        "tbg_group_plan")
        out, start = [], 0
        for i in range(min(m, max_segments)):
            end = int(ends[i])
            out.append((start, end, bool(flags[i] & 1), place[start:end].tolist()))
            start = end
        return out

    def record_accounts(self, ids, shards):
        a = _u128_array(ids)
        sh = np.ascontiguousarray(shards, dtype=np.uint8)
        self._check(self.lib.tbg_group_record_accounts(self.g, _ptr(a), _ptr(sh), len(a)),
                    "tbg_group_record_accounts")

    def record_transfers(self, ids, shards):
        a = _u128_array(ids)
        sh = np.ascontiguousarray(shards, dtype=np.uint8)
        self._check(self.lib.tbg_group_record_transfers(self.g, _ptr(a), _ptr(sh), len(a)),
                    "tbg_group_record_transfers")


class GpuShard:
    """One HIP executor (tbg.h, its HBM tables on `device`) with numpy calls -- a group's shard
    (`wrap`) or a standalone executor."""

    def __init__(self, account_capacity, transfer_capacity, batch_events_max=1 << 16,
                 batch_count_max=4096, pulse_batch_max=8190, device=0,
                 pulse_next_timestamp_init=(1 << 63) - 1, account_events_capacity=0):
        self.lib = native.load()
        o = native.options(account_capacity, transfer_capacity, batch_events_max,
                           batch_count_max, pulse_batch_max, device, pulse_next_timestamp_init,
                           account_events_capacity)
        self.g = self.lib.tbg_open(ctypes.byref(o))
        self._owned = True
        if not self.g:
            raise RuntimeError("tbg_open failed")

    @classmethod
    def wrap(cls, lib, g):
        """A shard over an executor someone else owns (a group's: closing it is theirs)."""
        self = cls.__new__(cls)
        self.lib, self.g, self._owned = lib, g, False
        return self

    def close(self):
        if self.g and self._owned:
            self.lib.tbg_close(self.g)
        self.g = None

    def _err(self, rc):
        raise RuntimeError(f"libtbg: {rc} {self.lib.tbg_last_error(self.g)}")

    def _call(self, fn, events, dtype, lens, batch_ts):
        ev = np.ascontiguousarray(events, dtype=dtype)
        ln = np.ascontiguousarray(lens, dtype=np.uint32)
        ts = np.ascontiguousarray(batch_ts, dtype=np.uint64)
        out = np.zeros(len(ev), dtype=RESULT_DTYPE)
        rc = fn(self.g, _ptr(ev), len(ev), ln.ctypes.data_as(native.c_u32p),
                ts.ctypes.data_as(native.c_u64p), len(ln), _ptr(out))
        if rc != 0:
            self._err(rc)
        return out

    def create_accounts(self, events, lens, batch_ts):
        return self._call(self.lib.tbg_create_accounts, events, ACCOUNT_DTYPE, lens, batch_ts)

    def create_transfers(self, events, lens, batch_ts):
        return self._call(self.lib.tbg_create_transfers, events, TRANSFER_DTYPE, lens, batch_ts)

    def pulse(self, timestamp):
        return int(self.lib.tbg_pulse(self.g, timestamp))

    def pulse_next_timestamp(self):
        return int(self.lib.tbg_pulse_next_timestamp(self.g))

    def dump(self):
        """(accounts, transfers, TransferPending statuses) in creation order."""
        na = self.lib.tbg_dump_accounts(self.g, None)
        a = np.zeros(max(na, 0), dtype=ACCOUNT_DTYPE)
        self.lib.tbg_dump_accounts(self.g, _ptr(a))
        nt = self.lib.tbg_dump_transfers(self.g, None, None)
        t = np.zeros(max(nt, 0), dtype=TRANSFER_DTYPE)
        s = np.zeros(max(nt, 0), dtype=np.uint8)
        self.lib.tbg_dump_transfers(self.g, _ptr(t), _ptr(s))
        return a, t, s

    def dump_account_events(self):
        """This executor's AccountEvents in timestamp order (tbg_dump_account_events)."""
        from .types import ACCOUNT_EVENT_DTYPE
        n = self.lib.tbg_dump_account_events(self.g, None)
        e = np.zeros(max(n, 0), dtype=ACCOUNT_EVENT_DTYPE)
        if n > 0:
            self.lib.tbg_dump_account_events(self.g, _ptr(e))
        return e
