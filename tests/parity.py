"""Executor-level parity harness: the HIP executor (libtbg.so) against the CPU oracle.

Both sides receive the same calls -- create_accounts / create_transfers over multi-batch commits,
pulses when `pulse_needed` -- with timestamps advanced by the TestContext rule
(state_machine_tests.zig:230-241: prepare_ts += 1 + events). Results must be byte-identical and,
at the end, so must every live Account row, every live Transfer row and every TransferPending
status (in creation order).
"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from tigerbeetle_amd import native  # noqa: E402
from tigerbeetle_amd.types import (  # noqa: E402
    ACCOUNT_DTYPE, ACCOUNT_EVENT_DTYPE, CHANGE_EVENT_DTYPE, CHANGE_EVENTS_FILTER_DTYPE,
    ACCOUNT_BALANCE_DTYPE, ACCOUNT_FILTER_DTYPE, QUERY_FILTER_DTYPE,
    RESULT_DTYPE, TRANSFER_DTYPE, TIMESTAMP_MAX, CreateAccountStatus, CreateTransferStatus)

import oracle_binding  # noqa: E402


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class ParityError(AssertionError):
    pass


class _DeviceBuffers:
    """hipMalloc'd body / batch bounds / results for Pair(device_calls=True)."""

    def __init__(self, events_max, batches_max):
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        self.hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_int]
        self.hip.hipFree.argtypes = [ctypes.c_void_p]
        self.hip.hipDeviceSynchronize.argtypes = []
        self.ev = self._alloc(events_max * 128)
        self.res = self._alloc(events_max * 16)
        self.ends = self._alloc(batches_max * 4)
        self.ts = self._alloc(batches_max * 8)

    def _alloc(self, nbytes):
        p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(p), nbytes) == 0, "hipMalloc"
        return p

    def put(self, p, a):
        # (the previous call's queued work -- AccountEvents appends read its body -- has finished:
        # the device call's contract is the stream's order)
        assert self.hip.hipDeviceSynchronize() == 0
        a = np.ascontiguousarray(a)
        assert self.hip.hipMemcpy(p, a.ctypes.data_as(ctypes.c_void_p), a.nbytes, 1) == 0

    def get(self, p, a):
        assert self.hip.hipDeviceSynchronize() == 0
        assert self.hip.hipMemcpy(a.ctypes.data_as(ctypes.c_void_p), p, a.nbytes, 2) == 0

    def free(self):
        for p in (self.ev, self.res, self.ends, self.ts):
            self.hip.hipFree(p)


class Pair:
    def __init__(self, account_capacity=1 << 16, transfer_capacity=1 << 20,
                 batch_events_max=1 << 16, batch_count_max=4096, pulse_batch_max=8190,
                 pulse_next_timestamp_init=TIMESTAMP_MAX, force_replay=False, device=0,
                 account_events=True, registered=False, device_calls=False):
        self.lib = native.load()
        self.olib = oracle_binding.load()
        o = native.TbgOptions()
        o.account_capacity = account_capacity
        o.transfer_capacity = transfer_capacity
        o.batch_events_max = batch_events_max
        o.batch_count_max = batch_count_max
        o.pulse_batch_max = pulse_batch_max
        o.device = device
        o.pulse_next_timestamp_init = pulse_next_timestamp_init
        # AccountEvents (one per created transfer and per expiry), compared in compare_state.
        o.account_events_capacity = 2 * transfer_capacity if account_events else 0
        self.account_events = account_events
        self.opt = o
        self.g = self.lib.tbg_open(ctypes.byref(o))
        if not self.g:
            raise RuntimeError("tbg_open failed")
        self._force_replay = force_replay
        self._apply_debug_modes()
        # registered: create_transfers bodies and results go through one page-aligned host pool
        # registered with the executor (tbg_register_host), as a replica's message pool: the
        # kernels read the body and write the results over PCIe (hostio.hpp, tr_ingest).
        self._pool = None
        if registered:
            ev_bytes = batch_events_max * 128
            raw = np.zeros(ev_bytes + batch_events_max * 16 + 8192, dtype=np.uint8)
            off = (-raw.ctypes.data) % 4096
            self._pool_raw = raw
            self._pool = raw[off:off + ev_bytes + batch_events_max * 16 + 4096]
            assert self.lib.tbg_register_host(self.g, self._pool.ctypes.data,
                                              self._pool.nbytes) == 0
            self._pool_results = ev_bytes
        # device_calls: create_transfers through tbg_create_transfers_device, body, batch bounds
        # and results in HBM (hipMalloc'd here), results copied back after the call.
        self._dev = _DeviceBuffers(batch_events_max, batch_count_max) if device_calls else None
        self.o = self.olib.tbo_open(pulse_batch_max, pulse_next_timestamp_init)
        self.prepare_timestamp = 0
        self._pulse_delta = pulse_batch_max
        self.calls = 0
        self.stats = {"events": 0, "fast": 0, "replayed": 0, "static_fail": 0, "ae_window": 0,
                      "ingest_finished": 0}
        self.seconds = {"gpu": 0.0, "oracle": 0.0}  # wall time of each side's create_* calls
        self.pulses = []  # per tbg_pulse: (wall seconds, transfers expired)

    def _apply_debug_modes(self):
        force_replay = self._force_replay
        if force_replay:  # True: every event through the flow replay; "serial": on one lane
            self.lib.tbg_debug_force_replay(self.g, 1)
        if force_replay == "serial":  # (and the appends on the call's stream)
            self.lib.tbg_debug_serial_replay(self.g, 1)
            self.lib.tbg_debug_ae_sync(self.g, 1)

    def compact(self):
        """tbg_compact on the executor (the oracle has nothing to compact); rows freed."""
        n = self.lib.tbg_compact(self.g)
        if n < 0:
            raise RuntimeError(f"tbg_compact: {n} {self.lib.tbg_last_error(self.g)}")
        return n

    def checkpoint_reopen(self, path):
        """Checkpoint the executor, close it, and continue on a ctx opened from the image."""
        rc = self.lib.tbg_checkpoint(self.g, str(path).encode())
        if rc != 0:
            raise RuntimeError(f"tbg_checkpoint: {rc} {self.lib.tbg_last_error(self.g)}")
        self.lib.tbg_close(self.g)
        self.g = self.lib.tbg_open_checkpoint(ctypes.byref(self.opt), str(path).encode())
        if not self.g:
            raise RuntimeError("tbg_open_checkpoint failed")
        self._apply_debug_modes()

    def close(self):
        if self._dev is not None:
            self._dev.free()
            self._dev = None
        if self.g:
            self.lib.tbg_close(self.g)
            self.g = None
        if self.o:
            self.olib.tbo_close(self.o)
            self.o = None

    def _batches(self, lens):
        """One commit holding len(lens) batches (a multi-batch body)."""
        n = int(sum(lens))
        self.prepare_timestamp += 1 + n
        ts = self.prepare_timestamp
        ends = np.cumsum(np.asarray(lens, dtype=np.int64))
        batch_ts = (ts - n + ends).astype(np.uint64)
        return n, np.asarray(lens, dtype=np.uint32), batch_ts

    def _check(self, kind, events, r_gpu, r_orc):
        if r_gpu.tobytes() != r_orc.tobytes():
            bad = np.nonzero((r_gpu["status"] != r_orc["status"]) |
                             (r_gpu["timestamp"] != r_orc["timestamp"]))[0]
            enum_t = CreateAccountStatus if kind == "accounts" else CreateTransferStatus
            lines = [f"create_{kind} call #{self.calls}: {len(bad)} results differ"]
            for i in bad[:12]:
                def name(s):
                    try:
                        return enum_t(int(s)).name
                    except ValueError:
                        return str(int(s))
                lines.append(f"  [{i}] gpu=({int(r_gpu[i]['timestamp'])}, "
                             f"{name(r_gpu[i]['status'])}) oracle=({int(r_orc[i]['timestamp'])}, "
                             f"{name(r_orc[i]['status'])}) flags={int(events[i]['flags']):#x}")
            raise ParityError("\n".join(lines))

    def _stats(self):
        s = native.TbgStats()
        self.lib.tbg_last_stats(self.g, ctypes.byref(s))
        self.last_stats = {k: getattr(s, k) for k in self.stats}
        for k in self.stats:
            self.stats[k] += getattr(s, k)

    def create_accounts(self, events: np.ndarray, lens=None):
        events = np.ascontiguousarray(events, dtype=ACCOUNT_DTYPE)
        lens = [len(events)] if lens is None else lens
        n, lens_a, batch_ts = self._batches(lens)
        r_gpu = np.zeros(n, dtype=RESULT_DTYPE)
        r_orc = np.zeros(n, dtype=RESULT_DTYPE)
        rc = self.lib.tbg_create_accounts(
            self.g, _ptr(events), n, lens_a.ctypes.data_as(native.c_u32p),
            batch_ts.ctypes.data_as(native.c_u64p), len(lens), _ptr(r_gpu))
        if rc != 0:
            raise RuntimeError(f"tbg_create_accounts: {rc} {self.lib.tbg_last_error(self.g)}")
        off = 0
        for b, ln in enumerate(lens):
            self.olib.tbo_create_accounts(self.o, _ptr(events[off:off + ln]), ln,
                                          int(batch_ts[b]), _ptr(r_orc[off:off + ln]))
            off += ln
        self.calls += 1
        self._stats()
        self._check("accounts", events, r_gpu, r_orc)
        self._maybe_pulse()
        return r_orc

    def create_transfers(self, events: np.ndarray, lens=None):
        events = np.ascontiguousarray(events, dtype=TRANSFER_DTYPE)
        lens = [len(events)] if lens is None else lens
        n, lens_a, batch_ts = self._batches(lens)
        r_gpu = np.zeros(n, dtype=RESULT_DTYPE)
        r_orc = np.zeros(n, dtype=RESULT_DTYPE)
        t0 = time.perf_counter()
        if self._dev is not None:
            D = self._dev
            D.put(D.ev, events)
            D.put(D.ends, np.cumsum(lens_a, dtype=np.uint32))
            D.put(D.ts, batch_ts)
            rc = self.lib.tbg_create_transfers_device(self.g, D.ev, n, D.ends, D.ts, len(lens),
                                                      D.res, None)
            if rc == 0:
                D.get(D.res, r_gpu)
        elif self._pool is not None:
            body = self._pool[:n * 128]
            body[:] = events.view(np.uint8).reshape(-1)
            res = self._pool[self._pool_results:self._pool_results + n * 16]
            rc = self.lib.tbg_create_transfers(
                self.g, ctypes.c_void_p(body.ctypes.data), n, lens_a.ctypes.data_as(native.c_u32p),
                batch_ts.ctypes.data_as(native.c_u64p), len(lens), ctypes.c_void_p(res.ctypes.data))
            r_gpu[:] = res.view(RESULT_DTYPE)
        else:
            rc = self.lib.tbg_create_transfers(
                self.g, _ptr(events), n, lens_a.ctypes.data_as(native.c_u32p),
                batch_ts.ctypes.data_as(native.c_u64p), len(lens), _ptr(r_gpu))
        t1 = time.perf_counter()
        if rc != 0:
            raise RuntimeError(f"tbg_create_transfers: {rc} {self.lib.tbg_last_error(self.g)}")
        off = 0
        for b, ln in enumerate(lens):
            self.olib.tbo_create_transfers(self.o, _ptr(events[off:off + ln]), ln,
                                           int(batch_ts[b]), _ptr(r_orc[off:off + ln]))
            off += ln
        self.seconds["gpu"] += t1 - t0
        self.seconds["oracle"] += time.perf_counter() - t1
        self.calls += 1
        self._stats()
        self._check("transfers", events, r_gpu, r_orc)
        self._maybe_pulse()
        return r_orc

    def set_balances(self, account_id, dp=0, dpo=0, cp=0, cpo=0):
        """Debug balance setter on both sides (the reference's table harness `setup`)."""
        U = native.U128.of
        a = self.lib.tbg_debug_set_account_balances(self.g, U(account_id), U(dp), U(dpo), U(cp),
                                                    U(cpo))
        b = self.olib.tbo_set_account_balances(self.o, U(account_id), U(dp), U(dpo), U(cp),
                                               U(cpo))
        assert a == 0 and b == 0, (a, b)

    def pulse_next(self):
        a = self.lib.tbg_pulse_next_timestamp(self.g)
        b = self.olib.tbo_pulse_next_timestamp(self.o)
        if a != b:
            raise ParityError(f"pulse_next_timestamp: gpu={a} oracle={b} (call #{self.calls})")
        return a

    def _maybe_pulse(self):
        # Best-effort pulse after the commit (state_machine_tests.zig:201-207, :243-256).
        if self.pulse_next() <= self.prepare_timestamp:
            # prepare(pulse): prepare_ts += 1 + batch_max.create_transfers (:1113).
            self.prepare_timestamp += 1 + self._pulse_delta
            ts = self.prepare_timestamp
            t0 = time.perf_counter()
            eg = self.lib.tbg_pulse(self.g, ts)
            self.pulses.append((time.perf_counter() - t0, eg))  # (wall seconds, expired)
            eo = self.olib.tbo_pulse(self.o, ts)
            if eg != eo:
                raise ParityError(f"pulse at {ts}: gpu expired {eg}, oracle {eo}")
            self.pulse_next()

    def tick(self, ns: int):
        self.prepare_timestamp += ns
        self._maybe_pulse()

    def compare_state(self):
        na = self.lib.tbg_dump_accounts(self.g, None)
        a_gpu = np.zeros(max(na, 0), dtype=ACCOUNT_DTYPE)
        self.lib.tbg_dump_accounts(self.g, _ptr(a_gpu))
        a_orc = np.zeros(self.olib.tbo_account_count(self.o), dtype=ACCOUNT_DTYPE)
        self.olib.tbo_dump_accounts(self.o, _ptr(a_orc))
        if a_gpu.tobytes() != a_orc.tobytes():
            raise ParityError(f"accounts differ: gpu {len(a_gpu)} rows, oracle {len(a_orc)} rows; "
                              f"first diff at {_first_diff(a_gpu, a_orc)}")
        nt = self.lib.tbg_dump_transfers(self.g, None, None)
        t_gpu = np.zeros(max(nt, 0), dtype=TRANSFER_DTYPE)
        s_gpu = np.zeros(max(nt, 0), dtype=np.uint8)
        self.lib.tbg_dump_transfers(self.g, _ptr(t_gpu), _ptr(s_gpu))
        ntr = self.olib.tbo_transfer_count(self.o)
        t_orc = np.zeros(ntr, dtype=TRANSFER_DTYPE)
        s_orc = np.zeros(ntr, dtype=np.uint8)
        self.olib.tbo_dump_transfers(self.o, _ptr(t_orc))
        self.olib.tbo_dump_pending_status(self.o, _ptr(s_orc))
        if t_gpu.tobytes() != t_orc.tobytes():
            raise ParityError(f"transfers differ: gpu {len(t_gpu)} rows, oracle {len(t_orc)}; "
                              f"first diff at {_first_diff(t_gpu, t_orc)}")
        if s_gpu.tobytes() != s_orc.tobytes():
            raise ParityError("TransferPending statuses differ")
        if self.account_events:
            ne = self.lib.tbg_dump_account_events(self.g, None)
            e_gpu = np.zeros(max(ne, 0), dtype=ACCOUNT_EVENT_DTYPE)
            self.lib.tbg_dump_account_events(self.g, _ptr(e_gpu))
            e_orc = np.zeros(self.olib.tbo_dump_account_events(self.o, None),
                             dtype=ACCOUNT_EVENT_DTYPE)
            self.olib.tbo_dump_account_events(self.o, _ptr(e_orc))
            # (the groove is keyed by timestamp: the oracle's insertion order sorted, stable)
            e_orc = e_orc[np.argsort(e_orc["timestamp"], kind="stable")]
            if e_gpu.tobytes() != e_orc.tobytes():
                raise ParityError(f"account events differ: gpu {len(e_gpu)}, oracle {len(e_orc)}; "
                                  f"first diff at {_first_diff(e_gpu, e_orc)}")
        return len(a_orc), len(t_orc)

    def scan(self, kind, f, limit_max=8190):
        """One scan on both sides (tbg_* vs tbo_*); they must agree byte for byte."""
        dt = {"get_account_balances": ACCOUNT_BALANCE_DTYPE,
              "query_accounts": ACCOUNT_DTYPE}.get(kind, TRANSFER_DTYPE)
        g = np.zeros(limit_max, dtype=dt)
        o = np.zeros(limit_max, dtype=dt)
        ng = getattr(self.lib, "tbg_" + kind)(self.g, _ptr(f), limit_max, _ptr(g))
        no = getattr(self.olib, "tbo_" + kind)(self.o, _ptr(f), limit_max, _ptr(o))
        if ng != no or g[:max(ng, 0)].tobytes() != o[:no].tobytes():
            raise ParityError(f"{kind} differs: gpu {ng}, oracle {no}, filter {f}; first diff at "
                              f"{_first_diff(g[:max(ng, 0)], o[:no])}")
        return no

    def compare_scans(self, rng, n=40, limit_max=8190):
        """`n` seeded filters over the current tables (random_scan_filters); returns the total
        number of results compared."""
        na = self.olib.tbo_account_count(self.o)
        nt = self.olib.tbo_transfer_count(self.o)
        a = np.zeros(na, dtype=ACCOUNT_DTYPE)
        t = np.zeros(nt, dtype=TRANSFER_DTYPE)
        self.olib.tbo_dump_accounts(self.o, _ptr(a))
        self.olib.tbo_dump_transfers(self.o, _ptr(t))
        total = 0
        for kind, f in random_scan_filters(rng, a, t, n):
            if kind == "get_account_balances" and not self.account_events:
                continue
            total += self.scan(kind, f, limit_max)
        return total

    def change_events(self, timestamp_min=0, timestamp_max=0, limit=1 << 31, limit_max=8190):
        """get_change_events on both sides; they must agree byte for byte."""
        f = np.zeros(1, dtype=CHANGE_EVENTS_FILTER_DTYPE)
        f["timestamp_min"], f["timestamp_max"], f["limit"] = timestamp_min, timestamp_max, limit
        cap = min(limit, limit_max)
        g = np.zeros(cap, dtype=CHANGE_EVENT_DTYPE)
        o = np.zeros(cap, dtype=CHANGE_EVENT_DTYPE)
        ng = self.lib.tbg_get_change_events(self.g, _ptr(f), limit_max, _ptr(g))
        no = self.olib.tbo_get_change_events(self.o, _ptr(f), limit_max, _ptr(o))
        if ng != no or g[:ng].tobytes() != o[:no].tobytes():
            raise ParityError(f"get_change_events differ: gpu {ng}, oracle {no}; first diff at "
                              f"{_first_diff(g[:ng], o[:no])}")
        return g[:ng]


def _pick(rng, values, zero_p=0.5):
    """0 (no condition) with probability zero_p, else one of `values` (or a random miss)."""
    if len(values) == 0 or rng.random() < zero_p:
        return 0
    return int(values[rng.integers(0, len(values))]) if rng.random() < 0.9 else \
        int(rng.integers(1, 1 << 30))


def random_scan_filters(rng, accounts, transfers, n):
    """Seeded AccountFilters and QueryFilters drawn from the objects that exist (so that most
    conditions match something), with random timestamp ranges, limits, orders, and a few invalid
    filters (zero limit, inverted range, no side, padding bits, reserved bytes)."""
    ts = transfers["timestamp"] if len(transfers) else np.zeros(1, dtype=np.uint64)
    ats = accounts["timestamp"] if len(accounts) else np.zeros(1, dtype=np.uint64)
    out = []
    for _ in range(n):
        kind = rng.choice(["get_account_transfers", "get_account_balances", "query_accounts",
                           "query_transfers"])
        if kind.startswith("get_"):
            f = np.zeros(1, dtype=ACCOUNT_FILTER_DTYPE)
            src = accounts["id"][:, 0] if len(accounts) else np.zeros(1, dtype=np.uint64)
            f["account_id"][0, 0] = src[rng.integers(0, len(src))] if rng.random() < 0.95 else 0
            f["user_data_128"][0, 0] = _pick(rng, transfers["user_data_128"][:, 0], 0.8)
            f["user_data_64"] = _pick(rng, transfers["user_data_64"], 0.85)
            f["user_data_32"] = _pick(rng, transfers["user_data_32"], 0.85)
            f["code"] = _pick(rng, transfers["code"], 0.8) & 0xFFFF
            f["flags"] = int(rng.choice([1, 2, 3, 3, 5, 6, 7, 7, 0, 8]))
            tsrc = ts
        else:
            f = np.zeros(1, dtype=QUERY_FILTER_DTYPE)
            objs = accounts if kind == "query_accounts" else transfers
            if len(objs):
                f["user_data_128"][0, 0] = _pick(rng, objs["user_data_128"][:, 0], 0.7)
                f["user_data_64"] = _pick(rng, objs["user_data_64"], 0.8)
                f["user_data_32"] = _pick(rng, objs["user_data_32"], 0.8)
                f["ledger"] = _pick(rng, objs["ledger"], 0.5)
                f["code"] = _pick(rng, objs["code"], 0.7) & 0xFFFF
            f["flags"] = int(rng.choice([0, 0, 1, 1, 2]))
            tsrc = ats if kind == "query_accounts" else ts
        r = rng.random()
        if r < 0.5:
            lo, hi = sorted(int(x) for x in rng.choice(tsrc, size=2))
            f["timestamp_min"], f["timestamp_max"] = lo, hi
        elif r < 0.6:
            f["timestamp_min"] = int(rng.choice(tsrc))
        elif r < 0.65:
            lo, hi = sorted(int(x) for x in rng.choice(tsrc, size=2))
            f["timestamp_min"], f["timestamp_max"] = hi + 1, lo  # inverted
        f["limit"] = int(rng.choice([1, 2, 5, 30, 1000, 0xFFFFFFFF, 0]))
        if rng.random() < 0.03:
            f["reserved"][0, 0] = 1
        out.append((kind, f))
    return out


def _first_diff(a, b):
    n = min(len(a), len(b))
    for i in range(n):
        if a[i].tobytes() != b[i].tobytes():
            return f"row {i}: gpu={a[i]} oracle={b[i]}"
    return f"length {len(a)} vs {len(b)}"
