"""Ledger sharding of the commit path across GPUs.

Debit and credit accounts of a transfer must share the transfer's ledger
(`accounts_must_have_the_same_ledger`, `transfer_must_have_the_same_ledger_as_accounts`,
src/state_machine.zig:3795-3798), so ledgers are independent shards: one executor per GPU owns a
contiguous range of ledgers -- their accounts, transfer ids, transfer rows and TransferPending
statuses. A client call (a multi-batch commit) is split by a router on the owner of the call,
each shard's slice travels to its GPU (point-to-point sends: RCCL over xGMI with the `nccl`
backend, gloo on CPU), every shard executes its slice, and the 16-byte results come back.

Exactness. A shard executes its slice as the reference would execute the whole call only if no
event of the slice can observe state held by another shard. `LedgerRouter` routes by
directories of where each account id and each transfer id (created, or orphaned by a transient
failure) lives. Hazards it executes exactly:

* a transfer whose debit and credit accounts live on different shards: the reference answers
  `accounts_must_have_the_same_ledger` (:3795-3798) unless an earlier static check fails first
  (:3774-3794), and never reads a balance. The router computes that status and sends the shard
  executing the event's chain a *surrogate* -- the event with its credit account set to its debit
  account -- which fails at the same position with `accounts_must_be_different`, non-transient
  like the true status, so a chain around it is rolled back exactly as the reference rolls it back;
  the router then writes the true status into the result;
* imported batches: their `must_not_regress` checks read the objects trees' global key ranges
  (:3656-3665, :3808-3817), so every shard's key maxima are raised to the global ones before the
  call (`raise_key_max`).

Refused (`RouteError`, before any shard executes) -- the remaining cases no shard can execute
alone:

* a linked chain whose (non-surrogate) events belong to different shards: a chain is atomic
  (:3002-3213) and its rollback would span shards;
* an id repeated within the call where the repeat could execute on a shard other than the
  first occurrence's (a duplicate's outcome depends on the first occurrence's result), or a
  cross-shard transfer whose id repeats an id of the call;
* imported events whose outcome depends on another shard: a timestamp at or below an imported
  timestamp of an earlier event of the call on another shard, or at or below the other groove's
  key maximum (a possible timestamp collision, :3660, :3812).

A post/void of a pending transfer that has a timeout resets `pulse_next_timestamp` when that
equals the pending transfer's expiry (:4227-4229) -- a comparison against the *global* value at
that point of the call, which no shard holds. The shards run with sharded pulse_next_timestamp
(`set_pnt_sharded`): each records every update at its event (min of a pending transfer's expiry,
applied; reset-if-equal of a post/void, only recorded) with the event's global timestamp. After a
call holding a post/void the updates of every shard are gathered, merged by timestamp and replayed
from the minimum of the shards' values at the call's start (`pnt_resets_fire`); when a reset
fires, every shard's value becomes timestamp_min -- the reference's value. No event's outcome
reads the value (only pulses do, between calls), so the call itself runs unchanged.

Events whose outcome is decided before any shard-local lookup can fail (`id_must_not_be_zero`,
accounts not found anywhere, pending transfer not found anywhere) go to the shard of their ledger.
An event whose id already exists goes to the shard holding it: `create_transfer_exists` and
`create_account_exists` run before any account lookup (:3636, :3733), and a post/void that exists
finds its pending transfer on the same shard (it was created there by posting it).

Timestamps are global: event k of batch b is stamped `batch_ts[b] - len[b] + k + 1`
(`execute_multi_batch`, :2702-2762). A shard receives each batch's events as maximal runs of
consecutive positions, each run a sub-batch whose timestamp is that of its last event, so every
event keeps its global timestamp. Runs never cut a chain (a chain crossing a run edge crosses a
shard edge, which the router refused), and no batch-level check besides chain ends and the
imported flag depends on the batch extent.

pulse: with the resets above excluded, `pulse_next_timestamp` only moves by `min` between pulses
(:3979-3980), so the sharded value is the minimum over shards (an all-reduce). The reference's
pulse scans the expires_at index in (expires_at, timestamp) order and stops after
`pulse_batch_max` entries, setting `pulse_next_timestamp` from the last one (:4969-4999,
scan_lookup.zig:150-175). Sharded: every shard reports how many of its entries have expired and
the first `pulse_batch_max` of their keys (an all-gather); below `pulse_batch_max` in total every
shard expires all of its own (and keeps its earliest unexpired expiry, whose minimum over shards
is the reference's); otherwise the `pulse_batch_max`-th key across shards is the cut: each shard
expires its entries up to it and sets `pulse_next_timestamp` to the cut's expiry. Timestamps are
unique, so the cut expires exactly `pulse_batch_max` transfers -- the reference's. Each expiry is
stamped with its position in the pulse's order over all shards (`pulse_plan`), as the reference
stamps it (:4540-4546): its AccountEvent carries that timestamp.
"""
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Set

import numpy as np

from .types import (ACCOUNT_DTYPE, RESULT_DTYPE, STATUS_CREATED, TRANSFER_DTYPE,
                    TRANSIENT_TRANSFER_STATUSES, AccountFlags, TransferFlags)

_U128_MAX = (1 << 128) - 1
# CreateTransferStatus values (src/tigerbeetle.zig:220-469) of the cross-shard checks.
_ACCOUNTS_MUST_BE_DIFFERENT = 12
_PENDING_ID_MUST_BE_ZERO = 13
_TIMEOUT_RESERVED_FOR_PENDING_TRANSFER = 17
_LEDGER_MUST_NOT_BE_ZERO = 19
_CODE_MUST_NOT_BE_ZERO = 20
_ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER = 23
_CLOSING_TRANSFER_MUST_BE_PENDING = 64


PNT_RESET = 1 << 63  # a recorded update that is a reset-if-equal (post/void of an expiry)
TIMESTAMP_MIN = 1


def pnt_resets_fire(starts, op_lists) -> bool:
    """Does a reset of pulse_next_timestamp fire in the call's order across shards? `starts`: the
    shards' values at the call's start; `op_lists`: per shard, its recorded updates as (event
    timestamp, op) -- op an expiry (a `min`), or an expiry | PNT_RESET (reset-if-equal)."""
    value = min(int(x) for x in starts)
    for _, op in sorted((int(t), int(o)) for ops in op_lists for t, o in ops):
        if op & PNT_RESET:
            if value == op & ~PNT_RESET:
                return True  # (timestamp_min from here on: every later `min` keeps it)
        elif op < value:
            value = op
    return False


class RouteError(RuntimeError):
    """The call holds an event that no single shard can execute exactly (see the module doc)."""


def _ids(col: np.ndarray) -> List[int]:
    lo = col[:, 0].tolist()
    hi = col[:, 1].tolist()
    return [a | (b << 64) for a, b in zip(lo, hi)]


@dataclass
class ShardSlice:
    """One shard's part of a call: global positions, sub-batch lengths and timestamps."""
    index: np.ndarray                       # int64 global positions, ascending
    lens: List[int] = field(default_factory=list)
    batch_ts: List[int] = field(default_factory=list)


@dataclass
class Plan:
    kind: str                               # "accounts" | "transfers"
    shard_of: np.ndarray                    # int32 per event
    slices: List[ShardSlice]
    # cross-shard transfers: event index -> the reference's status (the shard runs a surrogate)
    cross: Dict[int, int] = field(default_factory=dict)
    imported: bool = False                  # the call holds imported events (key ranges synced)
    post_void: bool = False                 # ... posts or voids (pulse_next_timestamp resolved)

    def shard_events(self, events: np.ndarray) -> np.ndarray:
        """The events as the shards execute them: cross-shard transfers as their surrogates."""
        if not self.cross:
            return events
        ev = events.copy()
        idx = np.fromiter(self.cross.keys(), dtype=np.int64)
        ev["credit_account_id"][idx] = ev["debit_account_id"][idx]
        return ev

    def patch(self, results: np.ndarray) -> np.ndarray:
        """The true statuses of cross-shard transfers whose surrogate failed as planned."""
        for k, st in self.cross.items():
            if int(results[k]["status"]) == _ACCOUNTS_MUST_BE_DIFFERENT:
                results[k]["status"] = st
        return results


def chain_starts(flags: np.ndarray, lens) -> np.ndarray:
    """True where an event starts a chain (a batch start, or the previous event is not linked)."""
    n = len(flags)
    start = np.ones(n, dtype=bool)
    if n > 1:
        start[1:] = (flags[:-1] & 1) == 0
    ends = np.cumsum(np.asarray(lens, dtype=np.int64))
    inner = ends[:-1]
    start[inner[inner < n]] = True
    return start


def split_runs(shard_of: np.ndarray, lens, batch_ts, shards: int) -> List[ShardSlice]:
    """Per shard, the maximal runs of consecutive positions of each batch, as sub-batches that
    keep every event's global timestamp."""
    slices = [ShardSlice(index=np.zeros(0, dtype=np.int64)) for _ in range(shards)]
    parts: List[List[np.ndarray]] = [[] for _ in range(shards)]
    s = 0
    for b, ln in enumerate(lens):
        ln = int(ln)
        if ln == 0:
            continue
        seg = shard_of[s:s + ln]
        cut = np.nonzero(np.diff(seg))[0] + 1
        starts = np.concatenate([[0], cut]).tolist()
        stops = np.concatenate([cut, [ln]]).tolist()
        ts_b = int(batch_ts[b])
        for a, z in zip(starts, stops):
            sh = int(seg[a])
            parts[sh].append(np.arange(s + a, s + z, dtype=np.int64))
            slices[sh].lens.append(z - a)
            # the run's last event (batch position z - 1) is stamped ts_b - ln + z
            slices[sh].batch_ts.append(ts_b - ln + z)
        s += ln
    for sh in range(shards):
        if parts[sh]:
            slices[sh].index = np.concatenate(parts[sh])
    return slices


class DictDirectory:
    """Host-side directories: account id -> shard; transfer id (created or orphaned) -> (shard,
    timed: a pending transfer with a timeout). The device router keeps the same directories in
    HBM (DeviceDirectory, include/tbr.h)."""

    def __init__(self):
        self.accounts: Dict[int, int] = {}
        self.transfers: Dict[int, tuple] = {}

    def account_shards(self, ids: List[int]) -> List[Optional[int]]:
        return [self.accounts.get(i) for i in ids]

    def transfer_info(self, ids: List[int]) -> List[Optional[tuple]]:
        return [self.transfers.get(i) for i in ids]

    def record_accounts(self, ids: List[int], shards: List[int]):
        for i, sh in zip(ids, shards):
            self.accounts[i] = sh

    def record_transfers(self, ids: List[int], shards: List[int], timed: List[bool]):
        for i, sh, t in zip(ids, shards, timed):
            self.transfers.setdefault(i, (sh, t))


def _u128_array(ids: List[int]) -> np.ndarray:
    a = np.zeros((len(ids), 2), dtype=np.uint64)
    if ids:
        a[:, 0] = [i & 0xFFFFFFFFFFFFFFFF for i in ids]
        a[:, 1] = [i >> 64 for i in ids]
    return a


class DeviceDirectory:
    """The directories of the device router (tbr_ctx, include/tbr.h), read and written in bulk:
    one source of truth for the device fast path and the exact host path."""
    TIMED = 0x80

    def __init__(self, lib, tbr):
        self.lib = lib
        self.tbr = tbr

    def _lookup(self, fn, ids):
        import ctypes
        if not ids:
            return []
        a = _u128_array(ids)
        out = np.zeros(len(ids), dtype=np.int32)
        rc = fn(self.tbr, a.ctypes.data_as(ctypes.c_void_p), len(ids),
                out.ctypes.data_as(ctypes.c_void_p))
        if rc < 0:
            raise RuntimeError(f"tbr lookup: {rc}")
        return out.tolist()

    def account_shards(self, ids):
        return [None if x < 0 else x for x in self._lookup(self.lib.tbr_account_shards, ids)]

    def transfer_info(self, ids):
        return [None if x < 0 else (x & 0x7F, bool(x & self.TIMED))
                for x in self._lookup(self.lib.tbr_transfer_shards, ids)]

    def _record(self, fn, ids, shards):
        import ctypes
        if not ids:
            return
        a = _u128_array(ids)
        sh = np.asarray(shards, dtype=np.uint8)
        rc = fn(self.tbr, a.ctypes.data_as(ctypes.c_void_p), sh.ctypes.data_as(ctypes.c_void_p),
                len(ids))
        if rc != 0:
            raise RuntimeError(f"tbr record: {rc}")

    def record_accounts(self, ids, shards):
        self._record(self.lib.tbr_record_accounts, ids, shards)

    def record_transfers(self, ids, shards, timed):
        self._record(self.lib.tbr_record_transfers, ids,
                     [s | (self.TIMED if t else 0) for s, t in zip(shards, timed)])


class LedgerRouter:
    """Routes create_accounts / create_transfers calls to ledger shards (module doc).

    Ledgers 1..`ledgers` map to shards by contiguous ranges (64 ledgers / G);
    other ledgers by `ledger % shards`. Placement of a new account follows its ledger; routing
    of later events follows the directories, so a placement never has to be recomputed.
    """

    def __init__(self, shards: int, ledgers: int = 64, directory=None):
        if shards < 1:
            raise ValueError("shards must be >= 1")
        self.shards = shards
        self.ledgers = ledgers
        self.dir = directory if directory is not None else DictDirectory()
        # objects trees' key_range.key_max over all shards (largest created timestamp)
        self.accounts_key_max = 0
        self.transfers_key_max = 0

    def shard_of_ledger(self, ledger: int) -> int:
        if 1 <= ledger <= self.ledgers:
            return (ledger - 1) * self.shards // self.ledgers
        return ledger % self.shards

    # -- planning ---------------------------------------------------------------------------

    @staticmethod
    def _place_chains(n, starts, pins_of, default_of, record):
        shard_of = np.zeros(n, dtype=np.int32)
        bounds = np.concatenate([np.nonzero(starts)[0], [n]]).astype(np.int64).tolist()
        for a, z in zip(bounds[:-1], bounds[1:]):
            pins = set()
            for k in range(a, z):
                pins |= pins_of(k)
            if len(pins) > 1:
                what = "linked chain" if z - a > 1 else "event"
                raise RouteError(f"{what} at {a}..{z - 1} spans shards {sorted(pins)}")
            sh = pins.pop() if pins else default_of(a)
            shard_of[a:z] = sh
            for k in range(a, z):
                record(k, sh)
        return shard_of

    def _check_imported(self, imported: np.ndarray, own_ts: np.ndarray, lens, batch_ts,
                        shard_of: np.ndarray, other_key_max: int, what: str):
        """Imported events whose checks another shard's state could decide (module doc): every
        earlier event of the call on another shard may have raised the global key range to its
        timestamp (an imported event's own, else its commit timestamp)."""
        lens_a = np.asarray(lens, dtype=np.int64)
        starts = np.cumsum(lens_a) - lens_a
        within = np.arange(int(lens_a.sum()), dtype=np.int64) - np.repeat(starts, lens_a)
        ts = np.repeat(np.asarray(batch_ts, dtype=np.int64) - lens_a, lens_a) + within + 1
        ts = np.where(imported, own_ts.astype(np.int64), ts).tolist()
        imp = imported.tolist()
        sh_of = shard_of.tolist()
        latest: Dict[int, int] = {}  # shard -> largest timestamp of its events so far
        for k, (t, sh) in enumerate(zip(ts, sh_of)):
            if imp[k]:
                if t <= other_key_max:
                    raise RouteError(f"imported {what} {k}: timestamp {t} may collide with an "
                                     f"object of the other groove on another shard")
                for osh, ot in latest.items():
                    if osh != sh and t <= ot:
                        raise RouteError(f"imported {what} {k}: timestamp {t} may regress past "
                                         f"an event of shard {osh}")
            latest[sh] = max(latest.get(sh, 0), t)

    def plan_accounts(self, events: np.ndarray, lens, batch_ts) -> Plan:
        n = len(events)
        flags = events["flags"]
        imported = (flags & int(AccountFlags.imported)) != 0
        ids = _ids(events["id"])
        ledgers = events["ledger"].tolist()
        in_call: Dict[int, int] = {}
        uniq = list(set(ids))
        known = {i: sh for i, sh in zip(uniq, self.dir.account_shards(uniq)) if sh is not None}

        def pins_of(k):
            i = ids[k]
            if i in known:
                return {known[i]}
            if i in in_call:
                return {in_call[i]}
            return set()

        def record(k, sh):
            i = ids[k]
            if i not in known and i != 0 and i != _U128_MAX:
                in_call.setdefault(i, sh)

        shard_of = self._place_chains(n, chain_starts(flags, lens), pins_of,
                                      lambda a: self.shard_of_ledger(ledgers[a]), record)
        if n and imported.any():
            self._check_imported(imported, events["timestamp"], lens, batch_ts, shard_of,
                                 self.transfers_key_max, "account")
        return Plan("accounts", shard_of, split_runs(shard_of, lens, batch_ts, self.shards),
                    imported=bool(n and imported.any()))

    def plan_transfers(self, events: np.ndarray, lens, batch_ts) -> Plan:
        n = len(events)
        flags = events["flags"]
        imported = (flags & int(TransferFlags.imported)) != 0
        ids = _ids(events["id"])
        drs = _ids(events["debit_account_id"])
        crs = _ids(events["credit_account_id"])
        pids = _ids(events["pending_id"])
        ledgers = events["ledger"].tolist()
        codes = events["code"].tolist()
        timeouts = events["timeout"].tolist()
        fl = flags.tolist()
        in_call: Dict[int, int] = {}
        in_call_timed: Set[int] = set()
        cross: Dict[int, int] = {}
        post_void = int(TransferFlags.post_pending_transfer | TransferFlags.void_pending_transfer)
        pending = int(TransferFlags.pending)
        closing = int(TransferFlags.closing_debit | TransferFlags.closing_credit)
        # the directories' answers for every id of the call, in bulk
        uniq_t = list(set(ids) | set(pids))
        tr_known = {i: v for i, v in zip(uniq_t, self.dir.transfer_info(uniq_t)) if v is not None}
        uniq_a = list(set(drs) | set(crs))
        acc_known = {i: v for i, v in zip(uniq_a, self.dir.account_shards(uniq_a))
                     if v is not None}

        def cross_status(k):
            # create_transfer :3774-3798 after the account ids: both accounts exist, on shards of
            # different ledgers.
            if pids[k] != 0:
                return _PENDING_ID_MUST_BE_ZERO
            if not fl[k] & pending:
                if timeouts[k] != 0:
                    return _TIMEOUT_RESERVED_FOR_PENDING_TRANSFER
                if fl[k] & closing:
                    return _CLOSING_TRANSFER_MUST_BE_PENDING
            if ledgers[k] == 0:
                return _LEDGER_MUST_NOT_BE_ZERO
            if codes[k] == 0:
                return _CODE_MUST_NOT_BE_ZERO
            return _ACCOUNTS_MUST_HAVE_THE_SAME_LEDGER

        def pins_of(k):
            i = ids[k]
            if i in tr_known:  # exists / id_already_failed: decided on the holder
                return {tr_known[i][0]}
            pins = set()
            if i in in_call:  # the repeat executes in full if the first occurrence fails
                pins.add(in_call[i])
            if fl[k] & post_void:
                p = pids[k]
                if p in tr_known:
                    pins.add(tr_known[p][0])
                elif p in in_call:
                    pins.add(in_call[p])
            else:
                a_dr, a_cr = acc_known.get(drs[k]), acc_known.get(crs[k])
                if a_dr is not None and a_cr is not None and a_dr != a_cr:
                    if i in in_call:
                        raise RouteError(f"cross-shard transfer {k} repeats an id of the call")
                    cross[k] = cross_status(k)  # a surrogate, on whichever shard runs its chain
                else:
                    pins |= {a for a in (a_dr, a_cr) if a is not None}
            return pins

        def record(k, sh):
            i = ids[k]
            if i not in tr_known and i != 0 and i != _U128_MAX:
                in_call.setdefault(i, sh)
                if (fl[k] & pending) and timeouts[k] > 0:
                    in_call_timed.add(i)

        shard_of = self._place_chains(n, chain_starts(flags, lens), pins_of,
                                      lambda a: self.shard_of_ledger(ledgers[a]), record)
        if n and imported.any():
            self._check_imported(imported, events["timestamp"], lens, batch_ts, shard_of,
                                 self.accounts_key_max, "transfer")
        return Plan("transfers", shard_of, split_runs(shard_of, lens, batch_ts, self.shards),
                    cross=cross, imported=bool(n and imported.any()),
                    post_void=bool(n and ((flags & post_void) != 0).any()))

    # -- directories --------------------------------------------------------------------------

    def commit(self, plan: Plan, events: np.ndarray, results: np.ndarray):
        """Record where the call's new objects (and orphaned transfer ids) now live."""
        status = results["status"]
        ids = events["id"]

        def key(k):
            return int(ids[k, 0]) | (int(ids[k, 1]) << 64)

        created = status == STATUS_CREATED
        if created.any():
            ts_max = int(results["timestamp"][created].max())
            if plan.kind == "accounts":
                self.accounts_key_max = max(self.accounts_key_max, ts_max)
            else:
                self.transfers_key_max = max(self.transfers_key_max, ts_max)
        if plan.kind == "accounts":
            ks = np.nonzero(created)[0].tolist()
            self.dir.record_accounts([key(k) for k in ks], [int(plan.shard_of[k]) for k in ks])
            return
        keep = status == STATUS_CREATED
        for st in TRANSIENT_TRANSFER_STATUSES:
            keep |= status == int(st)
        timed = ((status == STATUS_CREATED) &
                 ((events["flags"] & int(TransferFlags.pending)) != 0) & (events["timeout"] > 0))
        ks, seen = [], set()
        for k in np.nonzero(keep)[0].tolist():  # (the first holder of a repeated id)
            if key(k) not in seen:
                seen.add(key(k))
                ks.append(k)
        self.dir.record_transfers([key(k) for k in ks], [int(plan.shard_of[k]) for k in ks],
                                  [bool(timed[k]) for k in ks])


def gather_results(plan: Plan, shard_results: List[Optional[np.ndarray]], n: int) -> np.ndarray:
    out = np.zeros(n, dtype=RESULT_DTYPE)
    for sl, r in zip(plan.slices, shard_results):
        if len(sl.index):
            out[sl.index] = r
    return out


def pulse_cut(counts, key_lists, pulse_batch_max: int):
    """The global pulse cut (module doc): None when fewer than pulse_batch_max entries expired
    across shards, else the pulse_batch_max-th key (expires_at, timestamp) in index order. Each
    shard reports its first pulse_batch_max keys, which hold every key up to the global cut."""
    if sum(int(c) for c in counts) < pulse_batch_max:
        return None
    keys = sorted((int(e), int(t)) for ks in key_lists for e, t in ks)
    return keys[pulse_batch_max - 1]


def pulse_plan(counts, key_lists, pulse_batch_max: int, timestamp: int):
    """One sharded pulse (module doc): (cut key, pulse_next_timestamp for tbg_pulse_cut -- the
    cut's expires_at, or 0 for each shard's own next expiry when fewer than pulse_batch_max
    expire --, per shard the timestamps of its expiries). The reference stamps expiry i of the
    pulse's E (in (expires_at, timestamp) order over all shards) timestamp - E + i + 1
    (execute_expire_pending_transfers :4540-4546); a shard's expiries are a prefix of its keys."""
    cut = pulse_cut(counts, key_lists, pulse_batch_max)
    merged = sorted((int(e), int(t), s) for s, ks in enumerate(key_lists) for e, t in ks)
    if cut is not None:
        merged = [m for m in merged if (m[0], m[1]) <= cut]
    E = len(merged)
    stamps = [[] for _ in key_lists]
    for i, (_, _, s) in enumerate(merged):
        stamps[s].append(timestamp - E + i + 1)
    if cut is None:
        cut = (merged[-1][0], merged[-1][1]) if merged else (0, 0)
        return cut, 0, stamps
    return cut, cut[0], stamps


class LocalShards:
    """All shards in one process (one executor each: several HBM table sets on one GPU, or CPU
    executors in tests). `executors[s]` provides create_accounts / create_transfers
    (events, lens, batch_ts) -> results, pulse(timestamp) -> expired, pulse_next_timestamp()."""

    def __init__(self, router: LedgerRouter, executors, pulse_batch_max: int = 8190):
        if len(executors) != router.shards:
            raise ValueError("one executor per shard")
        self.router = router
        self.executors = executors
        self.pulse_batch_max = pulse_batch_max
        for ex in executors:
            ex.set_pnt_sharded(True)

    def _run(self, kind, events, lens, batch_ts):
        dtype = ACCOUNT_DTYPE if kind == "accounts" else TRANSFER_DTYPE
        events = np.ascontiguousarray(events, dtype=dtype)
        plan = (self.router.plan_accounts if kind == "accounts"
                else self.router.plan_transfers)(events, lens, batch_ts)
        if plan.imported:
            for ex in self.executors:
                ex.raise_key_max(self.router.accounts_key_max, self.router.transfers_key_max)
        exec_events = plan.shard_events(events)
        outs = []
        for sl, ex in zip(plan.slices, self.executors):
            if not len(sl.index):
                outs.append(None)
                continue
            fn = ex.create_accounts if kind == "accounts" else ex.create_transfers
            outs.append(fn(np.ascontiguousarray(exec_events[sl.index]), sl.lens,
                           np.asarray(sl.batch_ts, dtype=np.uint64)))
        results = plan.patch(gather_results(plan, outs, len(events)))
        self.router.commit(plan, events, results)
        if plan.post_void:  # (a shard that executed nothing of the call: its value alone)
            recorded = [ex.pnt_ops() if o is not None else (int(ex.pulse_next_timestamp()), [])
                        for ex, o in zip(self.executors, outs)]
            if pnt_resets_fire([s for s, _ in recorded], [ops for _, ops in recorded]):
                for ex in self.executors:
                    ex.set_pulse_next_timestamp(TIMESTAMP_MIN)
        return results

    def create_accounts(self, events, lens, batch_ts):
        return self._run("accounts", events, lens, batch_ts)

    def create_transfers(self, events, lens, batch_ts):
        return self._run("transfers", events, lens, batch_ts)

    def pulse_next_timestamp(self) -> int:
        return min(int(ex.pulse_next_timestamp()) for ex in self.executors)

    def pulse(self, timestamp: int) -> int:
        cands = [ex.pulse_candidates(timestamp, self.pulse_batch_max) for ex in self.executors]
        cut, pnt, stamps = pulse_plan([c for c, _ in cands], [k for _, k in cands],
                                      self.pulse_batch_max, timestamp)
        return sum(int(ex.pulse_cut(timestamp, cut[0], cut[1], pnt, st))
                   for ex, st in zip(self.executors, stamps))


class ShardGroup:
    """One shard per rank of a torch.distributed group (one process per GPU). Rank 0 owns the
    router and the client call; each call is a status broadcast, one point-to-point send of
    each shard's slice (event bytes, sub-batch lengths, timestamps) and one gather of the
    16-byte results. With the `nccl` backend (RCCL over xGMI) the slices travel device to
    device; with gloo they stay on the host. `executor` is this rank's shard.
    """

    def __init__(self, executor, router: Optional[LedgerRouter] = None, group=None,
                 device: str = "cpu", pulse_batch_max: int = 8190):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.rank == 0 and (router is None or router.shards != self.world):
            raise ValueError("rank 0 needs a router with one shard per rank")
        self.router = router
        self.executor = executor
        self.device = device
        self.pulse_batch_max = pulse_batch_max
        executor.set_pnt_sharded(True)

    def _peer(self, r: int) -> int:
        return r if self.group is None else self.dist.get_global_rank(self.group, r)

    def _send(self, a: np.ndarray, dst: int):
        import torch
        a = np.ascontiguousarray(a)
        hdr = torch.tensor([a.nbytes], dtype=torch.int64, device=self.device)
        self.dist.send(hdr, self._peer(dst), group=self.group)
        if a.nbytes:
            buf = torch.from_numpy(a.view(np.uint8).reshape(-1).copy()).to(self.device)
            self.dist.send(buf, self._peer(dst), group=self.group)

    def _recv(self, src: int, dtype) -> np.ndarray:
        import torch
        hdr = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.dist.recv(hdr, self._peer(src), group=self.group)
        nb = int(hdr.item())
        if nb == 0:
            return np.zeros(0, dtype=dtype)
        buf = torch.empty(nb, dtype=torch.uint8, device=self.device)
        self.dist.recv(buf, self._peer(src), group=self.group)
        return buf.cpu().numpy().view(dtype)

    def _bcast(self, value: int) -> int:
        import torch
        t = torch.tensor([value], dtype=torch.int64, device=self.device)
        self.dist.broadcast(t, self._peer(0), group=self.group)
        return int(t.item())

    def _run(self, kind, events=None, lens=None, batch_ts=None):
        dtype = ACCOUNT_DTYPE if kind == "accounts" else TRANSFER_DTYPE
        plan, err = None, None
        if self.rank == 0:
            events = np.ascontiguousarray(events, dtype=dtype)
            try:
                plan = (self.router.plan_accounts if kind == "accounts"
                        else self.router.plan_transfers)(events, lens, batch_ts)
            except RouteError as e:
                err = e
        # Status word: refused, the global key maxima an imported call needs on every shard, and
        # whether the call posts or voids (pulse_next_timestamp resolved across shards after it).
        word = self._bcast_words([0 if err is None else 1,
                                  int(plan is not None and plan.imported),
                                  self.router.accounts_key_max if self.rank == 0 else 0,
                                  self.router.transfers_key_max if self.rank == 0 else 0,
                                  int(plan is not None and plan.post_void)])
        if word[0]:  # every rank fails a refused call
            raise err if err is not None else RouteError("refused by the router on rank 0")
        if word[1]:
            self.executor.raise_key_max(word[2], word[3])
        if self.rank == 0:
            exec_events = plan.shard_events(events)
            for s in range(1, self.world):
                sl = plan.slices[s]
                self._send(exec_events[sl.index], s)
                self._send(np.asarray(sl.lens, dtype=np.uint32), s)
                self._send(np.asarray(sl.batch_ts, dtype=np.uint64), s)
            sl = plan.slices[0]
            mine = (exec_events[sl.index], sl.lens, np.asarray(sl.batch_ts, dtype=np.uint64))
        else:
            ev = self._recv(0, dtype)
            ln = self._recv(0, np.uint32)
            ts = self._recv(0, np.uint64)
            mine = (ev, ln.tolist(), ts)
        res = np.zeros(0, dtype=RESULT_DTYPE)
        failure = None
        if len(mine[0]):
            fn = (self.executor.create_accounts if kind == "accounts"
                  else self.executor.create_transfers)
            try:
                res = fn(np.ascontiguousarray(mine[0]), mine[1], mine[2])
            except Exception as e:  # noqa: BLE001 -- every rank must learn of it (below)
                failure = e
                res = np.zeros(0, dtype=RESULT_DTYPE)
        # Every rank reports a status word with its results, and every rank learns whether any
        # shard failed: a rank whose executor raised (capacity, watchdog) still answers, so no
        # rank blocks in a receive. After such a failure the shards' state is undefined.
        if self.rank != 0:
            self._send(np.asarray([0 if failure is None else 1], dtype=np.int64), 0)
            self._send(res, 0)
        else:
            statuses = [0 if failure is None else 1]
            outs = [res]
            for s in range(1, self.world):
                statuses.append(int(self._recv(s, np.int64)[0]))
                outs.append(self._recv(s, RESULT_DTYPE))
        failed = self._bcast(max(statuses) if self.rank == 0 else 0)
        if failed:
            if failure is not None:
                raise failure
            raise RuntimeError("a shard's executor failed; the shards' state is undefined")
        if word[4]:
            self.resolve_pnt(executed=len(mine[0]) > 0)
        if self.rank != 0:
            return None
        results = plan.patch(gather_results(plan, outs, len(events)))
        self.router.commit(plan, events, results)
        return results

    def resolve_pnt(self, executed=True):
        """Collective, after a call that posts or voids: every shard's recorded
        pulse_next_timestamp updates to rank 0 (its start value, then (timestamp, op) pairs; a
        shard that executed nothing of the call sends its value alone), replayed in call order
        there; the outcome broadcast."""
        if executed:
            start, ops = self.executor.pnt_ops()
        else:
            start, ops = int(self.executor.pulse_next_timestamp()), []
        mine = np.asarray([start] + [x for pair in ops for x in pair], dtype=np.uint64)
        if self.rank != 0:
            self._send(mine, 0)
            fired = self._bcast(0)
        else:
            starts, lists = [start], [ops]
            for s in range(1, self.world):
                a = self._recv(s, np.uint64)
                starts.append(int(a[0]))
                lists.append(list(zip(a[1::2].tolist(), a[2::2].tolist())))
            fired = self._bcast(int(pnt_resets_fire(starts, lists)))
        if fired:
            self.executor.set_pulse_next_timestamp(TIMESTAMP_MIN)

    def _bcast_words(self, words):
        import torch
        t = torch.tensor(words, dtype=torch.int64, device=self.device)
        self.dist.broadcast(t, self._peer(0), group=self.group)
        return [int(x) for x in t.tolist()]

    def create_accounts(self, events=None, lens=None, batch_ts=None):
        """Collective: rank 0 passes the call, the other ranks call with no arguments."""
        return self._run("accounts", events, lens, batch_ts)

    def create_transfers(self, events=None, lens=None, batch_ts=None):
        return self._run("transfers", events, lens, batch_ts)

    def pulse_next_timestamp(self) -> int:
        """Collective all-reduce(min) of the shards' pulse_next_timestamp."""
        import torch
        t = torch.tensor([int(self.executor.pulse_next_timestamp())], dtype=torch.int64,
                         device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
        return int(t.item())

    def pulse(self, timestamp: int) -> int:
        """Collective: every shard expires at the common pulse timestamp, up to the global cut
        (an all-gather of each shard's first pulse_batch_max expiry keys)."""
        import torch
        B = self.pulse_batch_max
        count, keys = self.executor.pulse_candidates(timestamp, B)
        mine = torch.full((B + 1, 2), (1 << 63) - 1, dtype=torch.int64)
        mine[0, 0] = int(count)
        if keys:
            mine[1:1 + len(keys)] = torch.tensor(keys, dtype=torch.int64)
        mine = mine.to(self.device)
        parts = [torch.empty_like(mine) for _ in range(self.world)]
        self.dist.all_gather(parts, mine, group=self.group)
        parts = [p.cpu() for p in parts]
        counts = [int(p[0, 0]) for p in parts]
        key_lists = [[(int(e), int(t)) for e, t in p[1:1 + min(c, B)].tolist()]
                     for p, c in zip(parts, counts)]
        cut, pnt, stamps = pulse_plan(counts, key_lists, B, timestamp)
        local = int(self.executor.pulse_cut(timestamp, cut[0], cut[1], pnt, stamps[self.rank]))
        t = torch.tensor([local], dtype=torch.int64, device=self.device)
        self.dist.all_reduce(t, group=self.group)
        return int(t.item())


class GpuShard:
    """A shard backed by libtbg.so (its HBM tables on `device`): the executor interface above."""

    def __init__(self, account_capacity, transfer_capacity, batch_events_max=1 << 16,
                 batch_count_max=4096, pulse_batch_max=8190, device=0,
                 pulse_next_timestamp_init=(1 << 63) - 1, account_events_capacity=0):
        import ctypes
        from . import native
        self._c = ctypes
        self._native = native
        self.lib = native.load()
        o = native.TbgOptions()
        o.account_capacity = account_capacity
        o.transfer_capacity = transfer_capacity
        o.batch_events_max = batch_events_max
        o.batch_count_max = batch_count_max
        o.pulse_batch_max = pulse_batch_max
        o.device = device
        o.pulse_next_timestamp_init = pulse_next_timestamp_init
        o.account_events_capacity = account_events_capacity
        self.g = self.lib.tbg_open(ctypes.byref(o))
        if not self.g:
            raise RuntimeError("tbg_open failed")

    @classmethod
    def wrap(cls, lib, g):
        """A shard over an executor the caller owns (closing it is the caller's)."""
        import ctypes
        from . import native
        self = cls.__new__(cls)
        self._c, self._native, self.lib, self.g, self._owned = ctypes, native, lib, g, False
        return self

    def close(self):
        if self.g and getattr(self, "_owned", True):
            self.lib.tbg_close(self.g)
        self.g = None

    def _call(self, fn, events, lens, batch_ts):
        c = self._c
        n = len(events)
        lens_a = np.asarray(lens, dtype=np.uint32)
        ts_a = np.asarray(batch_ts, dtype=np.uint64)
        out = np.zeros(n, dtype=RESULT_DTYPE)
        rc = fn(self.g, events.ctypes.data_as(c.c_void_p), n,
                lens_a.ctypes.data_as(self._native.c_u32p),
                ts_a.ctypes.data_as(self._native.c_u64p), len(lens_a),
                out.ctypes.data_as(c.c_void_p))
        if rc != 0:
            raise RuntimeError(f"libtbg: {rc} {self.lib.tbg_last_error(self.g)}")
        return out

    def create_accounts(self, events, lens, batch_ts):
        return self._call(self.lib.tbg_create_accounts,
                          np.ascontiguousarray(events, dtype=ACCOUNT_DTYPE), lens, batch_ts)

    def create_transfers(self, events, lens, batch_ts):
        return self._call(self.lib.tbg_create_transfers,
                          np.ascontiguousarray(events, dtype=TRANSFER_DTYPE), lens, batch_ts)

    def pulse(self, timestamp):
        return int(self.lib.tbg_pulse(self.g, timestamp))

    def pulse_candidates(self, timestamp, max_keys):
        c = self._c
        e = np.zeros(max(max_keys, 1), dtype=np.uint64)
        t = np.zeros(max(max_keys, 1), dtype=np.uint64)
        n = int(self.lib.tbg_pulse_candidates(self.g, timestamp, e.ctypes.data_as(c.c_void_p),
                                              t.ctypes.data_as(c.c_void_p), max_keys))
        if n < 0:
            raise RuntimeError(f"libtbg: {n} {self.lib.tbg_last_error(self.g)}")
        k = min(n, max_keys)
        return n, list(zip(e[:k].tolist(), t[:k].tolist()))

    def pulse_cut(self, timestamp, cut_expires_at, cut_timestamp, pulse_next_timestamp,
                  stamps=None):
        st = None if stamps is None else np.ascontiguousarray(stamps, dtype=np.uint64)
        n = int(self.lib.tbg_pulse_cut(self.g, timestamp, cut_expires_at, cut_timestamp,
                                       pulse_next_timestamp,
                                       None if st is None or len(st) == 0
                                       else st.ctypes.data_as(self._c.c_void_p)))
        if n < 0:
            raise RuntimeError(f"libtbg: {n} {self.lib.tbg_last_error(self.g)}")
        return n

    def pulse_next_timestamp(self):
        return int(self.lib.tbg_pulse_next_timestamp(self.g))

    def set_pnt_sharded(self, on):
        self.lib.tbg_set_pnt_sharded(self.g, 1 if on else 0)

    def pnt_ops(self):
        """The last call's recorded pulse_next_timestamp updates: (start, [(timestamp, op)])."""
        c = self._c
        start = c.c_uint64()
        n = int(self.lib.tbg_pnt_ops(self.g, None, None, 0, c.byref(start)))
        if n < 0:
            raise RuntimeError(f"libtbg: {n} {self.lib.tbg_last_error(self.g)}")
        ts = np.zeros(max(n, 1), dtype=np.uint64)
        ops = np.zeros(max(n, 1), dtype=np.uint64)
        if n:
            self.lib.tbg_pnt_ops(self.g, ts.ctypes.data_as(c.c_void_p),
                                 ops.ctypes.data_as(c.c_void_p), n, c.byref(start))
        return int(start.value), list(zip(ts[:n].tolist(), ops[:n].tolist()))

    def set_pulse_next_timestamp(self, value):
        rc = self.lib.tbg_set_pulse_next_timestamp(self.g, int(value))
        if rc != 0:
            raise RuntimeError(f"libtbg: {rc} {self.lib.tbg_last_error(self.g)}")

    def raise_key_max(self, accounts_key_max, transfers_key_max):
        rc = self.lib.tbg_raise_key_max(self.g, accounts_key_max, transfers_key_max)
        if rc != 0:
            raise RuntimeError(f"libtbg: {rc} {self.lib.tbg_last_error(self.g)}")

    def dump(self):
        c = self._c
        na = self.lib.tbg_dump_accounts(self.g, None)
        a = np.zeros(max(na, 0), dtype=ACCOUNT_DTYPE)
        self.lib.tbg_dump_accounts(self.g, a.ctypes.data_as(c.c_void_p))
        nt = self.lib.tbg_dump_transfers(self.g, None, None)
        t = np.zeros(max(nt, 0), dtype=TRANSFER_DTYPE)
        s = np.zeros(max(nt, 0), dtype=np.uint8)
        self.lib.tbg_dump_transfers(self.g, t.ctypes.data_as(c.c_void_p),
                                    s.ctypes.data_as(c.c_void_p))
        return a, t, s

    def dump_account_events(self):
        """This shard's AccountEvents in timestamp order (tbg_dump_account_events)."""
        from .types import ACCOUNT_EVENT_DTYPE
        n = self.lib.tbg_dump_account_events(self.g, None)
        e = np.zeros(max(n, 0), dtype=ACCOUNT_EVENT_DTYPE)
        if n > 0:
            self.lib.tbg_dump_account_events(self.g, e.ctypes.data_as(self._c.c_void_p))
        return e
