"""Ledger sharding of the commit path across GPUs.

Debit and credit accounts of a transfer must share the transfer's ledger
(`accounts_must_have_the_same_ledger`, `transfer_must_have_the_same_ledger_as_accounts`,
src/state_machine.zig:3795-3798), so ledgers are independent shards: one executor per GPU owns a
contiguous range of ledgers -- their accounts, transfer ids, transfer rows and TransferPending
statuses. A client call (a multi-batch commit) is executed by `Engine` on the call's owner (rank
0), which sends each shard its part, and every result comes back in call order -- identical to
the reference executing the whole call serially, for every call.

Placement. `LedgerRouter` keeps directories of where each account id and each transfer id
(created, or orphaned by a transient failure) lives, and places every event:

* an event whose id already exists goes to the id's holder: `create_transfer_exists` /
  `id_already_failed` / `create_account_exists` are decided before any account lookup (:3629,
  :3733-3738);
* a post/void goes to its pending transfer's shard (found in the directory or earlier in the
  call; a pending transfer found nowhere fails `pending_transfer_not_found` on any shard);
* a transfer goes to its accounts' shard, an account to its ledger's shard;
* a transfer whose two accounts live on different shards fails
  `accounts_must_have_the_same_ledger` unless an earlier static check fails first (:3748-3798),
  and never reads a balance: the router computes that status and the shard runs a *surrogate*
  (credit account := debit account), which fails at the same position with
  `accounts_must_be_different`, non-transient like the true status; the router writes the true
  status into the result;
* an event whose status follows from its batch alone (execute_create :3050-3064: the imported
  flag against the batch's first event) runs as an *inert* event that fails without effects
  (id 0 or an imported timestamp 0) and gets the router's status.

Segments. A call is executed as a sequence of *segments* -- maximal runs of whole linked chains
whose events cannot observe another shard's state -- each executed by every shard on its part,
the directories then updated from the results, the next segment placed with them. A segment ends
before a chain that

* repeats an id of an earlier chain of the segment and would otherwise run on another shard: its
  outcome depends on the first occurrence's (created or orphaned: decided by the holder; failed
  otherwise: executed where its accounts are) -- known once the segment has run;
* holds an imported event whose timestamp is at or below a timestamp an earlier event of the
  segment on another shard may create (`must_not_regress` reads the objects tree's key range
  over all shards, :3656-3660, :3808-3812); each segment with imported events starts with every
  shard's key maxima raised to the maxima over all shards (`sync_key_max`);
* spans shards -- a linked chain whose events live on different shards: it becomes a segment of
  its own, executed by the chain protocol below.

A linked chain across shards is atomic across them (:3033-3207). Every shard holding a part of
it *probes* the part: its events as one stamped batch (global timestamps), all linked, followed
by an inert sentinel that fails, so the part always rolls back and reports the first event that
failed on the shard. The chain's first failure is the minimum over shards (a shard's events see
only its own state, so events before the first failure execute exactly as in the reference).
No failure: every shard executes its part again as a chain, which now succeeds. A failure: the
statuses are the reference's (`linked_event_failed` before and after it), an orphan a probe left
for an event the reference never reaches is forgotten (`forget_orphans`; the failing event's own
orphan, :3172, stays), and each shard's pulse_next_timestamp is set back to its value before the
probe lowered by the pending transfers the reference did execute (it is not scoped: :3975-3982
are not undone by a discard).

Imported events read the *other* groove by timestamp (`indirect_lookup`, :3661-3665,
:3813-3817) -- asked of every shard before the call (`timestamps_exist`). An imported event
whose timestamp belongs to another shard's object, or (in a chain across shards) lies at or
below an imported timestamp the chain created earlier on another shard, fails
`imported_event_timestamp_must_not_regress` if it reaches those checks: a transfer runs with its
timestamp replaced by one that collides on its own shard (its debit account's), an account gets
the status the router computes from its static checks (:3623-3646).

Timestamps are global: event k of batch b is stamped `batch_ts[b] - len[b] + k + 1`
(`execute_multi_batch`, :2702-2762). A shard receives a non-imported batch's events as maximal
runs of consecutive positions, each run a sub-batch whose timestamp is that of its last event;
an imported batch's events as one stamped batch whose timestamp is the batch's (imported events'
`must_not_advance` bound, :3073).

pulse_next_timestamp. A post/void of a pending transfer that has a timeout resets it when it
equals the pending transfer's expiry (:4227-4229) -- a comparison against the *global* value at
that point of the call, which no shard holds. The shards run with sharded pulse_next_timestamp
(`set_pnt_sharded`): each records every update at its event (min of a pending transfer's expiry,
applied; reset-if-equal of a post/void, only recorded) with the event's global timestamp. After a
segment holding a post/void the updates of every shard are merged by timestamp and replayed from
the minimum of the shards' values at the segment's start (`pnt_resets_fire`); when a reset fires,
every shard's value becomes timestamp_min -- the reference's value. No event's outcome reads the
value (only pulses do, between calls).

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
from typing import Dict, List, Optional, Tuple

import numpy as np

from .types import (ACCOUNT_DTYPE, RESULT_DTYPE, STATUS_CREATED, TIMESTAMP_MAX, TRANSFER_DTYPE,
                    TRANSIENT_TRANSFER_STATUSES, AccountFlags, CreateAccountStatus,
                    CreateTransferStatus, TransferFlags)

_U128_MAX = (1 << 128) - 1
_CT = CreateTransferStatus
_CA = CreateAccountStatus
LINKED_EVENT_FAILED = 1   # (the same value for accounts and transfers)
LINKED_EVENT_CHAIN_OPEN = 2
_TRANSIENT = frozenset(int(s) for s in TRANSIENT_TRANSFER_STATUSES)

PNT_RESET = 1 << 63  # a recorded update that is a reset-if-equal (post/void of an expiry)
TIMESTAMP_MIN = 1


def pnt_resets_fire(starts, op_lists) -> bool:
    """Does a reset of pulse_next_timestamp fire in the call's order across shards? `starts`: the
    shards' values at the segment's start; `op_lists`: per shard, its recorded updates as (event
    timestamp, op) -- op an expiry (a `min`), or an expiry | PNT_RESET (reset-if-equal)."""
    value = min(int(x) for x in starts)
    for _, op in sorted((int(t), int(o)) for ops in op_lists for t, o in ops):
        if op & PNT_RESET:
            if value == op & ~PNT_RESET:
                return True  # (timestamp_min from here on: every later `min` keeps it)
        elif op < value:
            value = op
    return False


def _ids(col: np.ndarray) -> List[int]:
    lo = col[:, 0].tolist()
    hi = col[:, 1].tolist()
    return [a | (b << 64) for a, b in zip(lo, hi)]


def _u128_array(ids: List[int]) -> np.ndarray:
    a = np.zeros((len(ids), 2), dtype=np.uint64)
    if ids:
        a[:, 0] = [i & 0xFFFFFFFFFFFFFFFF for i in ids]
        a[:, 1] = [i >> 64 for i in ids]
    return a


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


@dataclass(frozen=True)
class _Kind:
    name: str
    dtype: np.dtype
    imported_flag: int
    inert_plain: int      # an inert event's status in a non-imported batch (id_must_not_be_zero)
    inert_imported: int   # ... in an imported batch (imported_event_timestamp_out_of_range)
    expected: int         # imported_event_expected
    not_expected: int     # imported_event_not_expected
    regress: int          # imported_event_timestamp_must_not_regress


ACCOUNTS = _Kind("accounts", ACCOUNT_DTYPE, int(AccountFlags.imported),
                 int(_CA.id_must_not_be_zero), int(_CA.imported_event_timestamp_out_of_range),
                 int(_CA.imported_event_expected), int(_CA.imported_event_not_expected),
                 int(_CA.imported_event_timestamp_must_not_regress))
TRANSFERS = _Kind("transfers", TRANSFER_DTYPE, int(TransferFlags.imported),
                  int(_CT.id_must_not_be_zero), int(_CT.imported_event_timestamp_out_of_range),
                  int(_CT.imported_event_expected), int(_CT.imported_event_not_expected),
                  int(_CT.imported_event_timestamp_must_not_regress))
_POST_VOID = int(TransferFlags.post_pending_transfer | TransferFlags.void_pending_transfer)
_PENDING = int(TransferFlags.pending)
_CLOSING = int(TransferFlags.closing_debit | TransferFlags.closing_credit)


def cross_status(pending_id: int, flags: int, timeout: int, ledger: int, code: int) -> int:
    """create_transfer's status (:3748-3798) for a transfer whose two accounts exist on different
    shards (so on different ledgers), from the checks after `accounts_must_be_different`."""
    if pending_id != 0:
        return int(_CT.pending_id_must_be_zero)
    if not flags & _PENDING:
        if timeout != 0:
            return int(_CT.timeout_reserved_for_pending_transfer)
        if flags & _CLOSING:
            return int(_CT.closing_transfer_must_be_pending)
    if ledger == 0:
        return int(_CT.ledger_must_not_be_zero)
    if code == 0:
        return int(_CT.code_must_not_be_zero)
    return int(_CT.accounts_must_have_the_same_ledger)


def account_static_status(a) -> Optional[int]:
    """create_account's checks that read no state (:3623-3646), except the id lookup: the first
    failing one, or None. (`a`: one ACCOUNT_DTYPE record.)"""
    if int(a["reserved"]) != 0:
        return int(_CA.reserved_field)
    f = int(a["flags"])
    if f & 0xFFC0:
        return int(_CA.reserved_flag)
    i = int(a["id"][0]) | (int(a["id"][1]) << 64)
    if i == 0:
        return int(_CA.id_must_not_be_zero)
    if i == _U128_MAX:
        return int(_CA.id_must_not_be_int_max)
    if (f & int(AccountFlags.debits_must_not_exceed_credits)) and \
            (f & int(AccountFlags.credits_must_not_exceed_debits)):
        return int(_CA.flags_are_mutually_exclusive)
    for name, st in (("debits_pending", _CA.debits_pending_must_be_zero),
                     ("debits_posted", _CA.debits_posted_must_be_zero),
                     ("credits_pending", _CA.credits_pending_must_be_zero),
                     ("credits_posted", _CA.credits_posted_must_be_zero)):
        if int(a[name][0]) or int(a[name][1]):
            return int(st)
    if int(a["ledger"]) == 0:
        return int(_CA.ledger_must_not_be_zero)
    if int(a["code"]) == 0:
        return int(_CA.code_must_not_be_zero)
    return None


def inert_event(kind: _Kind, imported_batch: bool, linked: bool) -> np.ndarray:
    """An event that fails in execute_create / create_* before reading any state, in a batch whose
    first event's imported flag is `imported_batch`: id 0 (id_must_not_be_zero), or in an imported
    batch an imported timestamp 0 (imported_event_timestamp_out_of_range)."""
    e = np.zeros(1, dtype=kind.dtype)
    f = (kind.imported_flag if imported_batch else 0) | (1 if linked else 0)
    e["flags"] = f
    return e[0]


# ---- directories ----------------------------------------------------------------------------

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
    """Placement by ledger and the directories (module doc).

    Ledgers 1..`ledgers` map to shards by contiguous ranges (64 ledgers / G);
    other ledgers by `ledger % shards`. Placement of a new account follows its ledger; routing
    of later events follows the directories, so a placement never has to be recomputed.
    """

    def __init__(self, shards: int, ledgers: int = 64, directory=None):
        if shards < 1 or shards > 127:
            raise ValueError("shards must be in 1..127")
        self.shards = shards
        self.ledgers = ledgers
        self.dir = directory if directory is not None else DictDirectory()

    def shard_of_ledger(self, ledger: int) -> int:
        if 1 <= ledger <= self.ledgers:
            return (ledger - 1) * self.shards // self.ledgers
        return ledger % self.shards

    def record(self, kind: _Kind, ids: List[int], shard_of: List[int], status: List[int],
               timed: List[bool]):
        """Records where a segment's new objects (and orphaned transfer ids) now live; returns the
        (id, shard, timed) entries recorded. A repeated id keeps its first holder."""
        out, seen = [], set()
        for i, sh, st, tm in zip(ids, shard_of, status, timed):
            keep = st == STATUS_CREATED or (kind is TRANSFERS and st in _TRANSIENT)
            if keep and i not in seen:
                seen.add(i)
                out.append((i, sh, bool(tm and st == STATUS_CREATED)))
        if kind is ACCOUNTS:
            self.dir.record_accounts([e[0] for e in out], [e[1] for e in out])
        else:
            self.dir.record_transfers([e[0] for e in out], [e[1] for e in out],
                                      [e[2] for e in out])
        return out


# ---- planning -------------------------------------------------------------------------------

class _Call:
    """A call's events with everything placement reads, computed once."""

    def __init__(self, kind: _Kind, events: np.ndarray, lens, batch_ts):
        self.kind = kind
        self.is_tr = kind is TRANSFERS
        self.events = events
        n = self.n = len(events)
        lens_a = np.asarray(lens, dtype=np.int64)
        if int(lens_a.sum()) != n:
            raise ValueError("batch lengths do not cover the events")
        bts = np.asarray(batch_ts, dtype=np.uint64).astype(np.int64)
        ends = np.cumsum(lens_a)
        starts = ends - lens_a
        b_of = np.repeat(np.arange(len(lens_a)), lens_a)
        within = np.arange(n, dtype=np.int64) - starts[b_of]
        self.b_of = b_of.tolist()
        self.batch_start = starts.tolist()
        self.batch_end = ends.tolist()
        self.batch_ts = bts.tolist()
        self.stamp = (bts[b_of] - lens_a[b_of] + within + 1).tolist()
        flags = events["flags"].astype(np.int64)
        self.flags = flags.tolist()
        linked = (flags & 1) != 0
        last = within == lens_a[b_of] - 1
        self.open_last = (linked & last).tolist()
        imp = (flags & kind.imported_flag) != 0
        g_batch = np.zeros(len(lens_a), dtype=bool)
        ne = lens_a > 0
        g_batch[ne] = imp[starts[ne]]
        self.g_batch = g_batch.tolist()
        G = g_batch[b_of] if n else np.zeros(0, dtype=bool)
        self.G = G.tolist()
        ts = events["timestamp"].tolist()
        self.ts = ts
        T = bts[b_of].tolist() if n else []
        # execute_create's batch-context statuses (:3050-3064), where no chain_open precedes them
        self.pre: Dict[int, int] = {}
        for k in np.nonzero((imp != G) & ~(linked & last))[0].tolist():
            self.pre[k] = kind.not_expected if imp[k] else kind.expected
        # imported events that reach create_* (valid timestamp, not advancing past the batch)
        self.imp_live = [bool(imp[k] and G[k] and 1 <= ts[k] <= TIMESTAMP_MAX and ts[k] < T[k])
                         for k in range(n)]
        self.ids = _ids(events["id"])
        if self.is_tr:
            self.drs = _ids(events["debit_account_id"])
            self.crs = _ids(events["credit_account_id"])
            self.pids = _ids(events["pending_id"])
            self.timeouts = events["timeout"].tolist()
            self.codes = events["code"].tolist()
        self.ledgers = events["ledger"].tolist()
        cs = np.nonzero(chain_starts(events["flags"], lens))[0].tolist() if n else []
        self.chain_end: Dict[int, int] = dict(zip(cs, cs[1:] + [n]))
        # potential creation timestamp of each event (imported-regress cuts): an imported event's
        # own, a non-imported one's commit timestamp; -1 for events that cannot create
        self.potential = [(ts[k] if self.imp_live[k] else (-1 if imp[k] else self.stamp[k]))
                          for k in range(n)]


@dataclass
class _Known:
    """The directories' answers for the ids a call references, kept current as segments commit."""
    accounts: Dict[int, int] = field(default_factory=dict)
    transfers: Dict[int, tuple] = field(default_factory=dict)


@dataclass
class _Seg:
    start: int
    end: int = 0
    chain: bool = False                       # one linked chain across shards
    shard_of: Dict[int, int] = field(default_factory=dict)
    cross: Dict[int, int] = field(default_factory=dict)     # k -> the reference's status
    decided: Dict[int, int] = field(default_factory=dict)   # k -> status (inert event)
    tprime: Dict[int, int] = field(default_factory=dict)    # k -> shard (timestamp surrogate)
    imported: bool = False
    post_void: bool = False


_CUT = object()


class Planner:
    """Places a call's events segment by segment (module doc)."""

    def __init__(self, router: LedgerRouter, call: _Call, known: _Known,
                 collisions: Dict[int, set]):
        self.r = router
        self.c = call
        self.known = known
        self.coll = collisions  # imported timestamp -> shards holding an object of the other groove

    def _natural_transfer(self, k, chain_first, seg_ids):
        """Where event k runs by what it names (not its own id): a shard, None (anywhere), or
        "cross" (two accounts on two shards)."""
        c, kn = self.c, self.known
        if c.flags[k] & _POST_VOID:
            p = c.pids[k]
            if p in kn.transfers:
                return kn.transfers[p][0]
            if p in chain_first:
                return chain_first[p]
            if p in seg_ids:
                return seg_ids[p]
            return None
        a_dr, a_cr = kn.accounts.get(c.drs[k]), kn.accounts.get(c.crs[k])
        if a_dr is not None and a_cr is not None and a_dr != a_cr:
            return "cross"
        return a_dr if a_dr is not None else a_cr

    def _place_chain(self, a: int, z: int, seg_ids: Dict[int, int]):
        c, kn = self.c, self.known
        pin: Dict[int, Optional[int]] = {}
        cross: Dict[int, int] = {}
        chain_first: Dict[int, int] = {}
        holders = kn.transfers if c.is_tr else kn.accounts
        for k in range(a, z):
            if k in c.pre:
                pin[k] = None
                continue
            i = c.ids[k]
            if i in holders:
                s = holders[i][0] if c.is_tr else holders[i]
            elif i in chain_first:  # the chain reaches it only if the first occurrence created it
                s = chain_first[i]
            else:
                nat = (self._natural_transfer(k, chain_first, seg_ids) if c.is_tr
                       else self.r.shard_of_ledger(c.ledgers[k]))
                if i in seg_ids:
                    if nat is None or nat == seg_ids[i]:
                        s = seg_ids[i]
                    else:
                        return _CUT
                elif nat == "cross":
                    cross[k] = cross_status(c.pids[k], c.flags[k], c.timeouts[k],
                                            c.ledgers[k], c.codes[k])
                    s = None
                else:
                    s = nat
            pin[k] = s
            if s is not None and i != 0 and i != _U128_MAX and i not in holders:
                chain_first.setdefault(i, s)
        shards = sorted({s for s in pin.values() if s is not None})
        if not shards:
            shards = [self.r.shard_of_ledger(c.ledgers[a])]
        # unpinned events (inert, surrogates, found nowhere) run with their neighbours
        last = shards[0]
        place = {}
        for k in range(a, z):
            if pin[k] is None:
                place[k] = last
            else:
                place[k] = last = pin[k]
        return place, cross, shards

    def _imported_decisions(self, a, z, place, multi, seg_ids, seg):
        """Imported events whose must_not_regress checks read another shard (module doc): a
        transfer runs with a timestamp surrogate, an account gets the router's status. Returns
        False when the chain must start a new segment instead."""
        c = self.c
        chain_max: Dict[int, int] = {}  # shard -> largest imported timestamp created so far
        holders = self.known.transfers if c.is_tr else self.known.accounts
        seen_ids = set()
        for k in range(a, z):
            if k in c.pre or not c.imp_live[k] or k in seg.cross:
                continue
            s, t = place[k], c.ts[k]
            hazard = bool(self.coll.get(t)) and s not in self.coll[t]
            if multi and any(osh != s and ot >= t for osh, ot in chain_max.items()):
                hazard = True
            if hazard:
                i = c.ids[k]
                if c.is_tr:
                    seg.tprime[k] = s
                elif i in holders or i in seen_ids:
                    pass  # create_account_exists decides it first (:3629), on the holder
                elif i in seg_ids:
                    return False  # (whether it exists is known once the segment has run)
                else:
                    st = account_static_status(c.events[k])
                    seg.decided[k] = c.kind.regress if st is None else st
            chain_max[s] = max(chain_max.get(s, 0), c.ts[k])
            seen_ids.add(c.ids[k])
        return True

    def plan(self, start: int) -> _Seg:
        c = self.c
        seg = _Seg(start)
        seg_ids: Dict[int, int] = {}
        seg_pot = [-1] * self.r.shards
        a = start
        while a < c.n:
            z = c.chain_end[a]
            placed = self._place_chain(a, z, seg_ids)
            if placed is _CUT:
                break
            place, cross, shards = placed
            multi = len(shards) > 1
            if multi and a > start:
                break
            trial = _Seg(start)
            trial.cross = cross
            if not self._imported_decisions(a, z, place, multi, seg_ids, trial):
                break
            if a > start:  # regress across shards within the segment
                cut = False
                for k in range(a, z):
                    if c.imp_live[k] and k not in c.pre and k not in trial.decided:
                        s = place[k]
                        if any(seg_pot[o] >= c.ts[k] for o in range(self.r.shards) if o != s):
                            cut = True
                            break
                if cut:
                    break
            seg.shard_of.update(place)
            seg.cross.update(trial.cross)
            seg.decided.update(trial.decided)
            seg.tprime.update(trial.tprime)
            for k in range(a, z):
                if k in c.pre or k in cross or k in trial.decided or k in trial.tprime:
                    continue
                i = c.ids[k]
                if i != 0 and i != _U128_MAX:
                    seg_ids.setdefault(i, place[k])
                s = place[k]
                seg_pot[s] = max(seg_pot[s], c.potential[k])
                if c.imp_live[k]:
                    seg.imported = True
                if c.is_tr and c.flags[k] & _POST_VOID:
                    seg.post_void = True
            a = z
            if multi:
                seg.chain = True
                break
        seg.end = a
        if seg.end == start:
            raise AssertionError("empty segment")  # (the first chain always fits)
        return seg


# ---- execution --------------------------------------------------------------------------------

ONE_CHAIN = 1  # tbg.h TBG_ONE_CHAIN


@dataclass
class SubCall:
    """One executor call of a shard: "batches" (events, lens, batch_ts) or "stamped" (events,
    per-event timestamps, the batch's timestamp; `one_chain`: the batch is one linked chain closed
    at its last event, whatever the events' linked flags -- a part of a chain across shards)."""
    mode: str
    events: np.ndarray
    aux: np.ndarray          # lens (u32) or stamps (u64)
    batch_ts: np.ndarray     # batch timestamps (u64) | one element: the stamped batch's
    one_chain: bool = False


def run_subcalls(ex, kind: _Kind, subcalls: List[SubCall]):
    """Executes a shard's sub-calls in order on executor `ex`: (results per sub-call, and for
    transfers the pulse_next_timestamp updates recorded over them as (start, [(ts, op)]))."""
    outs = []
    start, ops = None, []
    for sc in subcalls:
        ev = np.ascontiguousarray(sc.events, dtype=kind.dtype)
        if sc.mode == "batches":
            fn = ex.create_accounts if kind is ACCOUNTS else ex.create_transfers
            outs.append(fn(ev, [int(x) for x in sc.aux], np.asarray(sc.batch_ts, np.uint64)))
        else:
            fn = ex.create_accounts_stamped if kind is ACCOUNTS else ex.create_transfers_stamped
            outs.append(fn(ev, np.asarray(sc.aux, np.uint64), int(sc.batch_ts[0]),
                           ONE_CHAIN if sc.one_chain else 0))
        if kind is TRANSFERS:
            s, o = ex.pnt_ops()
            if start is None:
                start = s
            ops.extend(o)
    pnt = None
    if kind is TRANSFERS:
        pnt = (int(ex.pulse_next_timestamp()) if start is None else start, ops)
    return outs, pnt


class Engine:
    """Executes a call across shards exactly (module doc). `ops` is the shard group: LocalShards
    (all shards in this process) or ShardGroup (one per rank, run from rank 0)."""

    def __init__(self, router: LedgerRouter, ops, max_batches: int = 4096):
        self.router = router
        self.ops = ops
        # Batches per "batches" sub-call (the executors' batch_count_max): a shard's runs of a
        # call whose ledgers interleave event by event are many short batches.
        self.max_batches = max_batches
        self.segments = 0       # statistics: segments executed, of them chains across shards
        self.chain_segments = 0

    # -- setup ----------------------------------------------------------------------------------

    def _known(self, c: _Call) -> _Known:
        kn = _Known()
        d = self.router.dir
        if c.is_tr:
            uniq_t = list(set(c.ids) | set(c.pids))
            kn.transfers = {i: v for i, v in zip(uniq_t, d.transfer_info(uniq_t)) if v is not None}
            uniq_a = list(set(c.drs) | set(c.crs))
        else:
            uniq_a = list(set(c.ids))
        kn.accounts = {i: v for i, v in zip(uniq_a, d.account_shards(uniq_a)) if v is not None}
        return kn

    def _collisions(self, c: _Call) -> Dict[int, set]:
        ts = sorted({c.ts[k] for k in range(c.n) if c.imp_live[k]})
        if not ts:
            return {}
        found = self.ops.timestamps_exist(not c.is_tr, np.asarray(ts, dtype=np.uint64))
        coll: Dict[int, set] = {}
        for s, f in enumerate(found):
            for t in np.asarray(ts, dtype=np.uint64)[np.asarray(f, dtype=bool)].tolist():
                coll.setdefault(int(t), set()).add(s)
        return coll

    # -- the exec form of a segment's events ------------------------------------------------------

    def _exec_events(self, c: _Call, seg: _Seg, ks: List[int]) -> Tuple[np.ndarray, dict]:
        """Events k in `ks` as their shards run them, and the result patches (k -> (status the
        shard reports, the reference's status))."""
        ev = c.events[ks].copy() if ks else np.zeros(0, dtype=c.kind.dtype)
        patches = {}
        for j, k in enumerate(ks):
            g = c.G[k]
            inert_st = c.kind.inert_imported if g else c.kind.inert_plain
            if k in c.pre or k in seg.decided:
                ev[j] = inert_event(c.kind, g, bool(c.flags[k] & 1))
                patches[k] = (inert_st, c.pre[k] if k in c.pre else seg.decided[k])
            elif k in seg.cross:
                ev["credit_account_id"][j] = ev["debit_account_id"][j]
                patches[k] = (int(_CT.accounts_must_be_different), seg.cross[k])
        if seg.tprime:
            where = {k: j for j, k in enumerate(ks)}
            for k, t in self._tprime_values(c, seg).items():
                if k in where:
                    ev["timestamp"][where[k]] = t
        return ev, patches

    def _tprime_values(self, c: _Call, seg: _Seg) -> Dict[int, int]:
        """A timestamp that fails must_not_regress on the event's shard once the event reaches the
        imported checks: its debit account's (a post/void's: its pending transfer's), found in
        the shard's accounts by timestamp (:3813-3817). 1 when that account is not on the shard
        (the event fails before the imported checks)."""
        need_acc: Dict[int, set] = {}
        need_pend: Dict[int, set] = {}
        for k, s in seg.tprime.items():
            if c.flags[k] & _POST_VOID:
                need_pend.setdefault(s, set()).add(c.pids[k])
            else:
                need_acc.setdefault(s, set()).add(c.drs[k])
        pend_dr: Dict[Tuple[int, int], int] = {}
        for s, ids in need_pend.items():
            for p, row in self.ops.lookup_transfers(s, sorted(ids)).items():
                dr = int(row["debit_account_id"][0]) | (int(row["debit_account_id"][1]) << 64)
                pend_dr[(s, p)] = dr
                need_acc.setdefault(s, set()).add(dr)
        acc_ts: Dict[Tuple[int, int], int] = {}
        for s, ids in need_acc.items():
            for i, row in self.ops.lookup_accounts(s, sorted(ids)).items():
                acc_ts[(s, i)] = int(row["timestamp"])
        out = {}
        for k, s in seg.tprime.items():
            dr = pend_dr.get((s, c.pids[k])) if c.flags[k] & _POST_VOID else c.drs[k]
            out[k] = acc_ts.get((s, dr), 1) if dr is not None else 1
        return out

    # -- segments -------------------------------------------------------------------------------

    def _run_segment(self, c: _Call, seg: _Seg, results: np.ndarray):
        W = self.router.shards
        subcalls: List[List[SubCall]] = [[] for _ in range(W)]
        positions: List[List[List[int]]] = [[] for _ in range(W)]
        ks = list(range(seg.start, seg.end))
        ev_all, patches = self._exec_events(c, seg, ks)
        off = seg.start
        pending = [None] * W  # an open "batches" sub-call per shard: (positions, lens, batch_ts)

        def flush(s):
            if pending[s] is not None:
                pos, lens, bts = pending[s]
                subcalls[s].append(SubCall("batches", ev_all[np.asarray(pos) - off],
                                           np.asarray(lens, np.uint32),
                                           np.asarray(bts, np.uint64)))
                positions[s].append(pos)
                pending[s] = None

        b = c.b_of[seg.start]
        while b < len(c.batch_start) and c.batch_start[b] < seg.end:
            lo, hi = max(seg.start, c.batch_start[b]), min(seg.end, c.batch_end[b])
            if lo < hi and c.g_batch[b]:
                per = [[] for _ in range(W)]
                for k in range(lo, hi):
                    per[seg.shard_of[k]].append(k)
                for s in range(W):
                    if per[s]:
                        flush(s)
                        subcalls[s].append(SubCall(
                            "stamped", ev_all[np.asarray(per[s]) - off],
                            np.asarray([c.stamp[k] for k in per[s]], np.uint64),
                            np.asarray([c.batch_ts[b]], np.uint64)))
                        positions[s].append(per[s])
            elif lo < hi:
                k = lo
                while k < hi:
                    s = seg.shard_of[k]
                    j = k
                    while j < hi and seg.shard_of[j] == s:
                        j += 1
                    if pending[s] is not None and len(pending[s][1]) >= self.max_batches:
                        flush(s)  # (a sub-call holds at most the executor's batch_count_max)
                    if pending[s] is None:
                        pending[s] = ([], [], [])
                    pending[s][0].extend(range(k, j))
                    pending[s][1].append(j - k)
                    pending[s][2].append(c.stamp[j - 1])
                    k = j
            b += 1
        for s in range(W):
            flush(s)
        if seg.imported:
            self.ops.sync_key_max()
        outs, pnts = self.ops.execute(c.kind, subcalls)
        for s in range(W):
            for pos, r in zip(positions[s], outs[s]):
                results[pos] = r
        self._patch(results, patches)
        if c.is_tr and seg.post_void:
            self._resolve_pnt([p[0] for p in pnts], [p[1] for p in pnts])

    def _run_chain(self, c: _Call, seg: _Seg, results: np.ndarray):
        """One linked chain across shards (module doc). Every shard probes its part without the
        chain's last event: one chain (TBG_ONE_CHAIN) ending in an inert sentinel, so it always
        rolls back and reports its first failure. No failure before the last event: the last
        event's shard commits its part, the last event included -- the chain's outcome; if it
        succeeds, every other shard commits its part (the same state as its probe saw, so it
        succeeds)."""
        W = self.router.shards
        a, z = seg.start, seg.end
        last = z - 1
        open_ = c.open_last[last]
        b = c.b_of[a]
        T_b = c.batch_ts[b]
        g = c.g_batch[b]
        s_last = seg.shard_of[last]
        parts = [[] for _ in range(W)]
        for k in range(a, last):
            parts[seg.shard_of[k]].append(k)
        ev_all, patches = self._exec_events(c, seg, list(range(a, z)))

        def part_call(ks, sentinel):
            ev = ev_all[np.asarray(ks) - a]
            stamps = [c.stamp[k] for k in ks]
            if sentinel:
                ev = np.concatenate([ev, np.asarray([inert_event(c.kind, g, False)],
                                                    dtype=c.kind.dtype)])
                stamps.append(stamps[-1] + 1)
            return SubCall("stamped", ev, np.asarray(stamps, np.uint64),
                           np.asarray([T_b], np.uint64), one_chain=True)

        if seg.imported:
            self.ops.sync_key_max()
        saved = self.ops.pnt_values() if c.is_tr else None
        probe = [[part_call(parts[s], True)] if parts[s] else [] for s in range(W)]
        outs, pnts = self.ops.execute(c.kind, probe)
        first: Dict[int, int] = {}  # shard -> its part's first failing event
        for s in range(W):
            if not parts[s]:
                continue
            r = outs[s][0]
            results[parts[s]] = r[:len(parts[s])]
            for j, k in enumerate(parts[s]):
                if int(r["status"][j]) != LINKED_EVENT_FAILED:
                    first[s] = k
                    break
        fail = min(first.values()) if first else None
        if fail is None and open_:
            fail = last  # linked_event_chain_open (:3039-3042)
        if fail is None:
            # the last event decides: its shard commits its part with it
            ks = parts[s_last] + [last]
            o, p = self.ops.execute(c.kind, [[part_call(ks, False)] if s == s_last else []
                                             for s in range(W)])
            results[ks] = o[s_last][0]
            ops_lists = [pnts[s][1] if pnts[s] else [] for s in range(W)] if c.is_tr else None
            if c.is_tr:
                ops_lists[s_last] = p[s_last][1]
            if int(results["status"][last]) == STATUS_CREATED:
                rest = [[part_call(parts[s], False)] if parts[s] and s != s_last else []
                        for s in range(W)]
                if any(rest):
                    o2, p2 = self.ops.execute(c.kind, rest)
                    for s in range(W):
                        if rest[s]:
                            results[parts[s]] = o2[s][0]
                            if c.is_tr:
                                ops_lists[s] = p2[s][1]
                if (results["status"][a:z] != STATUS_CREATED).any():
                    raise RuntimeError("a linked chain across shards failed on its commit after "
                                       "its probe succeeded: the shards' state is undefined")
            else:
                # failed at its last event: that shard rolled back (orphaning it if transient,
                # :3172); the other shards' probes already did
                self._patch(results, {last: patches[last]} if last in patches else {})
            if c.is_tr and seg.post_void and pnt_resets_fire(saved, ops_lists):
                self.ops.set_pnt([TIMESTAMP_MIN] * W)
            return
        # The chain fails at `fail`: the reference executed (and rolled back) the events before it.
        for k in range(fail + 1, z):
            results[k]["timestamp"] = c.stamp[k]
            results[k]["status"] = LINKED_EVENT_FAILED
            results[k]["reserved"] = 0
        if open_:
            results[last]["timestamp"] = c.stamp[last]
            results[last]["status"] = LINKED_EVENT_CHAIN_OPEN
            results[last]["reserved"] = 0
        self._patch(results, {k: v for k, v in patches.items() if k <= fail})
        if c.is_tr:
            forget = [[] for _ in range(W)]
            for s, k in first.items():
                if k != fail and int(outs[s][0]["status"][parts[s].index(k)]) in _TRANSIENT:
                    forget[s].append(c.ids[k])
            if any(forget):
                self.ops.forget_orphans(forget)
            # pulse_next_timestamp: the shards' values before the probe, lowered by the updates of
            # the events the reference executed (those before the failure)
            cut = c.stamp[fail]
            kept = [[(t, o) for t, o in (p[1] if p else []) if t < cut] for p in pnts]
            values = []
            for s in range(W):
                v = int(saved[s])
                for _, o in kept[s]:
                    if not o & PNT_RESET and o < v:
                        v = o
                values.append(v)
            if pnt_resets_fire(saved, kept):
                values = [TIMESTAMP_MIN] * W
            self.ops.set_pnt(values)

    @staticmethod
    def _patch(results: np.ndarray, patches: dict):
        for k, (expect, status) in patches.items():
            if int(results["status"][k]) == expect:
                results["status"][k] = status

    def _resolve_pnt(self, starts, op_lists):
        if pnt_resets_fire(starts, op_lists):
            self.ops.set_pnt([TIMESTAMP_MIN] * self.router.shards)

    # -- the call ---------------------------------------------------------------------------------

    def run(self, kind: _Kind, events: np.ndarray, lens, batch_ts) -> np.ndarray:
        events = np.ascontiguousarray(events, dtype=kind.dtype)
        c = _Call(kind, events, lens, batch_ts)
        results = np.zeros(c.n, dtype=RESULT_DTYPE)
        if c.n == 0:
            return results
        known = self._known(c)
        planner = Planner(self.router, c, known, self._collisions(c))
        pos = 0
        while pos < c.n:
            seg = planner.plan(pos)
            if seg.chain:
                self._run_chain(c, seg, results)
                self.chain_segments += 1
            else:
                self._run_segment(c, seg, results)
            self.segments += 1
            ks = list(range(seg.start, seg.end))
            rec = self.router.record(
                kind, [c.ids[k] for k in ks], [seg.shard_of[k] for k in ks],
                results["status"][seg.start:seg.end].tolist(),
                [bool(c.is_tr and c.flags[k] & _PENDING and c.timeouts[k] > 0) for k in ks])
            for i, sh, timed in rec:
                if kind is ACCOUNTS:
                    known.accounts[i] = sh
                else:
                    known.transfers.setdefault(i, (sh, timed))
            pos = seg.end
        return results


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


# ---- shard groups -----------------------------------------------------------------------------

class LocalShards:
    """All shards in one process (one executor each: several HBM table sets on one GPU, or CPU
    executors in tests). `executors[s]` provides the shard executor interface (GpuShard)."""

    def __init__(self, router: LedgerRouter, executors, pulse_batch_max: int = 8190):
        if len(executors) != router.shards:
            raise ValueError("one executor per shard")
        self.router = router
        self.executors = executors
        self.pulse_batch_max = pulse_batch_max
        self.engine = Engine(router, self)
        for ex in executors:
            ex.set_pnt_sharded(True)

    # the shard-group operations the Engine issues
    def execute(self, kind, subcalls):
        outs, pnts = [], []
        for ex, scs in zip(self.executors, subcalls):
            o, p = run_subcalls(ex, kind, scs)
            outs.append(o)
            pnts.append(p)
        return outs, pnts

    def pnt_values(self):
        return [int(ex.pulse_next_timestamp()) for ex in self.executors]

    def set_pnt(self, values):
        for ex, v in zip(self.executors, values):
            ex.set_pulse_next_timestamp(int(v))

    def forget_orphans(self, ids_by_shard):
        for ex, ids in zip(self.executors, ids_by_shard):
            if ids:
                ex.forget_orphans(ids)

    def timestamps_exist(self, transfers, ts):
        return [ex.timestamps_exist(transfers, ts) for ex in self.executors]

    def sync_key_max(self):
        maxima = [ex.key_max() for ex in self.executors]
        a = max(m[0] for m in maxima)
        t = max(m[1] for m in maxima)
        for ex in self.executors:
            ex.raise_key_max(a, t)
        return a, t

    def lookup_accounts(self, s, ids):
        return self.executors[s].lookup_accounts(ids)

    def lookup_transfers(self, s, ids):
        return self.executors[s].lookup_transfers(ids)

    # the client interface
    def create_accounts(self, events, lens, batch_ts):
        return self.engine.run(ACCOUNTS, events, lens, batch_ts)

    def create_transfers(self, events, lens, batch_ts):
        return self.engine.run(TRANSFERS, events, lens, batch_ts)

    def pulse_next_timestamp(self) -> int:
        return min(self.pnt_values())

    def pulse(self, timestamp: int) -> int:
        cands = [ex.pulse_candidates(timestamp, self.pulse_batch_max) for ex in self.executors]
        cut, pnt, stamps = pulse_plan([c for c, _ in cands], [k for _, k in cands],
                                      self.pulse_batch_max, timestamp)
        return sum(int(ex.pulse_cut(timestamp, cut[0], cut[1], pnt, st))
                   for ex, st in zip(self.executors, stamps))


# ShardGroup commands (rank 0 -> every rank, a broadcast word vector)
_CMD_END, _CMD_ABORT, _CMD_EXEC, _CMD_PNT_GET, _CMD_PNT_SET, _CMD_FORGET, _CMD_TS_EXIST, \
    _CMD_KEY_MAX, _CMD_LOOKUP_ACC, _CMD_LOOKUP_TR = range(10)
_CMD_WORDS = 4


class ShardGroup:
    """One shard per rank of a torch.distributed group (one process per GPU). Rank 0 owns the
    router and the client call and runs the Engine; the other ranks serve its commands for the
    length of the call (the executor calls, pulse_next_timestamp reads and writes, key maxima,
    lookups), each a broadcast command word followed by point-to-point transfers of the data.
    With the `nccl` backend (RCCL over xGMI) the data travels device to device; with gloo it
    stays on the host. `executor` is this rank's shard.
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
        self.engine = Engine(router, self) if self.rank == 0 else None
        self._failure = None
        executor.set_pnt_sharded(True)

    # -- transport ------------------------------------------------------------------------------

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

    def _bcast_words(self, words):
        import torch
        t = torch.tensor(words, dtype=torch.int64, device=self.device)
        self.dist.broadcast(t, self._peer(0), group=self.group)
        return [int(x) for x in t.tolist()]

    def _bcast(self, value: int) -> int:
        return self._bcast_words([value])[0]

    def _cmd(self, cmd: int, *args):
        w = [cmd] + list(args)
        self._bcast_words(w + [0] * (_CMD_WORDS - len(w)))

    # -- commands: rank 0's side (the Engine's shard-group operations) ----------------------------

    def execute(self, kind, subcalls):
        self._cmd(_CMD_EXEC, int(kind is TRANSFERS))
        for s in range(1, self.world):
            self._send_subcalls(subcalls[s], s)
        mine = self._exec_local(kind, subcalls[0])
        outs, pnts, failed = [mine[0]], [mine[1]], [mine[2]]
        for s in range(1, self.world):
            o, p, f = self._recv_outcome(kind, s, [len(sc.events) for sc in subcalls[s]])
            outs.append(o)
            pnts.append(p)
            failed.append(f)
        if any(failed):
            if self._failure is not None:
                raise self._failure
            raise RuntimeError("a shard's executor failed; the shards' state is undefined")
        return outs, pnts

    def pnt_values(self):
        self._cmd(_CMD_PNT_GET)
        vals = [int(self.executor.pulse_next_timestamp())]
        for s in range(1, self.world):
            vals.append(int(self._recv(s, np.uint64)[0]))
        return vals

    def set_pnt(self, values):
        self._cmd(_CMD_PNT_SET)
        for s in range(1, self.world):
            self._send(np.asarray([values[s]], dtype=np.uint64), s)
        self.executor.set_pulse_next_timestamp(int(values[0]))

    def forget_orphans(self, ids_by_shard):
        self._cmd(_CMD_FORGET)
        for s in range(1, self.world):
            self._send(_u128_array(ids_by_shard[s]), s)
        if ids_by_shard[0]:
            self.executor.forget_orphans(ids_by_shard[0])

    def timestamps_exist(self, transfers, ts):
        self._cmd(_CMD_TS_EXIST, int(bool(transfers)))
        for s in range(1, self.world):
            self._send(np.asarray(ts, dtype=np.uint64), s)
        out = [self.executor.timestamps_exist(transfers, ts)]
        for s in range(1, self.world):
            out.append(self._recv(s, np.uint8).astype(bool))
        return out

    def sync_key_max(self):
        import torch
        self._cmd(_CMD_KEY_MAX)
        return self._key_max_collective(torch)

    def _key_max_collective(self, torch):
        a, t = self.executor.key_max()
        v = torch.tensor([int(a), int(t)], dtype=torch.int64, device=self.device)
        self.dist.all_reduce(v, op=self.dist.ReduceOp.MAX, group=self.group)
        a, t = (int(x) for x in v.tolist())
        self.executor.raise_key_max(a, t)
        return a, t

    def lookup_accounts(self, s, ids):
        return self._lookup(_CMD_LOOKUP_ACC, s, ids, ACCOUNT_DTYPE)

    def lookup_transfers(self, s, ids):
        return self._lookup(_CMD_LOOKUP_TR, s, ids, TRANSFER_DTYPE)

    def _lookup(self, cmd, s, ids, dtype):
        if s == 0:
            return (self.executor.lookup_accounts(ids) if cmd == _CMD_LOOKUP_ACC
                    else self.executor.lookup_transfers(ids))
        self._cmd(cmd, s)
        self._send(_u128_array(ids), s)
        rows = self._recv(s, dtype)
        return {int(r["id"][0]) | (int(r["id"][1]) << 64): r for r in rows}

    # -- serialisation of sub-calls and outcomes --------------------------------------------------

    def _send_subcalls(self, scs: List[SubCall], dst: int):
        self._send(np.asarray([len(scs)] + [(0 if sc.mode == "batches" else 1 + int(sc.one_chain))
                                            for sc in scs], dtype=np.int64), dst)
        for sc in scs:
            self._send(np.ascontiguousarray(sc.events), dst)
            self._send(np.asarray(sc.aux, dtype=np.uint64), dst)
            self._send(np.asarray(sc.batch_ts, dtype=np.uint64), dst)

    def _recv_subcalls(self, kind) -> List[SubCall]:
        hdr = self._recv(0, np.int64)
        out = []
        for j in range(int(hdr[0])):
            ev = self._recv(0, kind.dtype)
            aux = self._recv(0, np.uint64)
            bts = self._recv(0, np.uint64)
            out.append(SubCall("stamped" if hdr[1 + j] else "batches", ev, aux, bts,
                               one_chain=int(hdr[1 + j]) == 2))
        return out

    def _exec_local(self, kind, scs):
        try:
            outs, pnt = run_subcalls(self.executor, kind, scs)
            return outs, pnt, False
        except Exception as e:  # noqa: BLE001 -- every rank must learn of it
            self._failure = e
            return [], None, True

    def _send_outcome(self, kind, outs, pnt, failed):
        self._send(np.asarray([int(failed)], dtype=np.int64), 0)
        res = np.concatenate(outs) if outs else np.zeros(0, dtype=RESULT_DTYPE)
        self._send(res, 0)
        if kind is TRANSFERS:
            start, ops = pnt if pnt is not None else (0, [])
            self._send(np.asarray([start] + [x for pair in ops for x in pair], dtype=np.uint64), 0)

    def _recv_outcome(self, kind, s, lens):
        failed = bool(self._recv(s, np.int64)[0])
        res = self._recv(s, RESULT_DTYPE)
        pnt = None
        if kind is TRANSFERS:
            a = self._recv(s, np.uint64)
            pnt = (int(a[0]), list(zip(a[1::2].tolist(), a[2::2].tolist())))
        outs = []
        if not failed:
            off = 0
            for ln in lens:
                outs.append(res[off:off + ln])
                off += ln
        return outs, pnt, failed

    # -- the serving loop of ranks > 0 ------------------------------------------------------------

    def _serve(self):
        import torch
        while True:
            w = self._bcast_words([0] * _CMD_WORDS)
            cmd = w[0]
            if cmd == _CMD_END:
                return
            if cmd == _CMD_ABORT:
                f, self._failure = self._failure, None
                if f is not None:
                    raise f
                raise RuntimeError("the call failed on another rank; the shards' state is "
                                   "undefined")
            if cmd == _CMD_EXEC:
                kind = TRANSFERS if w[1] else ACCOUNTS
                scs = self._recv_subcalls(kind)
                outs, pnt, failed = self._exec_local(kind, scs)
                self._send_outcome(kind, outs, pnt, failed)
            elif cmd == _CMD_PNT_GET:
                self._send(np.asarray([self.executor.pulse_next_timestamp()], dtype=np.uint64), 0)
            elif cmd == _CMD_PNT_SET:
                self.executor.set_pulse_next_timestamp(int(self._recv(0, np.uint64)[0]))
            elif cmd == _CMD_FORGET:
                ids = self._recv(0, np.uint64).reshape(-1, 2)
                if len(ids):
                    self.executor.forget_orphans([int(a) | (int(b) << 64) for a, b in ids])
            elif cmd == _CMD_TS_EXIST:
                ts = self._recv(0, np.uint64)
                self._send(np.asarray(self.executor.timestamps_exist(bool(w[1]), ts),
                                      dtype=np.uint8), 0)
            elif cmd == _CMD_KEY_MAX:
                self._key_max_collective(torch)
            elif cmd in (_CMD_LOOKUP_ACC, _CMD_LOOKUP_TR):
                if w[1] == self.rank:
                    ids = self._recv(0, np.uint64).reshape(-1, 2)
                    ids = [int(a) | (int(b) << 64) for a, b in ids]
                    found = (self.executor.lookup_accounts(ids) if cmd == _CMD_LOOKUP_ACC
                             else self.executor.lookup_transfers(ids))
                    dtype = ACCOUNT_DTYPE if cmd == _CMD_LOOKUP_ACC else TRANSFER_DTYPE
                    rows = np.asarray(list(found.values()), dtype=dtype) if found \
                        else np.zeros(0, dtype=dtype)
                    self._send(rows, 0)
            else:
                raise RuntimeError(f"ShardGroup: unknown command {cmd}")

    def _call(self, kind, events, lens, batch_ts):
        if self.rank != 0:
            self._serve()
            return None
        try:
            res = self.engine.run(kind, events, lens, batch_ts)
        except BaseException:
            self._cmd(_CMD_ABORT)
            self._failure = None
            raise
        self._cmd(_CMD_END)
        return res

    # -- the client interface (collective: rank 0 passes the call, the others no arguments) -------

    def create_accounts(self, events=None, lens=None, batch_ts=None):
        return self._call(ACCOUNTS, events, lens, batch_ts)

    def create_transfers(self, events=None, lens=None, batch_ts=None):
        return self._call(TRANSFERS, events, lens, batch_ts)

    def resolve_pnt(self, executed=True):
        """Collective, after a call the device router executed that posts or voids: every shard's
        recorded pulse_next_timestamp updates to rank 0 (its start value, then (timestamp, op)
        pairs; a shard that executed nothing of the call sends its value alone), replayed in call
        order there; the outcome broadcast."""
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

    def sync_key_max_collective(self):
        """Collective (every rank): the key maxima over all shards raised on every shard."""
        import torch
        return self._key_max_collective(torch)

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
    """A shard backed by libtbg.so (its HBM tables on `device`): the shard executor interface."""

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

    def _stamped(self, fn, events, stamps, batch_timestamp, options):
        c = self._c
        n = len(events)
        st = np.ascontiguousarray(stamps, dtype=np.uint64)
        out = np.zeros(n, dtype=RESULT_DTYPE)
        rc = fn(self.g, events.ctypes.data_as(c.c_void_p), n, st.ctypes.data_as(c.c_void_p),
                int(batch_timestamp), int(options), out.ctypes.data_as(c.c_void_p))
        if rc != 0:
            raise RuntimeError(f"libtbg: {rc} {self.lib.tbg_last_error(self.g)}")
        return out

    def create_accounts(self, events, lens, batch_ts):
        return self._call(self.lib.tbg_create_accounts,
                          np.ascontiguousarray(events, dtype=ACCOUNT_DTYPE), lens, batch_ts)

    def create_transfers(self, events, lens, batch_ts):
        return self._call(self.lib.tbg_create_transfers,
                          np.ascontiguousarray(events, dtype=TRANSFER_DTYPE), lens, batch_ts)

    def create_accounts_stamped(self, events, stamps, batch_timestamp=0, options=0):
        return self._stamped(self.lib.tbg_create_accounts_stamped,
                             np.ascontiguousarray(events, dtype=ACCOUNT_DTYPE), stamps,
                             batch_timestamp, options)

    def create_transfers_stamped(self, events, stamps, batch_timestamp=0, options=0):
        return self._stamped(self.lib.tbg_create_transfers_stamped,
                             np.ascontiguousarray(events, dtype=TRANSFER_DTYPE), stamps,
                             batch_timestamp, options)

    def forget_orphans(self, ids):
        a = _u128_array(list(ids))
        n = int(self.lib.tbg_forget_orphans(self.g, a.ctypes.data_as(self._c.c_void_p), len(a)))
        if n < 0:
            raise RuntimeError(f"libtbg: {n} {self.lib.tbg_last_error(self.g)}")
        return n

    def timestamps_exist(self, transfers, ts):
        ts = np.ascontiguousarray(ts, dtype=np.uint64)
        out = np.zeros(len(ts), dtype=np.uint8)
        n = int(self.lib.tbg_timestamps_exist(self.g, int(bool(transfers)),
                                              ts.ctypes.data_as(self._c.c_void_p), len(ts),
                                              out.ctypes.data_as(self._c.c_void_p)))
        if n < 0:
            raise RuntimeError(f"libtbg: {n} {self.lib.tbg_last_error(self.g)}")
        return out.astype(bool)

    def key_max(self):
        """The objects trees' key_range.key_max (accounts, transfers; 0 = no key range)."""
        c = self._c
        a, t = c.c_uint64(), c.c_uint64()
        rc = self.lib.tbg_key_max(self.g, c.byref(a), c.byref(t))
        if rc != 0:
            raise RuntimeError(f"libtbg: {rc} {self.lib.tbg_last_error(self.g)}")
        return int(a.value), int(t.value)

    def lookup_accounts(self, ids):
        return self._lookup(self.lib.tbg_lookup_accounts, ids, ACCOUNT_DTYPE)

    def lookup_transfers(self, ids):
        return self._lookup(self.lib.tbg_lookup_transfers, ids, TRANSFER_DTYPE)

    def _lookup(self, fn, ids, dtype):
        ids = list(ids)
        if not ids:
            return {}
        a = _u128_array(ids)
        out = np.zeros(len(ids), dtype=dtype)
        n = int(fn(self.g, a.ctypes.data_as(self._c.c_void_p), len(ids),
                   out.ctypes.data_as(self._c.c_void_p)))
        if n < 0:
            raise RuntimeError(f"libtbg: {n} {self.lib.tbg_last_error(self.g)}")
        return {int(r["id"][0]) | (int(r["id"][1]) << 64): r for r in out[:n]}

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
