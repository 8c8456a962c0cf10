"""Shards in other processes behind the group's shard executor interface (include/tbg_group.h,
tbg_shard_ops): the exact engine (csrc/engine.cpp) running one process per GPU -- or per node --
over torch.distributed.

Rank 0 owns the group: the engine, its directories and the client calls. Every rank owns one
executor (its GPU's tbg_ctx, or in the tests the CPU oracle) bound through a C shard-ops table.
The group's ops table on rank 0 is a table of Python callbacks: an operation on rank 0's own shard
calls its C op with the engine's pointers as they are; an operation on shard s is sent to rank s
(a header word vector, then the input buffers) and rank s replies (a return code, then the output
buffers). Ranks > 0 serve until rank 0 ends the session. The transport is torch.distributed's
point-to-point send / recv of host tensors, so the process group must carry CPU tensors (gloo; an
RCCL group would need the buffers staged in device memory, which this module does not do).

The in-process group over a node's GPUs (tbg_group_open: device router, peer stores, per-shard
threads) is the production path; this transport is for executors the caller cannot put in one
process (separate nodes), and it is what the world-2 gloo test runs.
"""
import ctypes

import numpy as np

from . import shard as _shard

vp = ctypes.c_void_p
u32, u64, i64, cint = ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int
p32, p64, p8 = ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint64), \
    ctypes.POINTER(ctypes.c_uint8)

# tbg_shard_ops members, in order: (name, C signature)
SIGS = [
    ("create_accounts", ctypes.CFUNCTYPE(cint, vp, vp, u32, vp, vp, u32, vp)),
    ("create_transfers", ctypes.CFUNCTYPE(cint, vp, vp, u32, vp, vp, u32, vp)),
    ("create_accounts_stamped", ctypes.CFUNCTYPE(cint, vp, vp, u32, vp, u64, u32, vp)),
    ("create_transfers_stamped", ctypes.CFUNCTYPE(cint, vp, vp, u32, vp, u64, u32, vp)),
    ("forget_orphans", ctypes.CFUNCTYPE(i64, vp, vp, u32)),
    ("timestamps_exist", ctypes.CFUNCTYPE(i64, vp, cint, vp, u32, vp)),
    ("key_max", ctypes.CFUNCTYPE(cint, vp, vp, vp)),
    ("raise_key_max", ctypes.CFUNCTYPE(cint, vp, u64, u64)),
    ("set_pnt_sharded", ctypes.CFUNCTYPE(cint, vp, cint)),
    ("pnt_ops", ctypes.CFUNCTYPE(i64, vp, vp, vp, u64, vp)),
    ("pulse_next_timestamp", ctypes.CFUNCTYPE(u64, vp)),
    ("set_pulse_next_timestamp", ctypes.CFUNCTYPE(cint, vp, u64)),
    ("pulse_candidates", ctypes.CFUNCTYPE(i64, vp, u64, vp, vp, u32)),
    ("pulse_cut", ctypes.CFUNCTYPE(i64, vp, u64, u64, u64, u64, vp)),
    ("lookup_accounts", ctypes.CFUNCTYPE(i64, vp, vp, u32, vp)),
    ("lookup_transfers", ctypes.CFUNCTYPE(i64, vp, vp, u32, vp)),
]
OP = {name: i for i, (name, _) in enumerate(SIGS)}
_END = -1
_HDR = 8  # header words: op, up to 6 scalars, payload bytes


def _bytes(ptr, n):
    return np.frombuffer(ctypes.string_at(ptr, n), dtype=np.uint8).copy() if n else \
        np.zeros(0, dtype=np.uint8)


def _put(ptr, arr):
    if len(arr):
        ctypes.memmove(ptr, np.ascontiguousarray(arr).ctypes.data, arr.nbytes)


class _Local:
    """A rank's own executor: its C ops table called with raw pointers."""

    def __init__(self, ops: _shard.ShardOps, self_ptr):
        self.self = self_ptr
        self.fns = {name: sig(getattr(ops, name)) for name, sig in SIGS}

    def __call__(self, name, *args):
        return self.fns[name](self.self, *args)


class RemoteShards:
    """One shard per rank. Rank 0 (`rank == 0`): `group` is the tbg_group over every rank's shard
    (shard.Group); call `close()` to end the session. Other ranks: `serve()` until rank 0 ends it.
    `local_ops` / `local_self`: this rank's executor as a C shard-ops table and its pointer."""

    def __init__(self, local_ops: _shard.ShardOps, local_self, group=None, **group_options):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.dist = dist
        self.pg = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.local = _Local(local_ops, local_self)
        self._keys = {}  # shard -> its last pulse_candidates keys (pulse_cut's stamps count)
        self.group = None
        if self.rank == 0:
            self._cbs = [sig(self._callback(name)) for name, sig in SIGS]
            ops = _shard.ShardOps()
            for (name, _), cb in zip(SIGS, self._cbs):
                setattr(ops, name, ctypes.cast(cb, vp).value)
            # (self pointers: shard s is s + 1, never NULL)
            self.group = _shard.Group.open_shards(ops, [s + 1 for s in range(self.world)],
                                                  **group_options)

    # -- transport ------------------------------------------------------------------------------

    def _peer(self, r):
        return r if self.pg is None else self.dist.get_global_rank(self.pg, r)

    def _send(self, words, payload, dst):
        t = self.torch
        hdr = t.tensor(list(words) + [0] * (_HDR - 1 - len(words)) + [len(payload)],
                       dtype=t.int64)
        self.dist.send(hdr, self._peer(dst), group=self.pg)
        if len(payload):
            self.dist.send(t.from_numpy(np.ascontiguousarray(payload)), self._peer(dst),
                           group=self.pg)

    def _recv(self, src):
        t = self.torch
        hdr = t.zeros(_HDR, dtype=t.int64)
        self.dist.recv(hdr, self._peer(src), group=self.pg)
        words = [int(x) for x in hdr.tolist()]
        n = words[-1]
        payload = np.zeros(n, dtype=np.uint8)
        if n:
            buf = t.from_numpy(payload)
            self.dist.recv(buf, self._peer(src), group=self.pg)
        return words[:-1], payload

    def _rpc(self, s, name, scalars, payload):
        self._send([OP[name]] + list(scalars), payload, s)
        words, reply = self._recv(s)
        return words[0], reply

    # -- rank 0: the callbacks the engine calls ---------------------------------------------------

    def _callback(self, name):
        def cb(self_ptr, *args):
            try:
                s = int(self_ptr) - 1
                if s == 0:
                    return self.local(name, *args)
                return getattr(self, "_remote_" + name)(s, *args)
            except Exception:  # noqa: BLE001 -- an error code for the engine, never an exception
                import traceback
                traceback.print_exc()
                return -5
        return cb

    def _remote_create(self, name, s, ev, n, lens, bts, nb, out):
        lens_b = _bytes(lens, nb * 4)
        payload = np.concatenate([_bytes(ev, n * 128), lens_b, _bytes(bts, nb * 8)])
        rc, reply = self._rpc(s, name, [n, nb], payload)
        if rc == 0:
            _put(out, reply)
        return rc

    def _remote_create_accounts(self, s, *a):
        return self._remote_create("create_accounts", s, *a)

    def _remote_create_transfers(self, s, *a):
        return self._remote_create("create_transfers", s, *a)

    def _remote_stamped(self, name, s, ev, n, stamps, bts, opt, out):
        payload = np.concatenate([_bytes(ev, n * 128), _bytes(stamps, n * 8)])
        rc, reply = self._rpc(s, name, [n, bts, opt], payload)
        if rc == 0:
            _put(out, reply)
        return rc

    def _remote_create_accounts_stamped(self, s, *a):
        return self._remote_stamped("create_accounts_stamped", s, *a)

    def _remote_create_transfers_stamped(self, s, *a):
        return self._remote_stamped("create_transfers_stamped", s, *a)

    def _remote_forget_orphans(self, s, ids, n):
        return self._rpc(s, "forget_orphans", [n], _bytes(ids, n * 16))[0]

    def _remote_timestamps_exist(self, s, transfers, ts, n, out):
        rc, reply = self._rpc(s, "timestamps_exist", [transfers, n], _bytes(ts, n * 8))
        if rc >= 0:
            _put(out, reply)
        return rc

    def _remote_key_max(self, s, a, t):
        rc, reply = self._rpc(s, "key_max", [], np.zeros(0, np.uint8))
        if rc == 0:
            v = reply.view(np.uint64)
            ctypes.c_uint64.from_address(a).value = int(v[0])
            ctypes.c_uint64.from_address(t).value = int(v[1])
        return rc

    def _remote_raise_key_max(self, s, a, t):
        return self._rpc(s, "raise_key_max", [a, t], np.zeros(0, np.uint8))[0]

    def _remote_set_pnt_sharded(self, s, on):
        return self._rpc(s, "set_pnt_sharded", [on], np.zeros(0, np.uint8))[0]

    def _remote_pnt_ops(self, s, ts, ops, mx, start):
        rc, reply = self._rpc(s, "pnt_ops", [int(bool(ts and ops)), mx], np.zeros(0, np.uint8))
        v = reply.view(np.uint64)
        if start:
            ctypes.c_uint64.from_address(start).value = int(v[0])
        if rc > 0 and ts and ops:
            m = min(rc, mx)
            _put(ts, v[1:1 + m])
            _put(ops, v[1 + m:1 + 2 * m])
        return rc

    def _remote_pulse_next_timestamp(self, s):
        _, reply = self._rpc(s, "pulse_next_timestamp", [], np.zeros(0, np.uint8))
        return int(reply.view(np.uint64)[0])

    def _remote_set_pulse_next_timestamp(self, s, v):
        return self._rpc(s, "set_pulse_next_timestamp", [v], np.zeros(0, np.uint8))[0]

    def _remote_pulse_candidates(self, s, ts, e, t, mx):
        rc, reply = self._rpc(s, "pulse_candidates", [ts, mx], np.zeros(0, np.uint8))
        if rc >= 0:
            m = min(rc, mx)
            v = reply.view(np.uint64)
            _put(e, v[:m])
            _put(t, v[m:2 * m])
            self._keys[s] = list(zip(v[:m].tolist(), v[m:2 * m].tolist()))
        return rc

    def _remote_pulse_cut(self, s, ts, ce, ct, pnt, stamps):
        # (the shard's expiries: its candidates up to the cut -- pulse_plan's cut is the largest
        # key when nothing is cut, engine.hpp)
        m = sum(1 for k in self._keys.get(s, []) if k <= (ce, ct))
        payload = _bytes(stamps, m * 8) if stamps else np.zeros(0, np.uint8)
        return self._rpc(s, "pulse_cut", [ts, ce, ct, pnt, int(bool(stamps))], payload)[0]

    def _remote_lookup(self, name, s, ids, n, out):
        rc, reply = self._rpc(s, name, [n], _bytes(ids, n * 16))
        if rc > 0:
            _put(out, reply)
        return rc

    def _remote_lookup_accounts(self, s, *a):
        return self._remote_lookup("lookup_accounts", s, *a)

    def _remote_lookup_transfers(self, s, *a):
        return self._remote_lookup("lookup_transfers", s, *a)

    def close(self):
        """Rank 0: ends every other rank's serve() and closes the group."""
        if self.rank == 0 and self.group is not None:
            for s in range(1, self.world):
                self._send([_END], np.zeros(0, np.uint8), s)
            self.group.close()
            self.group = None

    # -- ranks > 0: serving ---------------------------------------------------------------------

    def serve(self):
        """Executes rank 0's operations on this rank's executor until rank 0 ends the session."""
        L = self.local
        names = [name for name, _ in SIGS]
        while True:
            words, payload = self._recv(0)
            op = words[0]
            if op == _END:
                return
            name = names[op]
            rc, reply = self._execute(L, name, words[1:], payload)
            self._send([rc], reply, 0)

    @staticmethod
    def _execute(L, name, w, payload):
        P = payload.ctypes.data
        empty = np.zeros(0, np.uint8)
        if name in ("create_accounts", "create_transfers"):
            n, nb = w[0], w[1]
            out = np.zeros(n * 16, np.uint8)
            rc = L(name, P, n, P + n * 128, P + n * 128 + nb * 4, nb, out.ctypes.data)
            return rc, out
        if name in ("create_accounts_stamped", "create_transfers_stamped"):
            n, bts, opt = w[0], w[1], w[2]
            out = np.zeros(n * 16, np.uint8)
            rc = L(name, P, n, P + n * 128, bts, opt, out.ctypes.data)
            return rc, out
        if name == "forget_orphans":
            return L(name, P, w[0]), empty
        if name == "timestamps_exist":
            out = np.zeros(w[1], np.uint8)
            return L(name, w[0], P, w[1], out.ctypes.data), out
        if name == "key_max":
            v = np.zeros(2, np.uint64)
            rc = L(name, v.ctypes.data, v.ctypes.data + 8)
            return rc, v.view(np.uint8)
        if name == "raise_key_max":
            return L(name, w[0], w[1]), empty
        if name == "set_pnt_sharded":
            return L(name, w[0]), empty
        if name == "pnt_ops":
            copy, mx = w[0], w[1]
            start = np.zeros(1, np.uint64)
            if not copy:
                return L(name, None, None, 0, start.ctypes.data), start.view(np.uint8)
            ts = np.zeros(max(mx, 1), np.uint64)
            ops = np.zeros(max(mx, 1), np.uint64)
            rc = L(name, ts.ctypes.data, ops.ctypes.data, mx, start.ctypes.data)
            m = max(min(rc, mx), 0)
            return rc, np.concatenate([start, ts[:m], ops[:m]]).view(np.uint8)
        if name == "pulse_next_timestamp":
            return 0, np.asarray([L(name)], np.uint64).view(np.uint8)
        if name == "set_pulse_next_timestamp":
            return L(name, w[0]), empty
        if name == "pulse_candidates":
            ts, mx = w[0], w[1]
            e = np.zeros(max(mx, 1), np.uint64)
            t = np.zeros(max(mx, 1), np.uint64)
            rc = L(name, ts, e.ctypes.data, t.ctypes.data, mx)
            m = max(min(rc, mx), 0)
            return rc, np.concatenate([e[:m], t[:m]]).view(np.uint8)
        if name == "pulse_cut":
            ts, ce, ct, pnt, has = w[0], w[1], w[2], w[3], w[4]
            return L(name, ts, ce, ct, pnt, P if has and len(payload) else None), empty
        if name in ("lookup_accounts", "lookup_transfers"):
            n = w[0]
            out = np.zeros(max(n, 1) * 128, np.uint8)
            rc = L(name, P, n, out.ctypes.data)
            return rc, out[:max(rc, 0) * 128]
        raise ValueError(name)
