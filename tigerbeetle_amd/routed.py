"""The routed data path across ledger shards, one process per GPU (north_star:
"RCCL over xGMI is used only to scatter batches and gather results").

A client call enters at rank 0 with its events resident in HBM. The device router (include/tbr.h)
assigns every event to the shard holding its ledger's accounts and scatters the call into
per-shard slices that keep each event's global commit timestamp; rank 0 sends every other shard
its slice (event bytes and timestamps: point-to-point sends, RCCL over xGMI under the `nccl`
backend), every rank executes its slice with tbg_create_transfers_stamped_device, the 16-byte
results come back, and rank 0 puts them in call order (tbr_settle_device, which also records the
ids that now exist on their shards).

The device router places single events, resubmitted ids (on their holder), post/voids (on
their pending transfer's shard) and linked chains that stay on one shard (include/tbr.h). A call
it cannot place -- any event that could observe another shard's state (imported events, ids that
repeat within the call, accounts unknown or on two shards, chains across shards) -- is executed
by the exact host engine instead (shard.Engine over the same directories, through
shard.ShardGroup): surrogates for cross-shard transfers, segments, the chain protocol for linked
chains across shards, key-range sync for imported batches -- every call executes exactly.

Imported calls take the device path when every event is imported, their timestamps increase and
lie above the imported floor -- the largest timestamp of any object on any shard, kept by rank 0
(the shards' key maxima after every host-path call, raised by each routed call's created
timestamps; tbr_set_imported_floor).

A routed call that posts or voids (the router's mode 2) resolves pulse_next_timestamp across the
shards after it (shard.ShardGroup.resolve_pnt: every shard's recorded updates gathered at rank 0,
replayed in call order, the outcome broadcast): a post/void of a pending transfer with a timeout
resets it against the value over all shards (post_or_void_pending_transfer :4227-4229).
"""
import ctypes

import numpy as np

from . import native
from .shard import DeviceDirectory, GpuShard, LedgerRouter, ShardGroup
from .types import RESULT_DTYPE, TRANSFER_DTYPE


class RoutedShards:
    """This rank's shard executor plus, on rank 0, the device router. Collective: rank 0 passes
    the call, the other ranks call with no arguments."""

    def __init__(self, executor_options: "native.TbgOptions", events_max: int,
                 router_transfer_capacity: int, router_account_capacity: int, ledgers: int = 64,
                 device_index: int = 0, group=None):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.nccl = dist.get_backend(group) == "nccl"
        self.dev = torch.device("cuda", device_index)
        self.lib = native.load()
        self.g = self.lib.tbg_open(ctypes.byref(executor_options))
        if not self.g:
            raise RuntimeError("tbg_open failed")
        self.shard = GpuShard.wrap(self.lib, self.g)
        self.tbr = None
        router = None
        if self.rank == 0:
            self.tbr = self.lib.tbr_open(self.world, router_account_capacity,
                                         router_transfer_capacity, events_max, device_index)
            if not self.tbr:
                raise RuntimeError("tbr_open failed")
            router = LedgerRouter(self.world, ledgers, DeviceDirectory(self.lib, self.tbr))
        self.router = router
        self.host = ShardGroup(self.shard, router, group=group,
                               device="cuda" if self.nccl else "cpu")
        u8 = torch.uint8
        self.ev = torch.empty(events_max * 128, dtype=u8, device=self.dev)   # slices
        self.ts = torch.empty(events_max, dtype=torch.int64, device=self.dev)
        self.res = torch.empty(events_max * 16, dtype=u8, device=self.dev)   # shard-order results
        self.pos = torch.empty(events_max, dtype=torch.int32, device=self.dev) if self.rank == 0 \
            else None
        self.fast_calls = 0
        self.host_calls = 0
        self.floor = None  # the imported floor (rank 0; None: unknown until a host-path call)

    def close(self):
        if self.tbr:
            self.lib.tbr_close(self.tbr)
            self.tbr = None
        if self.g:
            self.lib.tbg_close(self.g)
            self.g = None

    # -- transport: device tensors under nccl, host staging under gloo ----------------------------

    def _peer(self, r):
        return r if self.group is None else self.dist.get_global_rank(self.group, r)

    def _isend(self, t, dst):
        if self.nccl:
            return self.dist.isend(t, self._peer(dst), group=self.group)
        self.dist.send(t.cpu(), self._peer(dst), group=self.group)
        return None

    def _recv(self, t, src):
        if self.nccl:
            self.dist.recv(t, self._peer(src), group=self.group)
        else:
            h = torch_empty_like_cpu(self.torch, t)
            self.dist.recv(h, self._peer(src), group=self.group)
            t.copy_(h)

    def _bcast(self, words):
        t = self.torch.tensor(words, dtype=self.torch.int64,
                              device=self.dev if self.nccl else "cpu")
        self.dist.broadcast(t, self._peer(0), group=self.group)
        return [int(x) for x in t.tolist()]

    # -- calls --------------------------------------------------------------------------------------

    def _set_floor(self, floor):
        if self.rank == 0:
            self.floor = floor
            rc = self.lib.tbr_set_imported_floor(self.tbr, (1 << 64) - 1 if floor is None
                                                 else int(floor))
            if rc != 0:
                raise RuntimeError(f"tbr_set_imported_floor: {rc}")

    def _refresh_floor(self):
        """Collective: the key maxima over all shards (raised on every shard) as the floor."""
        a, t = self.host.sync_key_max_collective()
        self._set_floor(max(a, t))

    def record_accounts(self, ids: np.ndarray, shards: np.ndarray):
        """Rank 0: accounts that already exist on their shards (created there directly; the
        imported floor is unknown until the next host-path call)."""
        self._set_floor(None)
        rc = self.lib.tbr_record_accounts(self.tbr, np.ascontiguousarray(ids).ctypes.data_as(
            ctypes.c_void_p), np.ascontiguousarray(shards, dtype=np.uint8).ctypes.data_as(
            ctypes.c_void_p), len(ids))
        if rc != 0:
            raise RuntimeError(f"tbr_record_accounts: {rc}")

    def create_transfers(self, d_events=0, n=0, d_batch_ends=0, d_batch_ts=0, n_batches=0,
                         d_results=0, host_call=None):
        """Rank 0: the call's device pointers (and `host_call` = (events, lens, batch_ts) on the
        host, for a call the device router hands to the exact host router). Returns the mode:
        0 device fast path, 1 host router."""
        W = self.world
        if self.rank == 0:
            counts = (ctypes.c_uint32 * W)()
            rc = self.lib.tbr_route_device(self.tbr, d_events, n, d_batch_ends, d_batch_ts,
                                           n_batches, self.ev.data_ptr(), self.ts.data_ptr(),
                                           self.pos.data_ptr(), counts)
            if rc < 0:
                raise RuntimeError(f"tbr_route_device: {rc}")
            words = [int(rc)] + [int(c) for c in counts]
        else:
            words = [0] * (W + 1)
        words = self._bcast(words)
        mode, counts = words[0], words[1:]
        resolve = mode == 2
        if mode == 2:
            mode = 0
        if mode == 1:
            self.host_calls += 1
            if self.rank == 0:
                if host_call is None:
                    raise RuntimeError("the call needs the host router: pass host_call")
                events, lens, batch_ts = host_call
                res = self.host.create_transfers(events, lens, batch_ts)
                self.torch.cuda.synchronize(self.dev)
                buf = self.torch.from_numpy(res.view(np.uint8).copy()).to(self.dev)
                self._copy_to_ptr(buf, d_results)
            else:
                self.host.create_transfers()
            self._refresh_floor()
            return 1
        self.fast_calls += 1
        offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        mine = counts[self.rank]
        if self.rank == 0:
            reqs = []
            for s in range(1, W):
                a, c = int(offs[s]), counts[s]
                if c:
                    reqs.append(self._isend(self.ev[a * 128:(a + c) * 128], s))
                    reqs.append(self._isend(self.ts[a:a + c], s))
            self._execute(self.ev, self.ts, self.res, mine)
            for s in range(1, W):
                a, c = int(offs[s]), counts[s]
                if c:
                    self._recv(self.res[a * 16:(a + c) * 16], s)
            for r in reqs:
                if r is not None:
                    r.wait()
            self.torch.cuda.synchronize(self.dev)
            km = ctypes.c_uint64(0)
            rc = self.lib.tbr_settle_device(self.tbr, self.res.data_ptr(), self.pos.data_ptr(), n,
                                            d_results, ctypes.byref(km))
            if rc != 0:
                raise RuntimeError(f"tbr_settle_device: {rc}")
            if self.floor is not None:
                self._set_floor(max(self.floor, km.value))
        else:
            if mine:
                self._recv(self.ev[:mine * 128], 0)
                self._recv(self.ts[:mine], 0)
                self.torch.cuda.synchronize(self.dev)
                self._execute(self.ev, self.ts, self.res, mine)
                r = self._isend(self.res[:mine * 16], 0)
                if r is not None:
                    r.wait()
        if resolve:
            self.host.resolve_pnt(executed=mine > 0)
        return 0

    def _execute(self, ev, ts, res, n):
        if n == 0:
            return
        self.torch.cuda.synchronize(self.dev)
        rc = self.lib.tbg_create_transfers_stamped_device(self.g, ev.data_ptr(), n, ts.data_ptr(),
                                                          res.data_ptr(), None)
        if rc == 0:
            # The executor may leave work queued behind the call on its own stream (the
            # AccountEvents appends read the call's events and results): the next call's receive
            # into `ev` / `res` runs on torch's stream, so wait for it here.
            rc = self.lib.tbg_synchronize(self.g)
        if rc != 0:
            raise RuntimeError(f"tbg_create_transfers_stamped_device: {rc} "
                               f"{self.lib.tbg_last_error(self.g)}")

    def _copy_to_ptr(self, src, dst_ptr):
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        if hip.hipMemcpy(ctypes.c_void_p(dst_ptr), ctypes.c_void_p(src.data_ptr()),
                         src.numel(), 3) != 0:
            raise RuntimeError("hipMemcpy")

    # pulses and host-router calls go through the host group (collective)
    def create_accounts(self, events=None, lens=None, batch_ts=None):
        res = self.host.create_accounts(events, lens, batch_ts)
        self._refresh_floor()
        return res

    def pulse_next_timestamp(self):
        return self.host.pulse_next_timestamp()

    def pulse(self, timestamp):
        return self.host.pulse(timestamp)


def torch_empty_like_cpu(torch, t):
    return torch.empty(t.shape, dtype=t.dtype, device="cpu")


__all__ = ["RoutedShards", "RESULT_DTYPE", "TRANSFER_DTYPE"]
