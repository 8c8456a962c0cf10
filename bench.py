#!/usr/bin/env python3
"""bench.py -- validated create_transfers/s on MI355X (BASELINE.json metric), config 2 workload.

Workload (BASELINE.json configs[1]): 10,000 accounts (ledger 2, code 1, history)
and 10,000,000 uniform create_transfers in 8189-event batches (1,221 x 8189 + 1,231), sequential
ids, `amount = Exp(10_000) +| 1`, seed 42. A *step* is one pass of the hot path over that whole
synthetic input: one tbg_create_transfers_device call carrying all 1,222 batches (each batch with
its own commit timestamp, TestContext rule prepare_ts += 1 + n). Inputs are resident in HBM when
the timed region starts; every step uses fresh transfer ids, so every step does the full work.

Multi-GPU (weak scaling, SURVEY.md §8e, north_star "the account table and event stream shard
naturally by ledger"): the line at N > 1 is the executor group (include/tbg_group.h): ONE process
-- rank 0 of the launch -- owns every GPU's shard, as the reference's one replica owns its one
StateMachine; the other ranks wait at the barriers. Each step is ONE mixed-ledger client call of
--group-transfers x N transfers (ledger uniform per event over N ledgers, 10k accounts each)
resident in HBM on GPU 0: the device router places every event, the slices are peer-copied over
xGMI to their shards' GPUs, every shard executes on its own host thread, the results come back
and settle in call order -- all inside the timed region (`group`). The pre-partitioned figure
(one process per GPU, each executing its ledger's batches of one client stream from its own HBM,
no data-path collective) is reported beside it (`partitioned`; `--partitioned-line` makes it the
line). Timed regions are bracketed by a barrier + device synchronise on every rank; the reported
time is the max over ranks. At N = 1 `hazard_call` times 1M-event calls with 0.1 % injected
failures across ledgers (unknown / cross-ledger accounts, id 0, reserved flags, posts of pending
transfers found nowhere, exact repeats) through a group of 2 shards on the one GPU: the device
path keeps them, validated in closed form. `--group S` makes a group of S shards on one GPU the
line (a rehearsal).

Validation (after the timed region; the workload is order-independent, so the serial reference
outcome is known in closed form): every result of every step is `created` with its exact event
timestamp; every transfer row (config 2: all of them, looked up by id; config 5: a sample) equals
the event with its commit timestamp; every account row equals the created account with the exact
per-account sums as posted balances and zero pending balances (config 5: a sample).

`per_commit`: the rate the drop-in sees per replica commit (state_machine.zig:2564-2669): one
8189-event body per commit (tigerbeetle.zig:853-901) -- through tbg_create_transfers_device with the
body resident in HBM, and through the full StateMachine boundary (tb_sm_prepare / prefetch /
commit on host buffers, tb_state_machine.h).

Output: one JSON line on rank 0 with `roofline` (dominant kernel, HIP-event timed, SURVEY.md §8d
algorithmic bytes) and `cpu_baseline` (the serial C oracle pinned to one host core, bounded sample
of the same workload).
"""
import argparse
import ctypes
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from tigerbeetle_amd import native, workload  # noqa: E402
from tigerbeetle_amd.types import ACCOUNT_DTYPE, RESULT_DTYPE, TRANSFER_DTYPE  # noqa: E402

METRIC = "validated create_transfers/sec (1/2/4/8 GPU) + % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
# Measured HBM bytes per launch of each kernel (tools/pmc.sh: separate rocprofv3 --pmc passes of
# this bench's default workload; FETCH_SIZE doubled per the gfx950 note + WRITE_SIZE).
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")  # config 2 (the default workload)
TRAFFIC_FILE_CONFIG5 = os.path.join(ROOT, "profiles", "traffic_config5.json")
BATCH = 8189           # Operation.create_transfers.event_max (src/tigerbeetle.zig:853-901)
CREATED = 0xFFFFFFFF
MESSAGE_BODY_SIZE_MAX = (1 << 20) - 256  # constants.message_body_size_max (constants.zig:234)
OP_CREATE_ACCOUNTS, OP_CREATE_TRANSFERS = 146, 147  # tb_state_machine.h

# Algorithmic bytes per event of each kernel of the create_transfers path. tr_ingest does all of
# SURVEY.md §8d's per-event work -- event read 128, result write 16, transfer-row write 128, id-key
# probe 16 = 288 B; the per-account 256 B (row read + write) belong to the balance kernels, which
# are priced per distinct account (`path` below), not per event.
KERNEL_BYTES_PER_EVENT = {"tr_ingest": 128 + 16 + 128 + 16}


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["config2", "config5"], default="config2",
                    help="config2 (default, the metric's workload) or config5 (many accounts over "
                         "64 ledgers sharded by ledger)")
    ap.add_argument("--transfers", type=int, default=None,
                    help="events per step (config2: 10M, config5: 1M super-batch)")
    ap.add_argument("--accounts", type=int, default=None,
                    help="accounts per GPU (config2: 10k, config5: 125M = 1B / 8)")
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--amounts", choices=["exp", "wide"], default="exp",
                    help="config2 amounts: exp = Exp(10k) +| 1 (benchmark_load.zig); wide = "
                         "log-uniform over [1, 2^63) (every result still created)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="bounded CPU-oracle sample (rank 0, N=1)")
    ap.add_argument("--no-account-events-line", action="store_true",
                    help="skip the with_account_events measurement")
    ap.add_argument("--commit-reps", type=int, default=200,
                    help="8189-event commits timed for `per_commit` (0: skip)")
    ap.add_argument("--account-events", action="store_true",
                    help="record AccountEvents (the account_events groove, 256 B per created "
                         "transfer) inside the timed steps; SURVEY.md §8d excludes them from the "
                         "headline's algorithmic bytes")
    ap.add_argument("--group-transfers", type=int, default=2_000_000,
                    help="group line: transfers per shard per step (one call of this x shards)")
    ap.add_argument("--partitioned-line", action="store_true",
                    help="N > 1: the line is the pre-partitioned figure (N independent executors, "
                         "each with its ledger's batches resident in its HBM) instead of the group")
    ap.add_argument("--group", type=int, default=0,
                    help="single process: the line is the group of this many shards on GPU "
                         "--group-device (a rehearsal of the N-GPU group on one GPU)")
    ap.add_argument("--group-device", type=int, default=0)
    ap.add_argument("--hazard-rate", type=float, default=0.001,
                    help="`hazard_call`: injected failures per event (N=1 line, 2 shards, 1 GPU)")
    ap.add_argument("--no-hazard-call", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-validate", action="store_true")
    return ap.parse_args()


def dist_init(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as td
        # TBG_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (host staging, no RCCL).
        backend = os.environ.get("TBG_BENCH_BACKEND") or (
            "nccl" if torch.cuda.is_available() else "gloo")
        if torch.cuda.is_available():
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
        td.init_process_group(backend=backend)
        dist = td
    return world, rank, local, dist


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, x: float) -> float:
    if dist is None:
        return x
    import torch
    dev = "cuda" if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class Device:
    """Device buffers via the HIP runtime (the product library already links it)."""

    def __init__(self):
        self.hip = ctypes.CDLL("libamdhip64.so")
        self.hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        self.hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                       ctypes.c_int]
        self.hip.hipFree.argtypes = [ctypes.c_void_p]
        self.hip.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
        self.hip.hipDeviceSynchronize.argtypes = []
        self.hip.hipSetDevice.argtypes = [ctypes.c_int]
        self.ptrs = []

    def set_device(self, d):
        assert self.hip.hipSetDevice(d) == 0

    def upload(self, a: np.ndarray) -> ctypes.c_void_p:
        p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(p), max(a.nbytes, 16)) == 0, "hipMalloc"
        assert self.hip.hipMemcpy(p, a.ctypes.data_as(ctypes.c_void_p), a.nbytes, 1) == 0
        self.ptrs.append(p)
        return p

    def alloc(self, nbytes) -> ctypes.c_void_p:
        p = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(p), max(nbytes, 16)) == 0, "hipMalloc"
        # (touched once before any timed region: a page's first write is not the path's cost)
        assert self.hip.hipMemset(p, 0, max(nbytes, 16)) == 0, "hipMemset"
        self.ptrs.append(p)
        return p

    def download(self, p, a: np.ndarray):
        assert self.hip.hipMemcpy(a.ctypes.data_as(ctypes.c_void_p), p, a.nbytes, 2) == 0

    def sync(self):
        assert self.hip.hipDeviceSynchronize() == 0

    def free_all(self):
        for p in self.ptrs:
            self.hip.hipFree(p)
        self.ptrs = []


def u128_sums(idx, amt, n_out, reps):
    """Exact u128 sums of u64 amounts by index, times reps: (n_out, 2) u64 [lo, hi] words (the
    32-bit halves summed apart, so no u64 sum wraps for amounts up to 2^64 over < 2^32 events)."""
    lo = np.zeros(n_out, dtype=np.uint64)
    hi = np.zeros(n_out, dtype=np.uint64)
    np.add.at(lo, idx, amt & np.uint64(0xFFFFFFFF))
    np.add.at(hi, idx, amt >> np.uint64(32))
    out = np.zeros((n_out, 2), dtype=np.uint64)
    for i, (a, b) in enumerate(zip(lo.tolist(), hi.tolist())):
        v = (a + (b << 32)) * reps
        out[i] = (v & 0xFFFFFFFFFFFFFFFF, v >> 64)
    return out


def batch_plan(n):
    lens = [BATCH] * (n // BATCH) + ([n % BATCH] if n % BATCH else [])
    return np.asarray(lens, dtype=np.int64)


def step_timestamps(prepare_ts, lens):
    """TestContext rule per commit: prepare_ts += 1 + n; the batch's timestamp is prepare_ts."""
    ts = prepare_ts + np.cumsum(lens + 1)
    return ts.astype(np.uint64), int(ts[-1])


def global_step_timestamps(prepare_ts, lens, world, rank):
    """The client stream of one step holds world x len(lens) batches, global batch g = j * world
    + r being shard r's j-th batch (all shards have the same `lens`). TestContext rule over the
    whole stream: prepare_ts += 1 + len per batch. Returns (shard `rank`'s batch timestamps, the
    prepare_ts after the whole stream)."""
    per = np.repeat(np.asarray(lens, dtype=np.int64) + 1, world)
    cum = prepare_ts + np.cumsum(per)
    return cum[rank::world].astype(np.uint64), int(cum[-1])


def event_timestamps(lens, batch_ts):
    """Event i of batch b is stamped batch_ts[b] - len[b] + i + 1 (execute_multi_batch)."""
    lens = np.asarray(lens, dtype=np.int64)
    starts = np.cumsum(lens) - lens
    n = int(lens.sum())
    within = np.arange(n, dtype=np.int64) - np.repeat(starts, lens)
    return (np.repeat(batch_ts.astype(np.uint64) - lens.astype(np.uint64), lens)
            + within.astype(np.uint64) + np.uint64(1))


def measured_traffic(kernel, path=TRAFFIC_FILE):
    """(HBM bytes per launch, source) of `kernel` from a tools/pmc.sh summary, or (None, None)."""
    try:
        with open(path) as fh:
            d = json.load(fh)
        return float(d["kernels"][kernel]["hbm_bytes_per_launch"]), d.get("source")
    except (OSError, ValueError, KeyError, TypeError):
        return None, None


def cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(args, acc, base, lens, label):
    """The serial C oracle (oracle/liboracle.so) pinned to one host core (the equivalent of
    `taskset -c <core>`: sched_setaffinity of this process), bounded sample of the workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_binding
    olib = oracle_binding.load()
    allowed = sorted(os.sched_getaffinity(0))
    core = allowed[0]
    os.sched_setaffinity(0, {core})
    try:
        o = olib.tbo_open(8190, 1)
        res = np.zeros(len(acc), dtype=RESULT_DTYPE)
        olib.tbo_create_accounts(o, acc.ctypes.data_as(ctypes.c_void_p), len(acc), 1 + len(acc),
                                 res.ctypes.data_as(ctypes.c_void_p))
        ts = 2 + len(acc)
        out = np.zeros(BATCH, dtype=RESULT_DTYPE)
        done, off, b = 0, 0, 0
        t0 = time.perf_counter()
        while b < len(lens):
            n = int(lens[b])
            ts += 1 + n
            olib.tbo_create_transfers(o, base[off:off + n].ctypes.data_as(ctypes.c_void_p), n, ts,
                                      out.ctypes.data_as(ctypes.c_void_p))
            assert (out["status"][:n] == CREATED).all()
            done += n
            off += n
            b += 1
            if time.perf_counter() - t0 >= args.cpu_seconds:
                break
        elapsed = time.perf_counter() - t0
        olib.tbo_close(o)
    finally:
        os.sched_setaffinity(0, set(allowed))
    return {"value": round(done / elapsed, 1), "unit": "transfers/s", "cores": 1, "kind": "port",
            "cpu_model": cpu_model(), "nproc": os.cpu_count(), "cpus_allowed": len(allowed),
            "pinned_cpu": core,
            "sample": f"{done} of the {len(base)} {label} transfers ({b} batches of <= {BATCH}) "
                      f"through oracle/tb_oracle.c, single-threaded, pinned to cpu {core} "
                      f"(sched_setaffinity = taskset -c {core}), {elapsed:.1f} s"}


def lookup_transfer_rows(lib, g, ids_lo, chunk):
    """Rows of the transfers with ids (lo words, hi 0), in request order, via tbg_lookup."""
    out = np.zeros(len(ids_lo), dtype=TRANSFER_DTYPE)
    ids = np.zeros((chunk, 2), dtype=np.uint64)
    for a in range(0, len(ids_lo), chunk):
        z = min(len(ids_lo), a + chunk)
        ids[:z - a, 0] = ids_lo[a:z]
        got = lib.tbg_lookup_transfers(g, ids.ctypes.data_as(ctypes.c_void_p), z - a,
                                       out[a:z].ctypes.data_as(ctypes.c_void_p))
        if got != z - a:
            return None
    return out


class Config2:
    """BASELINE.json configs[1]: 10k accounts (ledger 2 + rank), 10M uniform transfers per step."""
    name = "config2"

    def __init__(self, args, rank, world):
        self.N = args.transfers or 10_000_000
        self.A = args.accounts or 10_000
        self.ledger = 2 + rank
        # Shard r's accounts: ids r * A + 1 .. (r + 1) * A on ledger 2 + r; its transfers of a
        # step: ids r * N + 1 .. (r + 1) * N (+ step * N * world), accounts of its ledger.
        self.acc = workload.accounts(self.A, seed=args.seed + rank, id_offset=rank * self.A,
                                     ledger=self.ledger)
        self.base = workload.transfers_uniform(self.N, self.A, seed=args.seed + rank,
                                               id_offset=rank * self.N,
                                               account_id_offset=rank * self.A,
                                               ledger=self.ledger, amounts=args.amounts)
        self.dr = self.base["debit_account_id"][:, 0].astype(np.int64) - 1 - rank * self.A
        self.cr = self.base["credit_account_id"][:, 0].astype(np.int64) - 1 - rank * self.A
        self.chunk = self.A
        self.default = (self.N, self.A) == (10_000_000, 10_000)
        self.account_ts = None
        self.config = {"workload": "config2: 10k accounts, 10M uniform create_transfers in "
                                   "8189-event batches, 1 ledger shard per GPU"
                                   + ("" if world == 1 else
                                      f" (one client stream of {world} x 1222 batches, batch g "
                                      f"on ledger 2 + g mod {world})"),
                       "transfers_per_step_per_gpu": self.N, "accounts_per_gpu": self.A}
        if args.amounts != "exp":
            self.config["amounts"] = "log-uniform over [1, 2^63)"

    def account_chunks(self):
        yield self.acc

    def validate_accounts(self, lib, g, reps):
        """Every account row byte for byte: the created account with its creation timestamp and
        the exact per-account sums as posted balances (pending balances zero)."""
        dump = np.zeros(self.A, dtype=ACCOUNT_DTYPE)
        if lib.tbg_dump_accounts(g, dump.ctypes.data_as(ctypes.c_void_p)) != self.A:
            return False, "account count"
        amt = self.base["amount"][:, 0].astype(np.uint64)
        want = self.acc.copy()
        want["timestamp"] = self.account_ts
        # (exact integer sums: bincount's float64 weights would round past 2^53)
        for col, idx in (("debits_posted", self.dr), ("credits_posted", self.cr)):
            want[col] = u128_sums(idx, amt, self.A, reps)
        ok = dump.tobytes() == want.tobytes()
        return ok, "" if ok else "account rows differ"

    def rows_to_check(self):
        return np.arange(self.N)  # every transfer row

    def cpu_sample(self):
        return self.acc, self.base, "config-2"


class Config5:
    """BASELINE.json configs[4], per GPU: `accounts` accounts (default 1B / 8 = 125M, what each
    GPU holds at 8 GPUs) of the shard's 64 / G ledgers (account k on ledger 1 + k mod 64), one
    1M-event super-batch per step, ledger uniform then debit / credit uniform within it."""
    name = "config5"

    def __init__(self, args, rank, world):
        self.N = args.transfers or 1_000_000
        self.A = args.accounts or 125_000_000
        self.rank, self.world = rank, world
        self.base, self.dr, self.cr = workload.transfers_config5(self.N, self.A, rank, world,
                                                                 seed=args.seed,
                                                                 id_offset=rank * self.N)
        self.chunk = min(self.A, 4_000_000)
        self.default = False
        self.account_ts = None
        first, per = workload.config5_ledgers(rank, world)
        self.config = {"workload": f"config5: {self.A} accounts per GPU on {per} of 64 ledgers "
                                   f"(1B accounts over 8 GPUs), 1M-event super-batches of "
                                   f"8189-event batches, sharded by ledger",
                       "transfers_per_step_per_gpu": self.N, "accounts_per_gpu": self.A,
                       "ledgers_per_gpu": per}

    def account_chunks(self):
        for j0 in range(0, self.A, self.chunk):
            j = np.arange(j0, min(self.A, j0 + self.chunk), dtype=np.int64)
            yield workload.accounts_config5(j, self.rank, self.world)
            if j0 and (j0 // self.chunk) % 8 == 0:
                print(f"config5: {j0 + len(j)} accounts created", file=sys.stderr, flush=True)

    def validate_accounts(self, lib, g, reps):
        """Sampled (SURVEY.md §8d at 1B scale): 65,536 touched accounts and 4,096 others looked up
        by id; their balances must equal the exact sums of the steps' amounts."""
        rng = np.random.default_rng(5)
        touched = np.unique(np.concatenate([self.dr, self.cr]))
        sample = np.concatenate([rng.choice(touched, size=min(65_536, len(touched)), replace=False),
                                 rng.integers(0, self.A, size=4_096)])
        sample = np.unique(sample)
        amt = self.base["amount"][:, 0].astype(np.uint64)
        pos = np.full(self.A, -1, dtype=np.int64)
        pos[sample] = np.arange(len(sample))
        exp_d = np.zeros(len(sample), dtype=np.uint64)
        exp_c = np.zeros(len(sample), dtype=np.uint64)
        md, mc = pos[self.dr] >= 0, pos[self.cr] >= 0
        np.add.at(exp_d, pos[self.dr[md]], amt[md])
        np.add.at(exp_c, pos[self.cr[mc]], amt[mc])
        ids = np.zeros((len(sample), 2), dtype=np.uint64)
        ids[:, 0] = (workload.config5_global_index(sample, self.rank, self.world) + 1)
        out = np.zeros(len(sample), dtype=ACCOUNT_DTYPE)
        found = lib.tbg_lookup_accounts(g, ids.ctypes.data_as(ctypes.c_void_p), len(sample),
                                        out.ctypes.data_as(ctypes.c_void_p))
        want = workload.accounts_config5(sample, self.rank, self.world)
        ok = found == len(sample)
        for col in ("id", "user_data_128", "user_data_64", "user_data_32", "ledger", "code",
                    "flags", "debits_pending", "credits_pending"):
            ok = ok and bool((out[col] == want[col]).all())
        ok = ok and bool((out["debits_posted"][:, 0] == exp_d * np.uint64(reps)).all())
        ok = ok and bool((out["credits_posted"][:, 0] == exp_c * np.uint64(reps)).all())
        ok = ok and bool((out["debits_posted"][:, 1] == 0).all())
        ok = ok and bool((out["credits_posted"][:, 1] == 0).all())
        return ok, "" if ok else "sampled account rows differ"

    def rows_to_check(self):
        return np.sort(np.random.default_rng(6).choice(self.N, size=min(self.N, 65_536),
                                                       replace=False))

    def cpu_sample(self):
        """The oracle holds only the accounts the sampled transfers touch (its hash maps do not
        depend on the account count): the first 1M transfers of the stream."""
        n = min(self.N, 1_000_000)
        j = np.unique(np.concatenate([self.dr[:n], self.cr[:n]]))
        return workload.accounts_config5(j, self.rank, self.world), self.base[:n], "config-5"


def per_commit(args, lib, dev, g, wl, prepare_ts, id_base):
    """One 8189-event body per replica commit: (a) tbg_create_transfers_device with the body in
    HBM, (b) the full StateMachine boundary on host buffers (tb_sm_prepare / prefetch / commit).
    Returns (report, prepare_ts)."""
    R, n = args.commit_reps, min(BATCH, wl.N)
    body_events = wl.base[:n]
    lens1 = np.asarray([n], dtype=np.int64)
    d_end = dev.upload(np.asarray([n], dtype=np.uint32))
    bufs = []
    for r in range(R):
        ev = body_events.copy()
        ev["id"][:, 0] += np.uint64(id_base + r * n)
        ts, prepare_ts = step_timestamps(prepare_ts, lens1)
        bufs.append((dev.upload(ev), dev.upload(ts), dev.alloc(n * 16), ts))
    dev.sync()
    lat = np.zeros(R)
    t_all = time.perf_counter()
    for r in range(R):
        d_ev, d_ts, d_res, _ = bufs[r]
        t0 = time.perf_counter()
        rc = lib.tbg_create_transfers_device(g, d_ev, n, d_end, d_ts, 1, d_res, None)
        lat[r] = time.perf_counter() - t0
        if rc != 0:
            raise RuntimeError(f"per-commit: {rc} {lib.tbg_last_error(g)}")
    dev.sync()
    t_all = time.perf_counter() - t_all
    ok = True
    res = np.zeros(n, dtype=RESULT_DTYPE)
    for r, (d_ev, d_ts, d_res, ts) in enumerate(bufs):
        dev.download(d_res, res)
        want_ts = event_timestamps(lens1, ts)
        ok &= bool((res["status"] == CREATED).all() and (res["timestamp"] == want_ts).all())
        # the transfer rows, byte for byte
        want = body_events.copy()
        want["id"][:, 0] += np.uint64(id_base + r * n)
        want["timestamp"] = want_ts
        got = lookup_transfer_rows(lib, g, want["id"][:, 0], n)
        ok &= got is not None and got.tobytes() == want.tobytes()
    device = {"events_per_commit": n, "commits": R, "transfers_per_s": round(n * R / t_all, 1),
              "us_per_commit_mean": round(t_all / R * 1e6, 1),
              "us_per_commit_p50": round(float(np.median(lat)) * 1e6, 1),
              "us_per_commit_p90": round(float(np.percentile(lat, 90)) * 1e6, 1),
              "us_per_commit_max": round(float(lat.max()) * 1e6, 1),
              "validated": bool(ok),
              "validation": "every result (status and timestamp), every transfer row",
              "note": "tbg_create_transfers_device, the body resident in HBM, one synchronous "
                      "call per commit"}

    # (b) the StateMachine boundary: a second executor behind tb_sm (its own tables).
    sm_opt = native.SmOptions()
    sm_opt.batch_size_limit = MESSAGE_BODY_SIZE_MAX
    sm_opt.message_body_size_max = MESSAGE_BODY_SIZE_MAX
    sm_opt.pulse_batch_max = 8190
    topt = native.TbgOptions()
    topt.account_capacity = wl.A if wl.name == "config2" else 1 << 21
    topt.transfer_capacity = (R + 3) * n
    topt.batch_events_max = BATCH
    topt.batch_count_max = 64
    topt.pulse_batch_max = 8190
    topt.device = 0
    topt.pulse_next_timestamp_init = 1
    topt.account_events_capacity = (R + 3) * n  # the drop-in records AccountEvents (CDC)
    sm = lib.tb_sm_open_gpu(ctypes.byref(sm_opt), ctypes.byref(topt))
    if not sm:
        return {"device": device, "state_machine": None}, prepare_ts
    out = ctypes.create_string_buffer(MESSAGE_BODY_SIZE_MAX + 256)
    cb = native.PREFETCH_CALLBACK(lambda ctx: None)
    op_counter = [0]

    def encode(records):
        payload = records.tobytes()
        trailer = lib.tb_multi_batch_trailer_total_size(128, 1)
        buf = ctypes.create_string_buffer(len(payload) + trailer + 2)
        ctypes.memmove(buf, payload, len(payload))
        size = lib.tb_multi_batch_encode_trailer(buf, len(payload), 128,
                                                 (ctypes.c_uint16 * 1)(len(records)), 1)
        return buf.raw[:size]

    def commit(operation, body):
        # TestContext.prepare / execute (state_machine_tests.zig:230-285)
        lib.tb_sm_set_commit_timestamp(sm, lib.tb_sm_get_prepare_timestamp(sm))
        lib.tb_sm_set_prepare_timestamp(sm, lib.tb_sm_get_prepare_timestamp(sm) + 1)
        lib.tb_sm_prepare(sm, operation, body, len(body))
        ts = lib.tb_sm_get_prepare_timestamp(sm)
        lib.tb_sm_set_prefetch_timestamp(sm, ts)
        op_counter[0] += 1
        lib.tb_sm_prefetch(sm, cb, None, op_counter[0], op_counter[0], operation, body, len(body))
        size = lib.tb_sm_commit(sm, 1, 0, op_counter[0], ts, operation, body, len(body), out)
        if size < 0:
            raise RuntimeError(f"tb_sm_commit: {size}")
        return ctypes.string_at(out, size)

    if wl.name == "config2":
        accs = wl.acc
    else:
        j = np.unique(np.concatenate([wl.dr[:n], wl.cr[:n]]))
        accs = workload.accounts_config5(j, wl.rank, wl.world)
    sm_ok = True
    for a in range(0, len(accs), BATCH):
        reply = commit(OP_CREATE_ACCOUNTS, encode(accs[a:a + BATCH]))
        r = np.frombuffer(reply[:16 * len(accs[a:a + BATCH])], dtype=RESULT_DTYPE)
        sm_ok &= bool((r["status"] == CREATED).all())
    # The replica's message bodies live in its message pool, registered once with the executor
    # for direct DMA (tb_sm_register_buffer): one page-aligned pool holding every body here.
    first = encode(body_events)
    stride = (len(first) + 4095) // 4096 * 4096
    # (body 0: one untimed warmup commit; bodies 1 .. R timed)
    pool_raw = np.zeros((R + 1) * stride + 4096, dtype=np.uint8)
    off0 = (-pool_raw.ctypes.data) % 4096
    pool = pool_raw[off0:off0 + (R + 1) * stride]
    for r in range(R + 1):
        ev = body_events.copy()
        ev["id"][:, 0] += np.uint64(r * n + 1)
        b = encode(ev)
        pool[r * stride:r * stride + len(b)] = np.frombuffer(b, dtype=np.uint8)
    assert lib.tb_sm_register_buffer(sm, pool.ctypes.data, pool.nbytes) == 0
    # (and one reply buffer per commit, so nothing is copied out inside the timed loop)
    reply_stride = (16 * n + 256 + 4095) // 4096 * 4096
    replies_raw = np.zeros((R + 1) * reply_stride + 4096, dtype=np.uint8)
    off1 = (-replies_raw.ctypes.data) % 4096
    replies_pool = replies_raw[off1:off1 + (R + 1) * reply_stride]
    assert lib.tb_sm_register_buffer(sm, replies_pool.ctypes.data, replies_pool.nbytes) == 0
    body_size = len(first)

    no_cb = native.PREFETCH_CALLBACK()  # (a null function pointer)

    def commit_pooled(r):
        # (TestContext.prepare / execute as above; the prefetch callback is null: it completes
        # synchronously and the harness has nothing to resume, where a Python callback would add a
        # GIL round trip to every commit that a native replica does not pay)
        body = ctypes.c_void_p(pool.ctypes.data + r * stride)
        prepare_ts = lib.tb_sm_get_prepare_timestamp(sm)
        lib.tb_sm_set_commit_timestamp(sm, prepare_ts)
        lib.tb_sm_set_prepare_timestamp(sm, prepare_ts + 1)
        lib.tb_sm_prepare(sm, OP_CREATE_TRANSFERS, body, body_size)
        ts = lib.tb_sm_get_prepare_timestamp(sm)
        lib.tb_sm_set_prefetch_timestamp(sm, ts)
        op_counter[0] += 1
        lib.tb_sm_prefetch(sm, no_cb, None, op_counter[0], op_counter[0], OP_CREATE_TRANSFERS, body,
                           body_size)
        size = lib.tb_sm_commit(sm, 1, 0, op_counter[0], ts, OP_CREATE_TRANSFERS, body, body_size,
                                ctypes.c_void_p(replies_pool.ctypes.data + r * reply_stride))
        if size < 0:
            raise RuntimeError(f"tb_sm_commit: {size}")
        return ts

    lat_sm = np.zeros(R + 1)
    commit_ts = np.zeros(R + 1, dtype=np.uint64)
    commit_ts[0] = commit_pooled(0)  # warmup (untimed)
    lib.tbg_synchronize(lib.tb_sm_executor_gpu(sm))
    t_all = time.perf_counter()
    for r in range(1, R + 1):
        t0 = time.perf_counter()
        commit_ts[r] = commit_pooled(r)
        lat_sm[r] = time.perf_counter() - t0
    t_all = time.perf_counter() - t_all
    lat_sm = lat_sm[1:]
    replies = replies_pool.reshape(R + 1, reply_stride)[:, :16 * n]
    # Validation after timing: every reply (each event created at ts - n + i + 1), every transfer
    # row (the event as submitted, stamped), and every touched account's balances (the exact
    # sums over the R bodies).
    g_sm = lib.tb_sm_executor_gpu(sm)
    within = np.arange(n, dtype=np.uint64)
    ids = np.zeros((n, 2), dtype=np.uint64)
    rows = np.zeros(n, dtype=TRANSFER_DTYPE)
    for r in range(R + 1):
        res = replies[r].view(RESULT_DTYPE)
        want_ts = commit_ts[r] - np.uint64(n) + within + np.uint64(1)
        sm_ok &= bool((res["status"] == CREATED).all() and (res["timestamp"] == want_ts).all())
        ids[:, 0] = body_events["id"][:, 0] + np.uint64(r * n + 1)
        got = lib.tbg_lookup_transfers(g_sm, ids.ctypes.data_as(ctypes.c_void_p), n,
                                       rows.ctypes.data_as(ctypes.c_void_p))
        want = body_events.copy()
        want["id"][:, 0] = ids[:, 0]
        want["timestamp"] = want_ts
        sm_ok &= got == n and rows.tobytes() == want.tobytes()
    dr_i, cr_i = wl.dr[:n], wl.cr[:n]
    amt = body_events["amount"][:, 0].astype(np.uint64)
    touched = np.unique(np.concatenate([dr_i, cr_i]))
    pos = {int(a): i for i, a in enumerate(touched)}
    exp_d = u128_sums(np.fromiter((pos[int(x)] for x in dr_i), dtype=np.int64, count=n), amt,
                      len(touched), R + 1)
    exp_c = u128_sums(np.fromiter((pos[int(x)] for x in cr_i), dtype=np.int64, count=n), amt,
                      len(touched), R + 1)
    acc_ids = np.zeros((len(touched), 2), dtype=np.uint64)
    acc_ids[:, 0] = (wl.acc["id"][touched, 0] if wl.name == "config2" else
                     workload.config5_global_index(touched, wl.rank, wl.world) + 1)
    acc_rows = np.zeros(len(touched), dtype=ACCOUNT_DTYPE)
    for a in range(0, len(touched), BATCH):
        z = min(len(touched), a + BATCH)
        sm_ok &= lib.tbg_lookup_accounts(g_sm, acc_ids[a:z].ctypes.data_as(ctypes.c_void_p), z - a,
                                         acc_rows[a:z].ctypes.data_as(ctypes.c_void_p)) == z - a
    sm_ok &= bool((acc_rows["debits_posted"] == exp_d).all() and
                  (acc_rows["credits_posted"] == exp_c).all() and
                  (acc_rows["debits_pending"] == 0).all() and (acc_rows["credits_pending"] == 0).all())
    n_events = lib.tbg_dump_account_events(g_sm, None)
    sm_ok &= n_events == (R + 1) * n  # one AccountEvent per created transfer
    lib.tb_sm_close(sm)
    smr = {"events_per_commit": n, "commits": R, "transfers_per_s": round(n * R / t_all, 1),
           "us_per_commit_mean": round(t_all / R * 1e6, 1),
           "us_per_commit_p50": round(float(np.median(lat_sm)) * 1e6, 1),
           "us_per_commit_p90": round(float(np.percentile(lat_sm, 90)) * 1e6, 1),
           "us_per_commit_p99": round(float(np.percentile(lat_sm, 99)) * 1e6, 1),
           "us_per_commit_max": round(float(lat_sm.max()) * 1e6, 1),
           "body_bytes": body_size, "validated": bool(sm_ok),
           "validation": "every reply (status and timestamp), every transfer row byte for byte, "
                         "every touched account's balances, one AccountEvent per transfer",
           "note": "tb_sm_prepare + tb_sm_prefetch + tb_sm_commit per 8189-event multi-batch "
                   "body on host buffers (body in and reply out over PCIe; the bodies' pool and "
                   "the reply buffer registered once, tb_sm_register_buffer), AccountEvents "
                   "recorded"}
    return {"device": device, "state_machine": smr}, prepare_ts


def account_events_line(args, lib, dev, wl, steps, d_ends, lens, N, A):
    """Config 2's step with the AccountEvents groove recorded: a second executor, the same
    accounts and the first three steps' inputs (HBM-resident, their own ids and timestamps), one
    warmup + two timed steps. Validated: every result created, exactly one AccountEvent per
    transfer. (The AccountEvents' contents are pinned by the GPU parity tests.)"""
    opt = native.TbgOptions()
    opt.account_capacity = A
    opt.transfer_capacity = 3 * N
    opt.batch_events_max = max(N, wl.chunk)
    opt.batch_count_max = len(lens)
    opt.pulse_batch_max = 8190
    opt.device = 0
    opt.pulse_next_timestamp_init = 1
    opt.account_events_capacity = 3 * N
    g2 = lib.tbg_open(ctypes.byref(opt))
    if not g2:
        return None
    try:
        prepare_ts = 0
        for acc in wl.account_chunks():
            res = np.zeros(len(acc), dtype=RESULT_DTYPE)
            a_lens = np.asarray([len(acc)], dtype=np.uint32)
            a_ts, prepare_ts = global_step_timestamps(prepare_ts, [len(acc)], 1, 0)
            rc = lib.tbg_create_accounts(g2, acc.ctypes.data_as(ctypes.c_void_p), len(acc),
                                         a_lens.ctypes.data_as(native.c_u32p),
                                         a_ts.ctypes.data_as(native.c_u64p), 1,
                                         res.ctypes.data_as(ctypes.c_void_p))
            if rc != 0:
                return None

        def step(s):
            d_ev, d_ts, d_res, _ = steps[s]
            rc = lib.tbg_create_transfers_device(g2, d_ev, N, d_ends, d_ts, len(lens), d_res, None)
            if rc != 0:
                raise RuntimeError(f"with_account_events: {rc} {lib.tbg_last_error(g2)}")

        step(0)
        lib.tbg_profile(g2, 1)
        lib.tbg_synchronize(g2)
        t0 = time.perf_counter()
        step(1)
        step(2)
        lib.tbg_synchronize(g2)
        t = time.perf_counter() - t0
        kms = {}
        i = 0
        name = ctypes.create_string_buffer(64)
        ms, cnt = ctypes.c_double(), ctypes.c_uint64()
        while lib.tbg_profile_read(g2, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt)):
            kms[name.value.decode()] = round(ms.value / 2, 4)
            i += 1
        lib.tbg_profile(g2, 0)
        ok = True
        r = np.zeros(N, dtype=RESULT_DTYPE)
        for s in range(3):
            dev.download(steps[s][2], r)
            ok &= bool((r["status"] == CREATED).all())
        n_ae = lib.tbg_dump_account_events(g2, None)
        ok &= n_ae == 3 * N
        return {"value": round(2 * N / t, 1), "unit": "transfers/s", "steps": 2, "warmup": 1,
                "ms_per_step": round(t / 2 * 1e3, 3), "account_events_per_step": N,
                "account_events_ms_per_step": kms.get("account_events"),
                "kernels_ms_per_step": kms, "validated": bool(ok),
                "validation": "every result created; one AccountEvent per transfer (3 steps)",
                "note": "config 2's step with the account_events groove recorded (256-B "
                        "AccountEvent per created transfer), a second executor"}
    finally:
        lib.tbg_close(g2)


def group_measure(args, shards, devices, N1, K, W, hazard_rate=0.0):
    """The sharded group (include/tbg_group.h): ONE mixed-ledger client call per step -- N1 x shards
    transfers, the ledger uniform per event over `shards` ledgers (10k accounts each), sequential
    fresh ids -- enters in HBM on the router's GPU (devices[0]); tbg_group_create_transfers_device
    routes it (device router), copies each shard's slice to its GPU (peer copies over xGMI),
    executes every shard on its own host thread, copies the results back and settles them in call
    order -- all inside the timed region, K steps after W warmup steps. `hazard_rate` > 0 injects
    failures whose statuses follow from the events alone (workload.hazard_transfers: unknown and
    cross-ledger accounts, id 0, reserved flags, posts of pending transfers found nowhere, exact
    repeats), which the device path places. Validation: every result equals the closed form
    (workload.hazard_expected: created or the injected status, at the event's timestamp or the
    repeated object's) and every account row holds exactly the sums of its created transfers.
    Runs in this process only (the group owns every shard's GPU)."""
    from tigerbeetle_amd import shard
    P = args.accounts or 10_000
    L = shards
    N = N1 * shards
    lib = native.load()
    dev = Device()
    dev.set_device(devices[0])
    lens = batch_plan(N)
    per_shard = int(N1 * 1.1) + 8192
    opts = [native.options(P, per_shard * (K + W), per_shard, batch_count_max=len(lens),
                           device=d, pulse_next_timestamp_init=1) for d in devices]
    g = shard.Group.open_gpu(opts, ledgers=L + 1, events_max=N, batch_count_max=len(lens),
                             router_device=devices[0], router_account_capacity=P * L + 4096,
                             router_transfer_capacity=N * (K + W) + 4096)
    try:
        acc = workload.group_accounts(L, P, seed=args.seed)
        prepare_ts = len(acc) + 1
        res = g.create_accounts(acc, [len(acc)], [prepare_ts])
        assert (res["status"] == CREATED).all(), "group create_accounts"
        d_ends = dev.upload(np.cumsum(lens).astype(np.uint32))
        # One generated call; step s is it with every nonzero id moved by s * N (fresh ids every
        # step; the injected repeats keep repeating, ids 0 stay 0)
        if hazard_rate > 0:
            base, kinds, src = workload.hazard_transfers(N, L, P, hazard_rate, seed=args.seed)
        else:
            base, _ = workload.mixed_ledger_transfers(N, L, P, seed=args.seed)
            kinds = np.full(N, -1, dtype=np.int64)
            src = kinds
        nonzero = (base["id"][:, 0] != 0) | (base["id"][:, 1] != 0)
        steps = []
        for s in range(W + K):
            t = base.copy()
            t["id"][nonzero, 0] += np.uint64(s * N)
            ts, prepare_ts = step_timestamps(prepare_ts, lens)
            steps.append((dev.upload(t), dev.upload(ts), dev.alloc(N * 16), ts))
            del t
        dev.sync()

        def run_step(s):
            d_ev, d_ts, d_res = steps[s][:3]
            g.create_transfers_device(d_ev.value, N, d_ends.value, d_ts.value, len(lens),
                                      d_res.value)

        for s in range(W):
            run_step(s)
        dev.sync()
        t0 = time.perf_counter()
        for s in range(W, W + K):
            run_step(s)
        dev.sync()
        t_wall = time.perf_counter() - t0
        st = g.stats()

        ok = st["device_calls"] == W + K and st["engine_calls"] == 1  # (the accounts call)
        r = np.zeros(N, dtype=RESULT_DTYPE)
        created = None
        for s in range(W + K):
            _, _, d_res, ts = steps[s]
            dev.download(d_res, r)
            want_st, want_ts, created = workload.hazard_expected(
                base, kinds, src, event_timestamps(lens, ts), L)
            ok &= bool((r["status"] == want_st).all() and (r["timestamp"] == want_ts).all() and
                       (r["reserved"] == 0).all())
        failed = int((~created).sum()) * (W + K)
        amt = base["amount"][created, 0]
        exp_d = np.zeros(L * P, dtype=np.uint64)
        exp_c = np.zeros(L * P, dtype=np.uint64)
        np.add.at(exp_d, base["debit_account_id"][created, 0].astype(np.int64) - 1, amt)
        np.add.at(exp_c, base["credit_account_id"][created, 0].astype(np.int64) - 1, amt)
        rows = g.lookup_accounts(np.arange(1, L * P + 1))
        ok &= len(rows) == L * P
        if ok:
            reps = np.uint64(W + K)
            ok &= bool((rows["debits_posted"][:, 0] == exp_d * reps).all() and
                       (rows["credits_posted"][:, 0] == exp_c * reps).all() and
                       (rows["debits_posted"][:, 1] == 0).all() and
                       (rows["debits_pending"] == 0).all() and (rows["credits_pending"] == 0).all())
        return {
            "value": round(N * K / t_wall, 1), "unit": "transfers/s", "steps": K, "warmup": W,
            "ms_per_step": round(t_wall / K * 1e3, 3), "validated": bool(ok),
            "shards": shards, "devices": list(devices), "transfers_per_step": N,
            "batches_per_step": int(len(lens)), "accounts_per_shard": P,
            "hazard_rate": hazard_rate, "injected_failures": failed,
            "group_stats": st,
            "workload": f"one mixed-ledger client call of {N1} transfers per shard per step over "
                        f"{shards} ledgers ({P} accounts each, ledger uniform per event)" +
                        (f", {hazard_rate:.2%} injected failures across ledgers"
                         if hazard_rate > 0 else "") +
                        f", entering in HBM on GPU {devices[0]}: device router + per-shard slices "
                        f"(peer copies) + execution on every shard + settle, all timed",
        }
    finally:
        g.close()
        dev.free_all()


def single_line(args, world, rank, local, dist):
    """The executor line: each rank's executor over its shard's batches of one client stream
    (module doc), config 2 or 5. Returns rank 0's line (None elsewhere)."""
    wl = (Config5 if args.workload == "config5" else Config2)(args, rank, world)
    N, A, K, W = wl.N, wl.A, args.steps, args.warmup
    R = args.commit_reps if rank == 0 and world == 1 and not args.no_validate else 0
    lib = native.load()
    dev = Device()
    dev.set_device(local)

    base = wl.base
    lens = batch_plan(N)
    ends = np.cumsum(lens).astype(np.uint32)

    opt = native.TbgOptions()
    opt.account_capacity = A
    # + two host-buffer steps (pcie_inclusive: pageable, registered) + the per-commit bodies
    opt.transfer_capacity = N * (K + W + 2) + R * BATCH
    opt.batch_events_max = max(N, wl.chunk)
    opt.batch_count_max = len(lens)
    opt.pulse_batch_max = 8190
    opt.device = local
    opt.pulse_next_timestamp_init = 1
    opt.account_events_capacity = N * (K + W + 1) + R * BATCH if args.account_events else 0
    g = lib.tbg_open(ctypes.byref(opt))
    assert g, "tbg_open failed"

    # Global timestamps: every create_accounts chunk and every step is one client stream of
    # `world` shards' batches, interleaved (global_step_timestamps).
    prepare_ts = 0
    acc_ts = []
    for acc in wl.account_chunks():
        res_acc = np.zeros(len(acc), dtype=RESULT_DTYPE)
        a_lens = np.asarray([len(acc)], dtype=np.uint32)
        a_ts, prepare_ts = global_step_timestamps(prepare_ts, [len(acc)], world, rank)
        rc = lib.tbg_create_accounts(g, acc.ctypes.data_as(ctypes.c_void_p), len(acc),
                                     a_lens.ctypes.data_as(native.c_u32p),
                                     a_ts.ctypes.data_as(native.c_u64p), 1,
                                     res_acc.ctypes.data_as(ctypes.c_void_p))
        assert rc == 0 and (res_acc["status"] == CREATED).all(), \
            f"create_accounts: {rc} {lib.tbg_last_error(g)}"
        if wl.name == "config2":
            acc_ts.append(event_timestamps(np.asarray([len(acc)]), a_ts))
        del acc, res_acc
    if acc_ts:
        wl.account_ts = np.concatenate(acc_ts)

    # Per-step inputs, resident in HBM before timing: fresh ids per step.
    d_ends = dev.upload(ends)
    steps = []
    for s in range(W + K):
        ev = base.copy()
        ev["id"][:, 0] += np.uint64(s * N * world)
        ts, prepare_ts = global_step_timestamps(prepare_ts, lens, world, rank)
        steps.append((dev.upload(ev), dev.upload(ts), dev.alloc(N * 16), ts))
        del ev
    dev.sync()

    def run_step(s):
        d_ev, d_ts, d_res, _ = steps[s]
        rc = lib.tbg_create_transfers_device(g, d_ev, N, d_ends, d_ts, len(lens), d_res, None)
        if rc != 0:
            raise RuntimeError(f"tbg_create_transfers_device: {rc} {lib.tbg_last_error(g)}")

    for s in range(W):
        run_step(s)
    lib.tbg_profile(g, 1)
    dev.sync()
    barrier(dist)
    dev.sync()
    t0 = time.perf_counter()
    for s in range(W, W + K):
        run_step(s)
    dev.sync()
    barrier(dist)
    t_local = time.perf_counter() - t0
    t_max = max_over_ranks(dist, t_local)

    # Kernel times (HIP events on the executor's stream over the timed steps).
    kernels = {}
    i = 0
    name = ctypes.create_string_buffer(64)
    ms, cnt = ctypes.c_double(), ctypes.c_uint64()
    while lib.tbg_profile_read(g, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt)):
        kernels[name.value.decode()] = (ms.value, cnt.value)
        i += 1
    lib.tbg_profile(g, 0)

    stats = native.TbgStats()
    lib.tbg_last_stats(g, ctypes.byref(stats))

    validated, validation = None, {}
    if not args.no_validate:
        t_val = time.perf_counter()
        ok = True
        r = np.zeros(N, dtype=RESULT_DTYPE)
        rows = wl.rows_to_check()
        for s in range(W + K):
            d_ev, d_ts, d_res, ts = steps[s]
            dev.download(d_res, r)
            want_ts = event_timestamps(lens, ts)
            ok &= bool((r["status"] == CREATED).all())
            ok &= bool((r["timestamp"] == want_ts).all() and (r["reserved"] == 0).all())
            # transfer rows: the event as submitted, stamped with its commit timestamp
            got = lookup_transfer_rows(lib, g, base["id"][rows, 0] + np.uint64(s * N * world),
                                       min(opt.batch_events_max, 1 << 21))
            if got is None:
                ok = False
                continue
            for a in range(0, len(rows), 1 << 21):
                sel = rows[a:a + (1 << 21)]
                want = base[sel].copy()
                want["id"][:, 0] += np.uint64(s * N * world)
                want["timestamp"] = want_ts[sel]
                ok &= got[a:a + len(sel)].tobytes() == want.tobytes()
        acc_ok, why = wl.validate_accounts(lib, g, W + K)
        ok &= acc_ok
        validated = bool(ok)
        validation = {"results": f"{W + K} steps x {N}: status and event timestamp",
                      "transfer_rows": f"{len(rows)} per step, byte for byte",
                      "accounts": "all rows byte for byte" if wl.name == "config2"
                                  else "sampled rows (balances exact)",
                      "seconds": round(time.perf_counter() - t_val, 1)}
        if not ok:
            print(json.dumps({"error": "validation failed", "why": why}), file=sys.stderr)

    # The same step through the host-buffer ABI (tbg_create_transfers: events copied in, results
    # copied out over PCIe) -- the rate a caller holding host buffers sees; never `value`.
    # Registered: the caller pins and maps its buffers once (tbg_register_host), as a replica
    # registers its message pool; pageable: plain host memory, staged by the runtime.
    pcie = None
    if not args.no_validate:
        h_lens = lens.astype(np.uint32)
        rates = {}
        for j, mode in enumerate(("pageable", "registered")):
            ev = base.copy()
            ev["id"][:, 0] += np.uint64((W + K + j) * N * world)
            ts, prepare_ts = global_step_timestamps(prepare_ts, lens, world, rank)
            h_res = np.zeros(N, dtype=RESULT_DTYPE)
            if mode == "registered":
                assert lib.tbg_register_host(g, ev.ctypes.data, ev.nbytes) == 0
                assert lib.tbg_register_host(g, h_res.ctypes.data, h_res.nbytes) == 0
            t0 = time.perf_counter()
            rc = lib.tbg_create_transfers(g, ev.ctypes.data_as(ctypes.c_void_p), N,
                                          h_lens.ctypes.data_as(native.c_u32p),
                                          ts.ctypes.data_as(native.c_u64p), len(lens),
                                          h_res.ctypes.data_as(ctypes.c_void_p))
            t_host = time.perf_counter() - t0
            if mode == "registered":
                lib.tbg_unregister_host(g, ev.ctypes.data)
                lib.tbg_unregister_host(g, h_res.ctypes.data)
            ok = rc == 0 and bool((h_res["status"] == CREATED).all())
            validated = bool(validated) and ok
            rates[mode] = (t_host, ok)
            del ev, h_res
        t_host = rates["registered"][0]
        t_page = rates["pageable"][0]
        pcie = {"value": round(N / t_host, 1), "unit": "transfers/s", "ms": round(t_host * 1e3, 3),
                "pcie_gb_per_s": round(N * 144 / t_host / 1e9, 1),
                "pageable": {"value": round(N / t_page, 1), "ms": round(t_page * 1e3, 3),
                             "pcie_gb_per_s": round(N * 144 / t_page / 1e9, 1)},
                "note": "one step through tbg_create_transfers with host buffers (events in, "
                        "results out over PCIe), registered once (tbg_register_host, as a "
                        "replica's message pool); `pageable`: unregistered host memory"}

    # The integrated drop-in records an AccountEvent for every created transfer
    # (state_machine.zig:4417, "For CDC we always insert the history"): the same steps on a second
    # executor with the account_events groove on (SURVEY.md §8d prices the 256-B AccountEvent
    # separately, so `value` above is the executor without it).
    with_ae = None
    if (rank == 0 and world == 1 and not args.no_validate and not args.account_events and
            wl.name == "config2" and W + K >= 3 and not args.no_account_events_line):
        with_ae = account_events_line(args, lib, dev, wl, steps, d_ends, lens, N, A)

    commits = None
    if R > 0:
        commits, prepare_ts = per_commit(args, lib, dev, g, wl, prepare_ts,
                                         (W + K + 2) * N * world)

    # Algorithmic bytes of the path: 288 B per event + 256 B per distinct account.
    distinct = len(np.union1d(wl.dr, wl.cr))
    path_bytes = 288 * N + 256 * distinct
    dev_ms_total = sum(v[0] for k, v in kernels.items() if k not in ("begin", "host_sync"))
    dom = max(((k, v) for k, v in kernels.items() if k in KERNEL_BYTES_PER_EVENT),
              key=lambda kv: kv[1][0], default=None)
    roofline = None
    if dom is not None:
        kname, (kms, kcount) = dom
        avg_s = kms / kcount / 1e3
        kbytes = KERNEL_BYTES_PER_EVENT[kname] * N
        # A sparse key space (config 5): tr_ingest also applies the balance deltas itself (u128
        # atomics on the accounts' rows; no bal_* kernel ran), so it does the path's per-account
        # work too: SURVEY.md §8d's 256 B per distinct account (row read + write).
        ingest_balances = kname == "tr_ingest" and not any(k.startswith("bal") for k in kernels)
        if ingest_balances:
            kbytes += 256 * distinct
        achieved = kbytes / avg_s / 1e9
        traffic, traffic_src = (measured_traffic(kname) if wl.default else
                                measured_traffic(kname, TRAFFIC_FILE_CONFIG5)
                                if wl.name == "config5" else (None, None))
        roofline = {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": traffic, "traffic_source": traffic_src,
                    "alg_bytes_per_launch": kbytes,
                    "alg_bytes_basis": "SURVEY.md §8d: 288 B per event (event 128 R, result 16 W, "
                                       "transfer row 128 W, id-key probe 16)" +
                                       (" + 256 B per distinct account (the kernel applies the "
                                        "balances: row read + write)" if ingest_balances else ""),
                    "avg_launch_ms": round(kms / kcount, 4),
                    "path": {"alg_bytes_per_step": path_bytes,
                             "alg_bytes_basis": "SURVEY.md §8d: 288 N + 256 D "
                                                f"(N = {N}, D = {distinct} distinct accounts)",
                             "device_ms_per_step": round(dev_ms_total / K, 4),
                             "achieved": round(path_bytes / (dev_ms_total / K / 1e3) / 1e9, 1),
                             "frac": round(path_bytes / (dev_ms_total / K / 1e3) / 1e9 /
                                           HBM_PEAK_GBS, 4),
                             "frac_wall": round(path_bytes / (t_max / K) / 1e9 / HBM_PEAK_GBS, 4)},
                    "kernels_ms_per_step": {k: round(v[0] / K, 4) for k, v in kernels.items()}}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        acc_s, base_s, label = wl.cpu_sample()
        cpu = cpu_baseline(args, acc_s, base_s, batch_plan(len(base_s)), label)

    if dist is not None and validated is not None:  # every shard validated its own partition
        validated = max_over_ranks(dist, 0.0 if validated else 1.0) == 0.0

    value = N * K * world / t_max
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "transfers/s",
            "n_gpus": world, "steps": K, "warmup": W,
            "ms_per_step": round(t_max / K * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u128",
            "data": "synthetic (seeded; benchmark_load.zig distributions, sequential ids)",
            "config": dict(wl.config, batches_per_step=int(len(lens)),
                           parallelism=f"ledger-shard x{world}",
                           account_events=bool(args.account_events)),
            "validated": validated,
            "validation": validation,
            "replayed_events_last_step": int(stats.replayed),
            "roofline": roofline,
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
            "per_commit": commits,
            "with_account_events": with_ae,
        }
    lib.tbg_close(g)
    dev.free_all()
    return line if rank == 0 else None


def group_line(args, grp, world, extra):
    """The JSON line whose `value` is the group's (group_measure)."""
    return {
        "metric": METRIC, "value": grp["value"], "unit": "transfers/s", "n_gpus": world,
        "steps": grp["steps"], "warmup": grp["warmup"], "ms_per_step": grp["ms_per_step"],
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u128",
        "data": "synthetic (seeded; benchmark_load.zig distributions, sequential ids)",
        "config": {"workload": "config2 over ledger shards: " + grp["workload"],
                   "transfers_per_step": grp["transfers_per_step"],
                   "accounts_per_shard": grp["accounts_per_shard"],
                   "batches_per_step": grp["batches_per_step"],
                   "parallelism": f"ledger-shard x{grp['shards']} (one process, devices "
                                  f"{grp['devices']}; tbg_group_create_transfers_device)"},
        "validated": grp["validated"], "group": grp, **extra}


def main():
    args = parse_args()
    world, rank, local, dist = dist_init(args)
    K, W = args.steps, args.warmup
    if args.group:
        grp = group_measure(args, args.group, [args.group_device] * args.group,
                            args.group_transfers, K, W)
        print(json.dumps(group_line(args, grp, 1, {"roofline": None, "cpu_baseline": None})))
        return
    line = single_line(args, world, rank, local, dist)
    if world == 1 and not args.no_hazard_call and not args.no_validate and \
            args.workload == "config2":
        # 1M-event calls with injected failures across ledgers over 2 shards on this GPU: the
        # device path keeps them (tbg_group.h), validated in closed form
        line["hazard_call"] = group_measure(args, 2, [local, local], 500_000, 5, 1,
                                            hazard_rate=args.hazard_rate)
    if world > 1 and not args.partitioned_line:
        # The N-GPU line: rank 0 owns every shard's GPU through the group; the other ranks wait.
        import torch
        barrier(dist)
        grp = None
        if rank == 0:
            n_dev = torch.cuda.device_count()
            grp = group_measure(args, world, [s % n_dev for s in range(world)],
                                args.group_transfers, K, W)
        barrier(dist)
        if rank == 0:
            part = {k: line[k] for k in ("value", "ms_per_step", "validated", "config")}
            part["note"] = ("N independent executors, each with its ledger's batches of one "
                            "client stream resident in its HBM (no data-path collective)")
            line = group_line(args, grp, world, {"roofline": line["roofline"],
                                                 "roofline_source": "the partitioned run's "
                                                                    "executor kernels",
                                                 "cpu_baseline": None, "partitioned": part})
    if rank == 0:
        print(json.dumps(line))
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
