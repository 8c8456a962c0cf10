#!/usr/bin/env python3
"""bench.py -- validated create_transfers/s on MI355X (BASELINE.json metric), config 2 workload.

Workload (BASELINE.json configs[1]): 10,000 accounts (ledger 2, code 1, history)
and 10,000,000 uniform create_transfers in 8189-event batches (1,221 x 8189 + 1,231), sequential
ids, `amount = Exp(10_000) +| 1`, seed 42. A *step* is one pass of the hot path over that whole
synthetic input: one tbg_create_transfers_device call carrying all 1,222 batches (each batch with
its own commit timestamp, TestContext rule prepare_ts += 1 + n). Inputs are resident in HBM when
the timed region starts; every step uses fresh transfer ids, so every step does the full work.

Multi-GPU (weak scaling): one process per GPU; each rank owns its own ledger shard
(own accounts and transfers, ledger 2 + rank) with no data-path collective. The timed region is
bracketed by a barrier + device synchronise on every rank; the reported time is the max over ranks.

Validation (after the timed region): every result must be `created`, and every account's final
balances must equal the exact per-account sums of the steps' amounts (the workload is
order-independent, so this is the serial reference outcome).

Output: one JSON line on rank 0 with `roofline` (dominant kernel, HIP-event timed) and
`cpu_baseline` (the serial C oracle on one host core, bounded sample of the same workload).
"""
import argparse
import ctypes
import json
import os
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
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")
BATCH = 8189           # Operation.create_transfers.event_max (src/tigerbeetle.zig:853-901)

# Algorithmic bytes per event of each kernel of the create_transfers path: the
# fields the kernel must read or write for its function, counted once.
KERNEL_BYTES_PER_EVENT = {
    # event 128 R, id-key claim 16 (8-B slot read + write), transfer row 128 W, result 16 W,
    # 2 packed balance items 16 W, info + liveness 2 W (FAST events write no other record)
    "tr_ingest": 128 + 16 + 128 + 16 + 16 + 2,
    # re-validation pass (skipped when ingest raised no commit flag): record 21 R, result
    # timestamp 8 R, liveness 1 W
    "tr_commit": 21 + 8 + 1,
    # 2 packed u64 items, read and written once (large key spaces)
    "bal_sort": 2 * 8 * 2,
    # sorted items read once (account rows are per distinct account)
    "bal_reduce": 2 * 8,
    # bucketed path (small key spaces): items read + written into their buckets
    "bal_scatter": 2 * 8 * 2,
    # bucketed items read once (slice partials are per bucket key, not per event)
    "bal_accumulate": 2 * 8,
}


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
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="bounded CPU-oracle sample (rank 0, N=1)")
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
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
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


def batch_plan(n):
    lens = [BATCH] * (n // BATCH) + ([n % BATCH] if n % BATCH else [])
    return np.asarray(lens, dtype=np.int64)


def step_timestamps(prepare_ts, lens):
    """TestContext rule per commit: prepare_ts += 1 + n; the batch's timestamp is prepare_ts."""
    ts = prepare_ts + np.cumsum(lens + 1)
    return ts.astype(np.uint64), int(ts[-1])


def measured_traffic(kernel):
    """(HBM bytes per launch, source) of `kernel` from TRAFFIC_FILE, or (None, None)."""
    try:
        with open(TRAFFIC_FILE) as fh:
            d = json.load(fh)
        return float(d["kernels"][kernel]["hbm_bytes_per_launch"]), d.get("source")
    except (OSError, ValueError, KeyError, TypeError):
        return None, None


def cpu_baseline(args, acc, base, lens, label):
    """The serial C oracle (oracle/liboracle.so) on one core, bounded sample of the workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_binding
    olib = oracle_binding.load()
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
        assert (out["status"][:n] == 0xFFFFFFFF).all()
        done += n
        off += n
        b += 1
        if time.perf_counter() - t0 >= args.cpu_seconds:
            break
    elapsed = time.perf_counter() - t0
    olib.tbo_close(o)
    return {"value": done / elapsed, "unit": "transfers/s", "cores": 1, "kind": "port",
            "sample": f"{done} of the {len(base)} {label} transfers ({b} batches of <= {BATCH}) "
                      f"through oracle/tb_oracle.c, single-threaded, {elapsed:.1f} s"}


class Config2:
    """BASELINE.json configs[1]: 10k accounts (ledger 2 + rank), 10M uniform transfers per step."""
    name = "config2"

    def __init__(self, args, rank, world):
        self.N = args.transfers or 10_000_000
        self.A = args.accounts or 10_000
        self.ledger = 2 + rank
        self.acc = workload.accounts(self.A, seed=args.seed, ledger=self.ledger)
        self.base = workload.transfers_uniform(self.N, self.A, seed=args.seed, ledger=self.ledger)
        self.dr = self.base["debit_account_id"][:, 0].astype(np.int64) - 1
        self.cr = self.base["credit_account_id"][:, 0].astype(np.int64) - 1
        self.chunk = self.A
        self.default = (self.N, self.A) == (10_000_000, 10_000)
        self.config = {"workload": "config2: 10k accounts, 10M uniform create_transfers in "
                                   "8189-event batches, 1 ledger shard per GPU",
                       "transfers_per_step_per_gpu": self.N, "accounts_per_gpu": self.A}

    def account_chunks(self):
        yield self.acc

    def validate(self, lib, g, reps):
        """Every account's final balances equal the exact per-account sums (the workload is
        order-independent, so this is the serial reference outcome)."""
        dump = np.zeros(self.A, dtype=ACCOUNT_DTYPE)
        assert lib.tbg_dump_accounts(g, dump.ctypes.data_as(ctypes.c_void_p)) == self.A
        amt = self.base["amount"][:, 0].astype(np.int64)
        exp_d = np.bincount(self.dr, weights=amt, minlength=self.A).astype(np.int64) * reps
        exp_c = np.bincount(self.cr, weights=amt, minlength=self.A).astype(np.int64) * reps
        ok = bool((dump["debits_posted"][:, 0].astype(np.int64) == exp_d).all())
        ok &= bool((dump["credits_posted"][:, 0].astype(np.int64) == exp_c).all())
        ok &= bool((dump["debits_posted"][:, 1] == 0).all() and (dump["credits_pending"] == 0).all())
        return ok

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
                                                                 seed=args.seed)
        self.chunk = min(self.A, 4_000_000)
        self.default = False
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

    def validate(self, lib, g, reps):
        """Sampled (SURVEY.md §8d at 1B scale): 65,536 touched accounts and 4,096 others looked up
        by id; their balances must equal the exact sums of the steps' amounts."""
        rng = np.random.default_rng(5)
        touched = np.unique(np.concatenate([self.dr, self.cr]))
        sample = np.concatenate([rng.choice(touched, size=min(65_536, len(touched)), replace=False),
                                 rng.integers(0, self.A, size=4_096)])
        sample = np.unique(sample)
        amt = self.base["amount"][:, 0].astype(np.int64)
        pos = np.full(self.A, -1, dtype=np.int64)
        pos[sample] = np.arange(len(sample))
        exp_d = np.zeros(len(sample), dtype=np.int64)
        exp_c = np.zeros(len(sample), dtype=np.int64)
        md, mc = pos[self.dr] >= 0, pos[self.cr] >= 0
        np.add.at(exp_d, pos[self.dr[md]], amt[md])
        np.add.at(exp_c, pos[self.cr[mc]], amt[mc])
        ids = np.zeros((len(sample), 2), dtype=np.uint64)
        ids[:, 0] = (workload.config5_global_index(sample, self.rank, self.world) + 1)
        out = np.zeros(len(sample), dtype=ACCOUNT_DTYPE)
        found = lib.tbg_lookup_accounts(g, ids.ctypes.data_as(ctypes.c_void_p), len(sample),
                                        out.ctypes.data_as(ctypes.c_void_p))
        ok = found == len(sample) and bool((out["id"][:, 0] == ids[:, 0]).all())
        ok &= bool((out["debits_posted"][:, 0].astype(np.int64) == exp_d * reps).all())
        ok &= bool((out["credits_posted"][:, 0].astype(np.int64) == exp_c * reps).all())
        return ok

    def cpu_sample(self):
        """The oracle holds only the accounts the sampled transfers touch (its hash maps do not
        depend on the account count): the first 1M transfers of the stream."""
        n = min(self.N, 1_000_000)
        j = np.unique(np.concatenate([self.dr[:n], self.cr[:n]]))
        return workload.accounts_config5(j, self.rank, self.world), self.base[:n], "config-5"


def main():
    args = parse_args()
    world, rank, local, dist = dist_init(args)
    wl = (Config5 if args.workload == "config5" else Config2)(args, rank, world)
    N, A, K, W = wl.N, wl.A, args.steps, args.warmup
    lib = native.load()
    dev = Device()
    dev.set_device(local)

    base = wl.base
    lens = batch_plan(N)
    ends = np.cumsum(lens).astype(np.uint32)

    opt = native.TbgOptions()
    opt.account_capacity = A
    opt.transfer_capacity = N * (K + W + 1)  # + one host-buffer step (pcie_inclusive)
    opt.batch_events_max = max(N, wl.chunk)
    opt.batch_count_max = len(lens)
    opt.pulse_batch_max = 8190
    opt.device = local
    opt.pulse_next_timestamp_init = 1
    g = lib.tbg_open(ctypes.byref(opt))
    assert g, "tbg_open failed"

    prepare_ts = 0
    for acc in wl.account_chunks():
        res_acc = np.zeros(len(acc), dtype=RESULT_DTYPE)
        a_lens = np.asarray([len(acc)], dtype=np.uint32)
        prepare_ts += 1 + len(acc)
        a_ts = np.asarray([prepare_ts], dtype=np.uint64)
        rc = lib.tbg_create_accounts(g, acc.ctypes.data_as(ctypes.c_void_p), len(acc),
                                     a_lens.ctypes.data_as(native.c_u32p),
                                     a_ts.ctypes.data_as(native.c_u64p), 1,
                                     res_acc.ctypes.data_as(ctypes.c_void_p))
        assert rc == 0 and (res_acc["status"] == 0xFFFFFFFF).all(), \
            f"create_accounts: {rc} {lib.tbg_last_error(g)}"
        del acc, res_acc

    # Per-step inputs, resident in HBM before timing: fresh ids per step.
    d_ends = dev.upload(ends)
    steps = []
    for s in range(W + K):
        ev = base.copy()
        ev["id"][:, 0] += np.uint64(s * N)
        ts, prepare_ts = step_timestamps(prepare_ts, lens)
        steps.append((dev.upload(ev), dev.upload(ts), dev.alloc(N * 16)))
        del ev
    dev.sync()

    def run_step(s):
        d_ev, d_ts, d_res = steps[s]
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

    validated = None
    if not args.no_validate:
        ok = True
        r = np.zeros(N, dtype=RESULT_DTYPE)
        for s in range(W + K):
            dev.download(steps[s][2], r)
            ok &= bool((r["status"] == 0xFFFFFFFF).all())
        ok &= wl.validate(lib, g, W + K)
        validated = ok
        if not ok:
            print(json.dumps({"error": "validation failed"}), file=sys.stderr)

    # The same step through the host-buffer ABI (tbg_create_transfers: events copied in, results
    # copied out over PCIe) -- the rate a caller holding host buffers sees; never `value`.
    pcie = None
    if not args.no_validate:
        ev = base.copy()
        ev["id"][:, 0] += np.uint64((W + K) * N)
        ts, prepare_ts = step_timestamps(prepare_ts, lens)
        h_lens = lens.astype(np.uint32)
        h_res = np.zeros(N, dtype=RESULT_DTYPE)
        t0 = time.perf_counter()
        rc = lib.tbg_create_transfers(g, ev.ctypes.data_as(ctypes.c_void_p), N,
                                      h_lens.ctypes.data_as(native.c_u32p),
                                      ts.ctypes.data_as(native.c_u64p), len(lens),
                                      h_res.ctypes.data_as(ctypes.c_void_p))
        t_host = time.perf_counter() - t0
        ok = rc == 0 and bool((h_res["status"] == 0xFFFFFFFF).all())
        validated = bool(validated) and ok
        pcie = {"value": round(N / t_host, 1), "unit": "transfers/s", "ms": round(t_host * 1e3, 3),
                "note": "one step through tbg_create_transfers with host buffers (events in, "
                        "results out over PCIe)"}

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
        achieved = kbytes / avg_s / 1e9
        traffic, traffic_src = measured_traffic(kname) if wl.default else (None, None)
        roofline = {"bound": "hbm", "kernel": kname, "achieved": round(achieved, 1),
                    "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": traffic, "traffic_source": traffic_src,
                    "alg_bytes_per_launch": kbytes,
                    "avg_launch_ms": round(kms / kcount, 4),
                    "path": {"alg_bytes_per_step": path_bytes,
                             "device_ms_per_step": round(dev_ms_total / K, 4),
                             "achieved": round(path_bytes / (dev_ms_total / K / 1e3) / 1e9, 1),
                             "frac": round(path_bytes / (dev_ms_total / K / 1e3) / 1e9 /
                                           HBM_PEAK_GBS, 4)},
                    "kernels_ms_per_step": {k: round(v[0] / K, 4) for k, v in kernels.items()}}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        acc_s, base_s, label = wl.cpu_sample()
        cpu = cpu_baseline(args, acc_s, base_s, batch_plan(len(base_s)), label)

    value = N * K * world / t_max
    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "transfers/s",
            "n_gpus": world, "steps": K, "warmup": W,
            "ms_per_step": round(t_max / K * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u128",
            "data": "synthetic (seeded; benchmark_load.zig distributions, sequential ids)",
            "config": dict(wl.config, batches_per_step=int(len(lens)),
                           parallelism=f"ledger-shard x{world}"),
            "validated": validated,
            "replayed_events_last_step": int(stats.replayed),
            "roofline": roofline,
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
        }
        print(json.dumps(line))
    lib.tbg_close(g)
    dev.free_all()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
