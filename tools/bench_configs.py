#!/usr/bin/env python3
"""Validated throughput of the order-dependent workloads (BASELINE.json configs 3 and 4).

Each call goes through the host-buffer C ABI (tbg_create_transfers: PCIe copies included) and the
serial CPU oracle on the same batches; every call's results and, at the end, every Account /
Transfer row and TransferPending status must be byte-identical (tests/parity.py). Prints one JSON
line per config with the GPU and oracle rates over the create_transfers calls.

  config3: 10k accounts, 100 hot accounts with debits_must_not_exceed_credits (Zipf 0.99 over the
           hot set takes 90% of debits, ~10% of credits go to hot accounts), funded from an
           unlimited source; 8189-event batches, `--batches` per commit.
  config4: 10k accounts; 30% pending with 1-5 s timeouts, later post (67%, full or partial) /
           void (33%, amount 0 or nonzero) of earlier pending transfers, 8-event linked chains on
           30% of events with one injected failure in 10% of chains (missing account, ledger
           mismatch, exceeds_credits, post of an already posted / voided transfer), 1%
           resubmitted ids; 1-2 s ticks with pulses between commits.
Usage: python tools/bench_configs.py [--transfers N] [--configs 3,4]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from parity import Pair  # noqa: E402
from tigerbeetle_amd import workload  # noqa: E402
from tigerbeetle_amd.types import NS_PER_S  # noqa: E402

BATCH = 8189


def kernel_ms(p):
    """Per-kernel milliseconds over the profiled calls (tbg_profile marks on the call stream)."""
    out, i = {}, 0
    name = ctypes.create_string_buffer(64)
    ms, cnt = ctypes.c_double(), ctypes.c_uint64()
    while p.lib.tbg_profile_read(p.g, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt)):
        out[name.value.decode()] = round(ms.value, 3)
        i += 1
    return out


def line(name, p, n, t_wall, extra):
    kms = kernel_ms(p)
    extra = dict(extra, kernels_ms=kms)
    s = p.seconds
    # Device time: the HIP-event spans of the calls' kernels, the AccountEvents appends included
    # (`account_events`: queued behind each call's results); the host:* entries (PCIe copies, the
    # host-side parts of the calls) and the pulses between calls (pulse:*) are left out.
    dev_ms = sum(v for k, v in kms.items() if not k.startswith(("host:", "pulse:")))
    return {"config": name, "transfers": n, "validated": True,
            "gpu_transfers_per_s": round(n / s["gpu"], 1),
            "device_ms": round(dev_ms, 3),
            "device_transfers_per_s": round(n / (dev_ms / 1e3), 1) if dev_ms else None,
            "oracle_transfers_per_s": round(n / s["oracle"], 1), "oracle_cores": 1,
            "gpu_s": round(s["gpu"], 3), "oracle_s": round(s["oracle"], 3),
            "replayed": p.stats["replayed"], "fast": p.stats["fast"],
            "static_fail": p.stats["static_fail"], "wall_s": round(t_wall, 1), **extra}


def config3(n, commits_batches):
    t0 = time.perf_counter()
    A = 10_000
    p = Pair(account_capacity=1 << 14, transfer_capacity=n + (1 << 12),
             batch_events_max=BATCH * commits_batches, batch_count_max=commits_batches)
    try:
        acc = workload.accounts(A, seed=3)
        acc["flags"][1:101] |= 2  # debits_must_not_exceed_credits
        p.create_accounts(acc)
        t = workload.transfers_hot_limits(n, n_accounts=A, n_hot=100, seed=3)
        p.create_transfers(workload.funding_transfers(
            100, workload.hot_funding_amounts(t, 100, 0.8), id_offset=1 << 40))
        p.seconds = {"gpu": 0.0, "oracle": 0.0}
        p.stats = {k: 0 for k in p.stats}
        p.lib.tbg_profile(p.g, 1)
        per_commit = BATCH * commits_batches
        failed = 0
        for off in range(0, n, per_commit):
            m = min(per_commit, n - off)
            lens = [BATCH] * (m // BATCH) + ([m % BATCH] if m % BATCH else [])
            r = p.create_transfers(t[off:off + m], lens)
            failed += int((r["status"] == 54).sum())
        p.compare_state()
        hot_debits = int(((t["debit_account_id"][:, 0] >= 2) &
                          (t["debit_account_id"][:, 0] < 102)).sum())
        return line("config3", p, n, time.perf_counter() - t0,
                    {"exceeds_credits": failed, "hot_debits": hot_debits,
                     "batches_per_commit": commits_batches})
    finally:
        p.close()


def config4(n, commits_batches):
    t0 = time.perf_counter()
    A = 10_000
    rng = np.random.default_rng(4)
    p = Pair(account_capacity=1 << 14, transfer_capacity=n + (1 << 12),
             batch_events_max=BATCH * commits_batches, batch_count_max=commits_batches)
    try:
        acc = workload.accounts(A, seed=4)
        acc["flags"][:16] |= 2  # debited only by injected exceeds_credits failures
        p.create_accounts(acc)
        p.seconds = {"gpu": 0.0, "oracle": 0.0}
        p.lib.tbg_profile(p.g, 1)
        pending, seen = np.zeros(0, dtype=np.uint64), np.zeros(0, dtype=np.uint64)
        resolved = np.zeros(0, dtype=np.uint64)
        per_commit = BATCH * commits_batches
        off, step = 0, 0
        while off < n:
            m = min(per_commit, n - off)
            t = workload.transfers_two_phase(m, A, seed=40 + step, id_offset=off,
                                             prior_pending_ids=pending, prior_ids=seen,
                                             prior_resolved_ids=resolved, n_limited=16)
            lens = [BATCH] * (m // BATCH) + ([m % BATCH] if m % BATCH else [])
            r = p.create_transfers(t, lens)
            created = r["status"] == 0xFFFFFFFF
            is_pending = (t["flags"] & 2) != 0
            pending = np.concatenate([pending, t["id"][created & is_pending, 0]])[-50_000:]
            pv = (t["flags"] & 12) != 0
            resolved = np.concatenate([resolved, t["pending_id"][created & pv, 0]])[-50_000:]
            seen = np.concatenate([seen, t["id"][:, 0]])[-200_000:]
            p.tick(int(rng.integers(1, 3)) * NS_PER_S)
            off += m
            step += 1
        p.compare_state()
        return line("config4", p, n, time.perf_counter() - t0,
                    {"commits": step, "batches_per_commit": commits_batches})
    finally:
        p.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--transfers", type=int, default=1_000_000)
    ap.add_argument("--batches", type=int, default=16, help="8189-event batches per commit")
    ap.add_argument("--configs", default="3,4")
    args = ap.parse_args()
    for c in args.configs.split(","):
        fn = {"3": config3, "4": config4}[c.strip()]
        print(json.dumps(fn(args.transfers, args.batches)), flush=True)


if __name__ == "__main__":
    main()
