"""Drivers of the order-dependent workloads (BASELINE.json configs 3 and 4) over a parity.Pair.

Test infrastructure: both the GPU parity tests (tests/test_configs34.py) and the builder's rate
tool (tools/bench_configs.py) run these, so the rates reported and the parity checked are of the
same calls. Every call goes through the host-buffer C ABI (tbg_create_transfers) and the serial
oracle on the same batches; the Pair compares every result, and `Pair.compare_state` every
Account / Transfer row, TransferPending status and AccountEvent.

  config3: 10k accounts, 100 hot accounts with debits_must_not_exceed_credits (Zipf 0.99 over the
           hot set takes 90% of debits, ~10% of credits go to hot accounts), funded from an
           unlimited source with 80% of what the stream debits from each (state_machine.zig
           :3903-3913 decides the last ~20% as exceeds_credits, in serial order).
  config4: 10k accounts; 30% pending with 1-5 s timeouts, later post (67%, full or partial) /
           void (33%) of earlier pending transfers, 8-event linked chains on 30% of events with
           one injected failure in 10% of chains, 1% resubmitted ids; 1-2 s ticks with pulses
           between commits (state_machine.zig:3033-3207, :4053-4299, :4511-4628).
"""
import numpy as np

from tigerbeetle_amd import workload
from tigerbeetle_amd.types import NS_PER_S

BATCH = 8189
EXCEEDS_CREDITS = 54


def commit_lens(m, batch=BATCH):
    """A commit of m events as a multi-batch body of <= `batch`-event batches."""
    return [batch] * (m // batch) + ([m % batch] if m % batch else [])


def config3(p, n, batches_per_commit=16, tail_single=0, accounts=10_000, n_hot=100, seed=3,
            before_calls=None, amounts="exp"):
    """Config 3 on Pair `p` (capacities: accounts + 1, n + tail_single + n_hot transfers).
    `tail_single` more events follow as one single-batch call (one replica commit of <= 8189
    events). `before_calls` (if given) runs after setup, before the measured calls. Returns a
    summary dict."""
    acc = workload.accounts(accounts, seed=seed)
    acc["flags"][1:n_hot + 1] |= 2  # debits_must_not_exceed_credits
    p.create_accounts(acc)
    t = workload.transfers_hot_limits(n + tail_single, n_accounts=accounts, n_hot=n_hot, seed=seed,
                                      amounts=amounts)
    p.create_transfers(workload.funding_transfers(
        n_hot, workload.hot_funding_amounts(t[:n], n_hot, 0.8), id_offset=1 << 40))
    if before_calls:
        before_calls()
    per_commit = BATCH * batches_per_commit
    failed, calls = 0, 0
    for off in range(0, n, per_commit):
        m = min(per_commit, n - off)
        r = p.create_transfers(t[off:off + m], commit_lens(m))
        failed += int((r["status"] == EXCEEDS_CREDITS).sum())
        calls += 1
    if tail_single:
        r = p.create_transfers(t[n:n + tail_single], [tail_single])
        failed += int((r["status"] == EXCEEDS_CREDITS).sum())
        calls += 1
    hot_debits = int(((t["debit_account_id"][:, 0] >= 2) &
                      (t["debit_account_id"][:, 0] < n_hot + 2)).sum())
    return {"exceeds_credits": failed, "hot_debits": hot_debits, "calls": calls,
            "batches_per_commit": batches_per_commit}


def config4(p, n, batches_per_commit=16, accounts=10_000, seed=4, n_limited=16,
            before_calls=None, amounts="exp"):
    """Config 4 on Pair `p`: commits of `batches_per_commit` x 8189 events, each followed by a
    1-2 s tick (the pulse runs when pulse_needed). Returns a summary dict with the statuses
    seen."""
    rng = np.random.default_rng(seed)
    acc = workload.accounts(accounts, seed=seed)
    acc["flags"][:n_limited] |= 2  # debited only by injected exceeds_credits failures
    p.create_accounts(acc)
    if before_calls:
        before_calls()
    pending, seen = np.zeros(0, dtype=np.uint64), np.zeros(0, dtype=np.uint64)
    resolved = np.zeros(0, dtype=np.uint64)
    per_commit = BATCH * batches_per_commit
    statuses = set()
    off, step = 0, 0
    while off < n:
        m = min(per_commit, n - off)
        t = workload.transfers_two_phase(m, accounts, seed=10 * seed + step, id_offset=off,
                                         prior_pending_ids=pending, prior_ids=seen,
                                         prior_resolved_ids=resolved, n_limited=n_limited,
                                         amounts=amounts)
        r = p.create_transfers(t, commit_lens(m))
        statuses |= set(int(x) for x in np.unique(r["status"]))
        created = r["status"] == 0xFFFFFFFF
        is_pending = (t["flags"] & 2) != 0
        pending = np.concatenate([pending, t["id"][created & is_pending, 0]])[-50_000:]
        pv = (t["flags"] & 12) != 0
        resolved = np.concatenate([resolved, t["pending_id"][created & pv, 0]])[-50_000:]
        seen = np.concatenate([seen, t["id"][:, 0]])[-200_000:]
        p.tick(int(rng.integers(1, 3)) * NS_PER_S)
        off += m
        step += 1
    return {"commits": step, "batches_per_commit": batches_per_commit,
            "statuses": sorted(statuses)}
