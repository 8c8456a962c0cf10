"""Configs 3 and 4 at BASELINE scale (10k accounts; 1M events per run) against the oracle.

The order-dependent workloads of BASELINE.json (configs[2], configs[3]) as the builder's rate tool
runs them (tests/configs34.py): commits of 16 x 8189 events (the executor's multi-batch calls) and
one-batch commits of <= 8189 events (one replica prepare, tigerbeetle.zig:853-901). Every call's
results byte for byte, then every Account / Transfer row, TransferPending status and AccountEvent
(parity.Pair). Config 3 also runs with the one-lane account walk (TBG_LANES_ONE_LANE), config 4
with every post/void replayed (TBG_NO_PV_FAST) on its one-batch form.
"""
import ctypes

import pytest

import configs34
from parity import Pair

pytestmark = pytest.mark.gpu

BATCH = configs34.BATCH


def _pair(n, batches, registered=False):
    # (batch_events_max also holds the 10k-account create_accounts call)
    return Pair(account_capacity=1 << 14, transfer_capacity=n + (1 << 14),
                batch_events_max=max(BATCH * batches, 1 << 14), batch_count_max=batches,
                registered=registered)


@pytest.mark.parametrize("walk", ["wave", "one_lane"])
def test_config3_baseline_scale(walk, monkeypatch):
    """10k accounts, 100 hot with debits_must_not_exceed_credits; 1M events as 8 calls of
    16 x 8189 (the last one shorter), then one single-batch 8189-event call
    (state_machine.zig:3903-3913 in serial order)."""
    if walk == "one_lane":
        monkeypatch.setenv("TBG_LANES_ONE_LANE", "1")
    p = _pair(1_000_000 + BATCH, 16)
    try:
        s = configs34.config3(p, 1_000_000, batches_per_commit=16, tail_single=BATCH)
        assert s["calls"] == 9
        # ~20% of each hot account's debits find its credits exhausted
        assert 0.1 * s["hot_debits"] < s["exceeds_credits"] < 0.35 * s["hot_debits"]
        assert p.stats["replayed"] > 500_000  # the walk decides most of the stream
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("registered", [False, True], ids=["pageable", "registered"])
def test_config3_one_batch_commits(registered):
    """Config 3 as replica commits: 25 single-batch calls of 8189 events (bodies and replies in a
    registered host pool: read and written by the kernels over PCIe)."""
    p = _pair(25 * BATCH, 1, registered)
    try:
        s = configs34.config3(p, 25 * BATCH, batches_per_commit=1)
        assert s["calls"] == 25 and s["exceeds_credits"] > 0
        p.compare_state()
    finally:
        p.close()


def test_config4_baseline_scale():
    """10k accounts; 1M events of pending / post / void / chains with injected failures /
    resubmits in 8 calls of 16 x 8189, a 1-2 s tick and a pulse after each
    (state_machine.zig:3033-3207, :4053-4299, :4511-4628)."""
    p = _pair(1_000_000, 16)
    try:
        s = configs34.config4(p, 1_000_000, batches_per_commit=16)
        assert s["commits"] == 8
        # created, exceeds_credits, pending_transfer_already_posted / _voided, the ledger
        # mismatch, and linked_event_failed all occur
        for st in (0xFFFFFFFF, 54, 24, 32, 1):
            assert st in s["statuses"], st
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("pv", ["fast", "replayed", "registered"])
def test_config4_one_batch_commits(pv, monkeypatch):
    """Config 4 as replica commits: 30 single-batch calls of 8189 events with ticks and pulses;
    post/voids FAST-claimed, or all replayed (TBG_NO_PV_FAST), or FAST with the bodies and
    replies in a registered host pool."""
    if pv == "replayed":
        monkeypatch.setenv("TBG_NO_PV_FAST", "1")
    p = _pair(30 * BATCH, 1, registered=pv == "registered")
    try:
        s = configs34.config4(p, 30 * BATCH, batches_per_commit=1)
        assert s["commits"] == 30
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("config", ["config3", "config4"])
def test_configs34_wide_amounts(config):
    """Amounts log-uniform over [1, 2^63) (workload amounts="wide"): the account lanes' windows
    on u128 (owners' balances past 2^62), balance items too wide to pack (tr_commit's atomics),
    AccountEvents past the one-pass paths' 2^19 gate; 300k events, every result, row and
    AccountEvent against the oracle."""
    n = 300_000
    p = _pair(n + BATCH, 16)
    try:
        drive = configs34.config3 if config == "config3" else configs34.config4
        s = drive(p, n, batches_per_commit=16, amounts="wide")
        if config == "config3":
            assert s["exceeds_credits"] > 0
        p.compare_state()
    finally:
        p.close()


def _profile(p):
    out, i = {}, 0
    name = ctypes.create_string_buffer(64)
    ms, cnt = ctypes.c_double(), ctypes.c_uint64()
    while p.lib.tbg_profile_read(p.g, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt)):
        out[name.value.decode()] = ms.value
        i += 1
    return out


@pytest.mark.parametrize("config", ["config3", "config4"])
def test_profile_span_marks(config):
    """tbg_profile(ctx, 3), the span marks tools/bench_configs.py reports `device_ms` from: only the
    call's device spans are recorded (no per-kernel entries), and the calls stay exact against the
    oracle; with every mark (mode 1) the per-kernel entries appear."""
    n = 4 * 16 * BATCH
    seen = {}
    for mode in (3, 1):
        p = _pair(n, 16)
        try:
            drive = configs34.config3 if config == "config3" else configs34.config4
            drive(p, n, batches_per_commit=16, before_calls=lambda: p.lib.tbg_profile(p.g, mode))
            seen[mode] = _profile(p)
            p.compare_state()
        finally:
            p.close()
    spans = {k for k in seen[3] if not k.startswith(("host:", "pulse:"))}
    assert spans and spans <= {"host_sync", "call", "account_events"}, seen[3]
    assert {"host_sync", "call"} <= spans
    assert "tr_ingest" in seen[1] and ("tr_lanes" in seen[1] or "tr_flow" in seen[1])
