"""Every environment knob of libtbg.so that changes how a call executes, set, against the oracle.

The executor reads these at each call (tigerbeetle_amd/csrc/executor.hip). Each one selects
another exact path or engine shape for the same results: the order-dependent workloads of configs
3 and 4 (tests/configs34.py: limit accounts, pending / post / void, linked chains with injected
failures) run under each setting and every result, row, TransferPending status and AccountEvent is
compared with the oracle (parity.Pair). Knobs covered elsewhere: TBG_LANES_ONE_LANE and
TBG_NO_PV_FAST (test_configs34.py), TBG_NO_SPIN_SYNC, TBG_NO_INGEST_FINISH, TBG_NO_LEAN_LOOKUP, TBG_NO_WINDOW,
TBG_NO_AE_WINDOW, TBG_WALK_SEQ, TBG_NO_ADDITIVE, TBG_NO_DOOM, TBG_NO_FREE_OWNERS
(test_gpu_parity.py). Diagnostics that change no path: TBG_CALL_TIMEOUT_MS (the host's wait bound)
and TBG_PULSE_HOST_TRACE (a printed trace).
"""
import pytest

import configs34
from parity import Pair

pytestmark = pytest.mark.gpu

BATCH = configs34.BATCH

KNOBS = [
    ("TBG_NO_LANES", "1"),        # the flow replay instead of the account lanes
    ("TBG_FLOW_LPW", "8"),        # flow engine: 8 lanes per wave
    ("TBG_FLOW_WAVES", "1"),      # ... one wave per workgroup
    ("TBG_FLOW_BLOCKS", "7"),     # ... 7 workgroups (an odd count)
    ("TBG_FLOW_XCD", "8"),        # ... workgroups packed onto one XCD
    ("TBG_FLOW_BACKOFF", "0"),    # ... no backoff in the hand-off waits
    ("TBG_FLOW_DEBUG", "1"),      # ... with its critical-path counters
]


@pytest.mark.parametrize("name,value", KNOBS, ids=[k for k, _ in KNOBS])
def test_knob_config4(name, value, monkeypatch):
    monkeypatch.setenv(name, value)
    n = 200_000
    p = Pair(account_capacity=1 << 14, transfer_capacity=n + (1 << 14),
             batch_events_max=max(BATCH * 16, 1 << 14), batch_count_max=16)
    try:
        configs34.config4(p, n, batches_per_commit=16)
        assert p.stats["replayed"] > 0
        p.compare_state()
    finally:
        p.close()


@pytest.mark.parametrize("name,value", KNOBS[:2], ids=[k for k, _ in KNOBS[:2]])
def test_knob_config3(name, value, monkeypatch):
    monkeypatch.setenv(name, value)
    n = 200_000
    p = Pair(account_capacity=1 << 14, transfer_capacity=n + (1 << 14),
             batch_events_max=max(BATCH * 16, 1 << 14), batch_count_max=16)
    try:
        s = configs34.config3(p, n, batches_per_commit=16)
        assert s["exceeds_credits"] > 0
        p.compare_state()
    finally:
        p.close()
