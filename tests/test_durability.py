"""Durability of the HBM tables (include/tbg.h): tbg_compact (StateMachine.compact,
src/state_machine.zig:2912-2935), tbg_checkpoint / tbg_open_checkpoint (StateMachine.checkpoint
:2937-2958, open :964-978). Compaction and checkpoints are invisible to the results: a workload
with compactions or a checkpoint + reopen in the middle must match the uninterrupted CPU oracle
byte for byte (every result, every table row, AccountEvents, get_change_events)."""
import numpy as np
import pytest

from parity import Pair
from test_gpu_parity import _split
from tigerbeetle_amd import workload
from tigerbeetle_amd.types import NS_PER_S, TIMESTAMP_MAX

pytestmark = pytest.mark.gpu


def _workload_steps(p, rng, seed, steps, per_step=300, id_space=400, after_step=None):
    n_acc = 24
    a = workload.fuzz_accounts(rng, 40, n_acc)
    p.create_accounts(a, _split(len(a), rng, 12))
    clean = workload.accounts(n_acc, seed=seed, id_offset=0, ledger=1)
    clean["flags"] = rng.choice([0, 0, 2, 4, 8], size=n_acc).astype(np.uint16)
    p.create_accounts(clean, _split(n_acc, rng, 8))
    ids_seen = []
    for step in range(steps):
        pend = np.array(ids_seen[-200:], dtype=np.uint64) if ids_seen else None
        t = workload.fuzz_transfers(rng, per_step, id_space, n_acc + 1, pending_ids=pend)
        ids_seen.extend(int(x) for x in t["id"][:, 0])
        p.create_transfers(t, _split(len(t), rng, 64))
        if step % 3 == 2:
            p.tick(int(rng.integers(1, 3)) * NS_PER_S)
        if after_step:
            after_step(step)


@pytest.mark.parametrize("force_replay", [False, True], ids=["parallel", "flow"])
@pytest.mark.parametrize("seed", range(3))
def test_compact_under_capacity_pressure(seed, force_replay):
    """A transfer store of 2,048 rows takes 12 x 300 events only because every step compacts:
    the rows of failed events are dropped, created rows and orphaned ids stay (later duplicates
    of them still find them), expiries and pulses keep their order."""
    rng = np.random.default_rng(7000 + seed)
    p = Pair(account_capacity=1 << 12, transfer_capacity=2048, batch_events_max=4096,
             pulse_batch_max=16, pulse_next_timestamp_init=TIMESTAMP_MAX,
             force_replay=force_replay)
    freed = []
    try:
        _workload_steps(p, rng, seed, steps=12, after_step=lambda s: freed.append(p.compact()))
        p.compare_state()
        p.change_events()
        assert sum(freed) > 12 * 300 - 2048, freed
    finally:
        p.close()


@pytest.mark.parametrize("seed", range(3))
def test_checkpoint_reopen(seed, tmp_path):
    """Checkpoint mid-stream, close, reopen from the image, continue: the same as never stopping."""
    rng = np.random.default_rng(8000 + seed)
    p = Pair(account_capacity=1 << 12, transfer_capacity=1 << 15, batch_events_max=4096,
             pulse_batch_max=16, pulse_next_timestamp_init=TIMESTAMP_MAX)
    path = tmp_path / "tables.tbgckpt"

    def maybe_checkpoint(step):
        if step in (2, 5):
            p.checkpoint_reopen(path)
        if step == 6:
            p.compact()
            p.checkpoint_reopen(path)

    try:
        _workload_steps(p, rng, seed, steps=9, after_step=maybe_checkpoint)
        p.compare_state()
        p.change_events()
    finally:
        p.close()


def test_checkpoint_rejects_other_geometry(tmp_path):
    """An image opens only into a ctx with the same table geometry."""
    import ctypes
    p = Pair(account_capacity=1 << 10, transfer_capacity=1 << 12, batch_events_max=1024)
    try:
        p.create_accounts(workload.accounts(8, seed=1, ledger=1))
        path = tmp_path / "img"
        assert p.lib.tbg_checkpoint(p.g, str(path).encode()) == 0
        o = p.opt
        o.transfer_capacity = 1 << 14
        assert not p.lib.tbg_open_checkpoint(ctypes.byref(o), str(path).encode())
        assert not p.lib.tbg_open_checkpoint(ctypes.byref(o), str(tmp_path / "none").encode())
    finally:
        p.opt.transfer_capacity = 1 << 12
        p.close()


@pytest.mark.parametrize("damage", ["flip_row_byte", "flip_header_byte", "truncate", "no_footer"])
def test_checkpoint_rejects_torn_or_corrupt_images(damage, tmp_path):
    """Every section and the header carry a checksum: an image with one flipped byte, a cut-off
    tail or a missing footer opens nothing (StateMachine.open must not install torn tables);
    the intact image still opens and matches."""
    import ctypes
    import os
    p = Pair(account_capacity=1 << 10, transfer_capacity=1 << 12, batch_events_max=1024)
    try:
        p.create_accounts(workload.accounts(64, seed=1, ledger=1))
        p.create_transfers(workload.transfers_uniform(500, 64, seed=1, ledger=1))
        path = tmp_path / "img"
        assert p.lib.tbg_checkpoint(p.g, str(path).encode()) == 0
        assert not os.path.exists(str(path) + ".tmp")
        good = path.read_bytes()
        g = p.lib.tbg_open_checkpoint(ctypes.byref(p.opt), str(path).encode())
        assert g
        p.lib.tbg_close(g)
        bad = bytearray(good)
        if damage == "flip_row_byte":
            bad[len(bad) // 2] ^= 0x40
        elif damage == "flip_header_byte":
            bad[40] ^= 0x01
        elif damage == "truncate":
            bad = bad[:len(bad) - 1000]
        else:
            bad = bad[:len(bad) - 8]
        path.write_bytes(bytes(bad))
        assert not p.lib.tbg_open_checkpoint(ctypes.byref(p.opt), str(path).encode())
        path.write_bytes(good)
        g = p.lib.tbg_open_checkpoint(ctypes.byref(p.opt), str(path).encode())
        assert g
        p.lib.tbg_close(p.g)
        p.g = g
        p.compare_state()
    finally:
        p.close()
