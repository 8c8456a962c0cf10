#!/usr/bin/env python3
"""Where a replica commit's time goes: one 8189-event create_transfers body per commit through
the StateMachine boundary (tb_sm_prepare / prefetch / commit, host buffers), with and without
AccountEvents, and through tbg_create_transfers_device (body in HBM). Prints, per commit, the wall
time and the executor's per-kernel HIP-event times (tbg_profile marks).
Usage: python tools/commit_profile.py [--commits 200]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tigerbeetle_amd import native, workload  # noqa: E402
from tigerbeetle_amd.types import RESULT_DTYPE  # noqa: E402

BATCH = 8189
MBSM = (1 << 20) - 256


def kernel_ms(lib, g):
    out, i = {}, 0
    name = ctypes.create_string_buffer(64)
    ms, cnt = ctypes.c_double(), ctypes.c_uint64()
    while lib.tbg_profile_read(g, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt)):
        out[name.value.decode()] = ms.value
        i += 1
    return out


def run_sm(lib, R, account_events, mode=1):
    sm_opt = native.SmOptions()
    sm_opt.batch_size_limit = MBSM
    sm_opt.message_body_size_max = MBSM
    sm_opt.pulse_batch_max = 8190
    o = native.TbgOptions()
    o.account_capacity = 10_000
    o.transfer_capacity = (R + 2) * BATCH
    o.batch_events_max = BATCH
    o.batch_count_max = 64
    o.pulse_batch_max = 8190
    o.device = 0
    o.pulse_next_timestamp_init = 1
    o.account_events_capacity = (R + 2) * BATCH if account_events else 0
    sm = lib.tb_sm_open_gpu(ctypes.byref(sm_opt), ctypes.byref(o))
    g = lib.tb_sm_executor_gpu(sm)
    out = ctypes.create_string_buffer(MBSM + 256)
    cb = native.PREFETCH_CALLBACK(lambda ctx: None)
    op = [0]

    def encode(records):
        payload = records.tobytes()
        trailer = lib.tb_multi_batch_trailer_total_size(128, 1)
        buf = ctypes.create_string_buffer(len(payload) + trailer + 2)
        ctypes.memmove(buf, payload, len(payload))
        size = lib.tb_multi_batch_encode_trailer(buf, len(payload), 128,
                                                 (ctypes.c_uint16 * 1)(len(records)), 1)
        return buf.raw[:size]

    def commit(operation, body):
        lib.tb_sm_set_commit_timestamp(sm, lib.tb_sm_get_prepare_timestamp(sm))
        lib.tb_sm_set_prepare_timestamp(sm, lib.tb_sm_get_prepare_timestamp(sm) + 1)
        lib.tb_sm_prepare(sm, operation, body, len(body))
        ts = lib.tb_sm_get_prepare_timestamp(sm)
        lib.tb_sm_set_prefetch_timestamp(sm, ts)
        op[0] += 1
        lib.tb_sm_prefetch(sm, cb, None, op[0], op[0], operation, body, len(body))
        size = lib.tb_sm_commit(sm, 1, 0, op[0], ts, operation, body, len(body), out)
        assert size >= 0
        return size

    acc = workload.accounts(10_000, seed=42)
    for a in range(0, 10_000, BATCH):
        commit(146, encode(acc[a:a + BATCH]))
    base = workload.transfers_uniform(BATCH, 10_000, seed=42)
    bodies = []
    for r in range(R):
        ev = base.copy()
        ev["id"][:, 0] += np.uint64(r * BATCH + 1)
        bodies.append(encode(ev))
    commit(147, bodies[0])  # warm
    lib.tbg_profile(g, mode)
    t0 = time.perf_counter()
    for r in range(1, R):
        commit(147, bodies[r])
    wall = (time.perf_counter() - t0) / (R - 1)
    k = {n: round(v / (R - 1) * 1e3, 1) for n, v in kernel_ms(lib, g).items()}
    lib.tb_sm_close(sm)
    return {"us_per_commit": round(wall * 1e6, 1),
            "transfers_per_s": round(BATCH / wall, 1), "kernel_us_per_commit": k}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--commits", type=int, default=200)
    a = ap.parse_args()
    lib = native.load()
    print(json.dumps({"state_machine_account_events": run_sm(lib, a.commits, True)}))
    print(json.dumps({"state_machine_no_account_events": run_sm(lib, a.commits, False)}))
    # host phases only (no HIP events between launches): the undistorted split
    print(json.dumps({"state_machine_account_events_host": run_sm(lib, a.commits, True, 2)}))
    print(json.dumps({"state_machine_no_account_events_host": run_sm(lib, a.commits, False, 2)}))


if __name__ == "__main__":
    main()
