#!/usr/bin/env python3
"""A replica's commit loop through the StateMachine boundary, as bench.py's per_commit measures it:
one 8189-event create_transfers body per commit from a registered (page-locked) message pool, the
reply into a registered buffer, AccountEvents recorded (or not: --no-account-events).

Run it under `rocprofv3 --kernel-trace --memory-copy-trace --output-format csv` and pass the
traces to `--timeline` afterwards to see, per commit, the copies and kernels and the gaps between
them. Alone it prints the wall time per commit and the host phases (tbg_profile mode 2).
Usage: python tools/commit_timeline.py [--commits 100] [--no-account-events]
       python tools/commit_timeline.py --timeline <kernel_trace.csv> <memory_copy_trace.csv>"""
import argparse
import csv
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tigerbeetle_amd import native, workload  # noqa: E402

BATCH = 8189
MBSM = (1 << 20) - 256


def profile_read(lib, g):
    out, i = {}, 0
    name = ctypes.create_string_buffer(64)
    ms, cnt = ctypes.c_double(), ctypes.c_uint64()
    while lib.tbg_profile_read(g, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt)):
        out[name.value.decode()] = ms.value
        i += 1
    return out


def run(lib, R, account_events, mode):
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
    assert sm
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

    def commit(operation, body, size):
        lib.tb_sm_set_commit_timestamp(sm, lib.tb_sm_get_prepare_timestamp(sm))
        lib.tb_sm_set_prepare_timestamp(sm, lib.tb_sm_get_prepare_timestamp(sm) + 1)
        lib.tb_sm_prepare(sm, operation, body, size)
        ts = lib.tb_sm_get_prepare_timestamp(sm)
        lib.tb_sm_set_prefetch_timestamp(sm, ts)
        op[0] += 1
        lib.tb_sm_prefetch(sm, cb, None, op[0], op[0], operation, body, size)
        rc = lib.tb_sm_commit(sm, 1, 0, op[0], ts, operation, body, size, out)
        assert rc >= 0, rc

    acc = workload.accounts(10_000, seed=42)
    for a in range(0, 10_000, BATCH):
        b = encode(acc[a:a + BATCH])
        commit(146, b, len(b))
    base = workload.transfers_uniform(BATCH, 10_000, seed=42)
    first = encode(base)
    stride = (len(first) + 4095) // 4096 * 4096
    raw = np.zeros((R + 1) * stride + 4096, dtype=np.uint8)
    off = (-raw.ctypes.data) % 4096
    pool = raw[off:off + (R + 1) * stride]
    for r in range(R + 1):
        ev = base.copy()
        ev["id"][:, 0] += np.uint64(r * BATCH + 1)
        b = encode(ev)
        pool[r * stride:r * stride + len(b)] = np.frombuffer(b, dtype=np.uint8)
    assert lib.tb_sm_register_buffer(sm, pool.ctypes.data, pool.nbytes) == 0
    assert lib.tb_sm_register_buffer(sm, ctypes.addressof(out), len(out)) == 0
    size = len(first)
    commit(147, ctypes.c_void_p(pool.ctypes.data), size)  # warm
    lib.tbg_synchronize(g)
    lib.tbg_profile(g, mode)
    lat = np.zeros(R)
    t0 = time.perf_counter()
    for r in range(1, R + 1):
        t = time.perf_counter()
        commit(147, ctypes.c_void_p(pool.ctypes.data + r * stride), size)
        lat[r - 1] = time.perf_counter() - t
    wall = (time.perf_counter() - t0) / R
    prof = {k: round(v / R * 1e3, 1) for k, v in profile_read(lib, g).items()}
    lib.tb_sm_close(sm)
    return {"account_events": account_events, "profile_mode": mode,
            "us_per_commit": round(wall * 1e6, 1), "us_p50": round(float(np.median(lat)) * 1e6, 1),
            "transfers_per_s": round(BATCH / wall, 1), "us_per_commit_by_phase": prof}


def timeline(kernel_csv, copy_csv, last=6):
    rows = []
    with open(kernel_csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("void ", "").replace("tbg::", "")[:44]))
    if copy_csv and os.path.exists(copy_csv):
        with open(copy_csv) as f:
            for r in csv.DictReader(f):
                kind = r.get("Direction") or r.get("Operation") or "copy"
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                             f"COPY {kind} {r.get('Size', '')}"))
    rows.sort()
    # the last `last` commits: from the last `last` tr_chunk_info launches on
    anchor = "stage_in" if any(r[2].startswith("stage_in") for r in rows) else "tr_chunk_info"
    starts = [i for i, r in enumerate(rows) if r[2].startswith(anchor)]
    if len(starts) < last + 1:
        return
    i0 = starts[-last - 1]
    # back up to the copies that precede it (the body upload)
    while i0 > 0 and rows[i0 - 1][2].startswith("COPY"):
        i0 -= 1
    t_base, prev_end = rows[i0][0], rows[i0][0]
    for s, e, name in rows[i0:]:
        print(f"{(s - t_base) / 1e3:9.2f} us  gap {(s - prev_end) / 1e3:7.2f}  dur {(e - s) / 1e3:7.2f}  {name}")
        prev_end = max(prev_end, e)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--commits", type=int, default=100)
    ap.add_argument("--no-account-events", action="store_true")
    ap.add_argument("--mode", type=int, default=2, help="tbg_profile mode (0 off, 1 kernels, 2 host)")
    ap.add_argument("--timeline", nargs="+")
    a = ap.parse_args()
    if a.timeline:
        timeline(a.timeline[0], a.timeline[1] if len(a.timeline) > 1 else None)
        return
    lib = native.load()
    print(json.dumps(run(lib, a.commits, not a.no_account_events, a.mode)))


if __name__ == "__main__":
    main()
