#!/usr/bin/env python3
"""Host-buffer calls (tbg_create_transfers: events in, results out over PCIe) of config 2's 10M-event
step, with pageable buffers and with registered ones (tbg_register_host: pinned and mapped, as a
replica registers its message pool once). Prints one JSON line per call.
Usage (repo root, via gpurun): python tools/pcie_host.py [--transfers N] [--calls C]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tigerbeetle_amd import native, workload  # noqa: E402
from tigerbeetle_amd.types import RESULT_DTYPE  # noqa: E402

CREATED = 0xFFFFFFFF


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--transfers", type=int, default=10_000_000)
    ap.add_argument("--calls", type=int, default=2)
    args = ap.parse_args()
    N, A = args.transfers, 10_000
    lib = native.load()
    modes = ["pageable", "registered"]
    opts = native.options(A, N * args.calls * len(modes) + 1, N, batch_count_max=N // 8189 + 2)
    g = lib.tbg_open(ctypes.byref(opts))
    assert g, "tbg_open"
    acc = workload.accounts(A, seed=1)
    res = np.zeros(A, dtype=RESULT_DTYPE)
    ts = np.asarray([A], dtype=np.uint64)
    assert lib.tbg_create_accounts(g, acc.ctypes.data, A,
                                   np.asarray([A], np.uint32).ctypes.data_as(native.c_u32p),
                                   ts.ctypes.data_as(native.c_u64p), 1,
                                   res.ctypes.data) == 0
    lens = np.full(N // 8189, 8189, dtype=np.uint32)
    if N % 8189:
        lens = np.append(lens, np.uint32(N % 8189))
    prepare = A + 1
    call = 0
    for mode in modes:
        for _ in range(args.calls):
            ev = workload.transfers_uniform(N, A, seed=call, id_offset=call * N)
            out = np.zeros(N, dtype=RESULT_DTYPE)
            if mode == "registered":
                assert lib.tbg_register_host(g, ev.ctypes.data, ev.nbytes) == 0
                assert lib.tbg_register_host(g, out.ctypes.data, out.nbytes) == 0
            bts = (prepare + np.cumsum(lens)).astype(np.uint64)
            prepare = int(bts[-1]) + 1
            t0 = time.perf_counter()
            rc = lib.tbg_create_transfers(g, ev.ctypes.data, N, lens.ctypes.data_as(native.c_u32p),
                                          bts.ctypes.data_as(native.c_u64p),
                                          len(lens), out.ctypes.data)
            dt = time.perf_counter() - t0
            ok = rc == 0 and bool((out["status"] == CREATED).all())
            if mode == "registered":
                lib.tbg_unregister_host(g, ev.ctypes.data)
                lib.tbg_unregister_host(g, out.ctypes.data)
            moved = N * (128 + 16)
            print(json.dumps({"mode": mode, "call": call, "ms": round(dt * 1e3, 3),
                              "transfers_per_s": round(N / dt, 1),
                              "pcie_gb_per_s": round(moved / dt / 1e9, 1), "validated": ok}),
                  flush=True)
            call += 1
    lib.tbg_close(g)


if __name__ == "__main__":
    main()
