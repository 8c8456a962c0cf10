#!/usr/bin/env python3
"""create_accounts throughput: C calls of N accounts each (host buffers, registered), validated
(every result created). Prints one JSON line. Usage: python tools/accounts_rate.py [--n N] [--calls C]"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--calls", type=int, default=4)
    args = ap.parse_args()
    N, C = args.n, args.calls
    lib = native.load()
    opts = native.options(N * C + 16, 1 << 10, N, batch_count_max=N // 8189 + 2)
    g = lib.tbg_open(ctypes.byref(opts))
    assert g, "tbg_open"
    lens = np.full(N // 8189, 8189, dtype=np.uint32)
    if N % 8189:
        lens = np.append(lens, np.uint32(N % 8189))
    prepare, times, ok = 1, [], True
    for c in range(C):
        acc = workload.accounts(N, seed=c, id_offset=c * N)
        out = np.zeros(N, dtype=RESULT_DTYPE)
        assert lib.tbg_register_host(g, acc.ctypes.data, acc.nbytes) == 0
        assert lib.tbg_register_host(g, out.ctypes.data, out.nbytes) == 0
        bts = (prepare + np.cumsum(lens)).astype(np.uint64)
        prepare = int(bts[-1]) + 1
        t0 = time.perf_counter()
        rc = lib.tbg_create_accounts(g, acc.ctypes.data, N, lens.ctypes.data_as(native.c_u32p),
                                     bts.ctypes.data_as(native.c_u64p), len(lens), out.ctypes.data)
        times.append(time.perf_counter() - t0)
        ok &= rc == 0 and bool((out["status"] == 0xFFFFFFFF).all())
        lib.tbg_unregister_host(g, acc.ctypes.data)
        lib.tbg_unregister_host(g, out.ctypes.data)
    lib.tbg_close(g)
    t = sorted(times)[len(times) // 2]
    print(json.dumps({"lib": os.environ.get("TBG_LIB", "default"), "accounts_per_call": N,
                      "ms_per_call_median": round(t * 1e3, 3),
                      "accounts_per_s": round(N / t, 1), "validated": ok}))


if __name__ == "__main__":
    main()
