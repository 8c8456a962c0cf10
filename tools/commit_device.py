#!/usr/bin/env python3
"""Device per-commit timing: 300 tbg_create_transfers_device calls of one 8189-event body each
(config 2 shape, body in HBM), the wall time per call and, with tbg_profile mode 2, the host
phases. Usage: python tools/commit_device.py [profile mode]"""
import ctypes, sys, os, time, json
sys.path.insert(0, os.getcwd())
import numpy as np
import bench
from tigerbeetle_amd import native, workload
lib = native.load()
dev = bench.Device(); dev.set_device(0)
o = native.TbgOptions(); o.account_capacity = 1 << 14; o.transfer_capacity = 1 << 22; o.batch_events_max = 8189
o.batch_count_max = 64; o.pulse_batch_max = 8190; o.device = 0; o.pulse_next_timestamp_init = 1
g = lib.tbg_open(ctypes.byref(o))
acc = workload.accounts(10_000, seed=42)
for a in range(0, 10_000, 8189):
    part = acc[a:a + 8189]
    res = np.zeros(len(part), dtype=bench.RESULT_DTYPE)
    lib.tbg_create_accounts(g, part.ctypes.data_as(ctypes.c_void_p), len(part), (ctypes.c_uint32 * 1)(len(part)), (ctypes.c_uint64 * 1)(1_000_000 + a + len(part)), 1, res.ctypes.data_as(ctypes.c_void_p))
n = 8189; R = 300
base = workload.transfers_uniform(n, 10_000, seed=42)
d_end = dev.upload(np.asarray([n], dtype=np.uint32))
bufs = []
ts = 10_000_000
for r in range(R + 1):
    ev = base.copy(); ev["id"][:, 0] += np.uint64(r * n + 1)
    ts += n
    bufs.append((dev.upload(ev), dev.upload(np.asarray([ts], dtype=np.uint64)), dev.alloc(n * 16)))
dev.sync()
d_ev, d_ts, d_res = bufs[0]
assert lib.tbg_create_transfers_device(g, d_ev, n, d_end, d_ts, 1, d_res, None) == 0
dev.sync()
lib.tbg_profile(g, int(sys.argv[1]) if len(sys.argv) > 1 else 2)
t0 = time.perf_counter()
for r in range(1, R + 1):
    d_ev, d_ts, d_res = bufs[r]
    assert lib.tbg_create_transfers_device(g, d_ev, n, d_end, d_ts, 1, d_res, None) == 0
wall = (time.perf_counter() - t0) / R
out, i = {}, 0
name = ctypes.create_string_buffer(64); ms = ctypes.c_double(); cnt = ctypes.c_uint64()
while lib.tbg_profile_read(g, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt)):
    out[name.value.decode()] = round(ms.value / R * 1e3, 2); i += 1
print(json.dumps({"us_per_commit": round(wall * 1e6, 1), "phases_us": out}))
