"""CPU / GPU crossover of the host-to-host control cycle.

For each batch size B: the GPU's wbc_cycle (host arrays in, host arrays out; WBC_RESIDENT for
B <= 4, the launch path above) on cold stance QPs, mean latency over N cycles, against the
structure-exploiting CPU restatement (oracle/wbc_fast.c, the engine's own algorithm on the CPU) on 1
and 16 threads over the same inputs.  The crossover is the smallest B where the GPU cycle is faster.
Prints one JSON line.  Usage (GPU box): python tools/cycle_sweep.py [cycles]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import wbc_ref as R  # noqa: E402  (the CPU side of the comparison only)

from quadrupedwholebodycontroller_amd import RESIDENT, STATELESS, Engine, workloads  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 300
out = {"cycles": N, "rows": []}
for B in (1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048, 4096):
    inp = workloads.stance_cold(B, seed=9)
    e = Engine(B)
    flags = STATELESS | (RESIDENT if B <= 4 else 0)
    args = (inp["base_pose"], inp["nu"], inp["qj"], inp["ref"], inp["contacts"], inp["switching"], flags)
    for _ in range(20):
        e.cycle(*args, want_x=False)
    lat = []
    for _ in range(N):
        t0 = time.perf_counter()
        e.cycle(*args, want_x=False)
        lat.append(time.perf_counter() - t0)
    e.close()
    gpu_us = float(np.mean(lat)) * 1e6
    row = {"batch": B, "gpu_cycle_us": gpu_us, "gpu_cycle_us_p99": float(np.percentile(lat, 99)) * 1e6}
    for th in (1, 16):
        reps = max(1, int(2000 // B))
        R.cpu_run_batch(inp, "fast", threads=th)  # warm
        t0 = time.perf_counter()
        for _ in range(reps):
            R.cpu_run_batch(inp, "fast", threads=th)
        row[f"cpu_us_{th}t"] = (time.perf_counter() - t0) / reps * 1e6
    out["rows"].append(row)
    print(json.dumps(row), flush=True)
for th in (1, 16):
    x = next((r["batch"] for r in out["rows"] if r["gpu_cycle_us"] < r[f"cpu_us_{th}t"]), None)
    out[f"crossover_batch_vs_{th}t"] = x
print(json.dumps(out))
