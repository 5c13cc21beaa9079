"""Where a B = 1 control cycle's time goes (BASELINE configs[0], the drop-in's own use case): the step
kernel alone (HIP events around back-to-back wbc_step launches on resident inputs), and the whole
host-to-host wbc_cycle (pack, H2D, step, D2H, synchronize) measured on the host clock, stateful stance
hold as wbc_control_loop runs it.  Usage (GPU box): python tools/b1_probe.py [cycles]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrupedwholebodycontroller_amd import NO_X, STATELESS, TIMED, Engine, workloads  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
inp = workloads.stance_cold(1, seed=1)
inp["switching"][:] = 0
res = {}
for name, flags in (("stateful", 0), ("stateless", STATELESS)):
    e = Engine(1)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    for _ in range(20):
        e.step(flags | NO_X)
    ks = []
    for _ in range(200):
        e.step(flags | NO_X | TIMED)
        ks.append(e.last_kernel_ms() * 1e3)
    args = (inp["base_pose"], inp["nu"], inp["qj"], inp["ref"], inp["contacts"], inp["switching"])
    for _ in range(50):
        e.cycle(*args, flags=flags, want_x=False)
    t = []
    for _ in range(N):
        t0 = time.perf_counter()
        e.cycle(*args, flags=flags, want_x=False)
        t.append((time.perf_counter() - t0) * 1e6)
    e.close()
    t, ks = np.array(t), np.array(ks)
    res[name] = dict(kernel_us_p50=float(np.median(ks)), cycle_us_mean=float(t.mean()), cycle_us_p50=float(np.median(t)),
                     cycle_us_p99=float(np.percentile(t, 99)))
print(json.dumps(res))
