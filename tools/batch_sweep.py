"""Step-kernel time against batch size on the headline workload (stateless four-contact stance, cold):
the staircase that shows the kernel is one wave's dependency chain, not a throughput limit.  At one
wave per SIMD (B = 4096: 1024 waves of four QPs on 1024 SIMDs) a smaller batch leaves SIMDs idle yet
takes nearly as long; a second round of waves (B > 4096) adds a second chain.  DESIGN.md 4.13.
Usage (GPU box): python tools/batch_sweep.py [reps]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrupedwholebodycontroller_amd import NO_X, STATELESS, TIMED, Engine, workloads  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 50
full = workloads.stance_cold(16384, seed=1)
res = []
for B in (4, 64, 256, 1024, 2048, 3072, 4096, 4100, 6144, 8192, 12288, 16384):
    e = Engine(B)
    e.set_state(full["base_pose"][:B], full["nu"][:B], full["qj"][:B])
    e.set_reference(full["ref"][:B], full["contacts"][:B], full["switching"][:B])
    for _ in range(5):
        e.step(STATELESS | NO_X)
    ks = []
    for _ in range(REPS):
        e.step(STATELESS | NO_X | TIMED)
        ks.append(e.last_kernel_ms() * 1e3)
    it = e.outputs()["iters"]
    e.close()
    ks = np.array(ks)
    res.append(dict(B=B, waves=(B + 3) // 4, kernel_us_p50=round(float(np.median(ks)), 2),
                    kernel_us_min=round(float(ks.min()), 2), max_iters=int(it.max()),
                    qp_per_s_M=round(B / float(np.median(ks)), 1)))
    print(json.dumps(res[-1]), flush=True)
