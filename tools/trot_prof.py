"""Where the stateful trot step (BASELINE configs[2]) spends its solve: loop passes (adds, drops
and the hotstart's warm-set re-adds) against the counted iterations, and per-sub-step loop cycles.
Usage (GPU box): WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so python tools/trot_prof.py [B] [T]
(with the default library it prints iterations only)."""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from quadrupedwholebodycontroller_amd import NO_X, Engine, workloads

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
T = int(sys.argv[2]) if len(sys.argv) > 2 else 100
seq = list(workloads.trot_sequence(B, steps=T, seed=2))
e = Engine(B)
ist = "istamps" in os.environ.get("WBC_LIB", "")
rows = []
for t, s in enumerate(seq):
    e.set_state(s["base_pose"], s["nu"], s["qj"])
    e.set_reference(s["ref"], s["contacts"], s["switching"])
    e.step(NO_X)
    if t >= 10 and t % 10 == 0:
        e.synchronize()
        o = e.outputs()
        r = dict(t=t, mean_iters=float(o["iters"].mean()), max_iters=int(o["iters"].max()),
                 masks=np.bincount(s["contacts"], minlength=16).nonzero()[0].tolist())
        if ist:
            d = e.debug()
            r["mean_loop_passes"] = float(d[:, 6].mean())
            r["mean_drops"] = float(d[:, 7].mean())
            r["loop_cycles_median"] = float(np.median(d[:, 0:6].sum(1)))
        rows.append(r)
        print(json.dumps(r), flush=True)
e.close()
