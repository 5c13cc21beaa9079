"""Cycles per sub-step of the default step's active-set loop (solve16), from the WBC_ISTAMPS build:
summed over the passes of segment 0 of each wave (lane 0 writes), reported per pass.
Usage (GPU box): WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so python tools/ist16.py [config] [B]"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrupedwholebodycontroller_amd import STATELESS, Engine, workloads

cfg = sys.argv[1] if len(sys.argv) > 1 else "stance_cold"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
inp = getattr(workloads, cfg)(B, seed=1 if cfg == "stance_cold" else 3)
e = Engine(B)
e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
for _ in range(3):
    e.step(STATELESS)
e.synchronize()
D = e.debug()[0::4]
passes = D[:, 6]
ok = passes > 0
names = ["chosen row's normal (LDS)", "d = J^T n, R^-1 d, z", "slack rates", "step lengths",
         "select + Householder add", "mirror (+ drop path)"]
tot = D[ok, 0:6].sum(0) / passes[ok].sum()
res = {n: round(float(v), 1) for n, v in zip(names, tot)}
res["per pass"] = round(float(tot.sum()), 1)
res["mean passes (segment 0)"] = float(passes[ok].mean())
res["mean drops"] = float(D[ok, 7].mean())
print(json.dumps(dict(config=cfg, batch=B, cycles_per_pass=res), indent=1))
