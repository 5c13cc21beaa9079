"""Per-phase cycle breakdown of wbc_step_kernel from the diagnostic stamps build.
Usage (GPU box): WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_stamps.so python tools/stamps.py [config] [B]"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrupedwholebodycontroller_amd import FUSED, STATELESS, Engine, workloads
from quadrupedwholebodycontroller_amd._capi import DBG

cfg = sys.argv[1] if len(sys.argv) > 1 else "stance_cold"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
inp = getattr(workloads, cfg)(B, seed=1)
e = Engine(B)
e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
for _ in range(3):
    e.step(STATELESS | FUSED)  # the stamps live in the fused kernel
e.synchronize()
d = e.debug()[:, DBG["STAMPS"]:DBG["STAMPS"] + 7]
names = ["update", "qp_setup(H_s chol, x0)", "normals+C0", "GI loop", "primal recovery", "outputs"]
dd = np.diff(d, axis=1)
res = {n: dict(median=float(np.median(dd[:, i])), mean=float(dd[:, i].mean()), p90=float(np.percentile(dd[:, i], 90)))
       for i, n in enumerate(names)}
res["total"] = dict(median=float(np.median(d[:, 6] - d[:, 0])), mean=float((d[:, 6] - d[:, 0]).mean()))
span = d[:, 6].max() - d[:, 0].min()
res["kernel_span_cycles"] = float(span)
out = e.outputs()
res["mean_iters"] = float(out["iters"].mean())
print(json.dumps(dict(config=cfg, batch=B, phases_cycles=res), indent=1))
