"""Cycles per phase of the four-contact stance solve (wbc_solve_stance_kernel), from the WBC_STAMPS
build.  Usage (GPU box): WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_stamps.so python tools/sstamps.py [B]"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrupedwholebodycontroller_amd import STATELESS, Engine, workloads
from quadrupedwholebodycontroller_amd._capi import DBG

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
inp = workloads.stance_cold(B, seed=1)
e = Engine(B)
e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
for _ in range(3):
    e.step(STATELESS)  # all-stance: update kernel, then the stance solve kernel
e.synchronize()
d = e.debug()[:, DBG["STAMPS"]:DBG["STAMPS"] + 6]
names = ["unpack + normals + slacks", "C0 = M n", "active-set loop", "primal", "outputs"]
dd = np.diff(d, axis=1)
res = {n: dict(median=float(np.median(dd[:, i])), mean=float(dd[:, i].mean()), p90=float(np.percentile(dd[:, i], 90)))
       for i, n in enumerate(names)}
res["total"] = dict(median=float(np.median(d[:, 5] - d[:, 0])))
res["kernel_span_cycles"] = float(d[:, 5].max() - d[:, 0].min())
start = np.sort(d[:, 0] - d[:, 0].min())
res["start_offsets_cycles"] = dict(p10=float(np.percentile(start, 10)), p50=float(np.percentile(start, 50)),
                                   p90=float(np.percentile(start, 90)), max=float(start.max()))
res["mean_iters"] = float(e.outputs()["iters"].mean())
print(json.dumps(dict(config="stance_cold", batch=B, stance_solve_cycles=res), indent=1))
