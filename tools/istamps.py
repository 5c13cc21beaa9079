"""Cycles per sub-step of the active-set loop (summed over iterations), from the WBC_ISTAMPS build.
Usage (GPU box): WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so python tools/istamps.py [config] [B]"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrupedwholebodycontroller_amd import FUSED, STATELESS, Engine, workloads

cfg = sys.argv[1] if len(sys.argv) > 1 else "stance_cold"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
inp = getattr(workloads, cfg)(B, seed=1 if cfg == "stance_cold" else 3)
e = Engine(B)
e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
for _ in range(3):
    e.step(STATELESS | FUSED)  # the stamps live in the fused kernel
e.synchronize()
d = e.debug()[:, 0:6]
out = e.outputs()
names = ["selection", "column broadcast", "Rinv d, n^T z, |z|^2", "step/multipliers", "Householder update",
         "bookkeeping+barrier+drop"]
it = out["iters"].astype(float)
res = {n: dict(median=float(np.median(d[:, i])), mean=float(d[:, i].mean())) for i, n in enumerate(names)}
res["total"] = float(np.median(d.sum(1)))
res["mean_iters"] = float(it.mean())
cnt = e.debug()[:, 6:8]
res["mean_loop_passes"] = float(cnt[:, 0].mean())  # adds + drops + rebuild re-adds
res["mean_drops"] = float(cnt[:, 1].mean())
print(json.dumps(dict(config=cfg, batch=B, loop_cycles=res), indent=1))
u = e.debug()[:, 8:19]
un = ["inputs+sincos", "stage A (leg chains)", "stage B (bodies)", "Jf + CoM sums", "Ic sum+inv", "stage C (joints)",
      "hb sum, y, zeta, lane0", "Jbar/Mbar/bbar", "Tdot_inv", "bounds, wrench, history"]
du = np.diff(u, axis=1)
print(json.dumps({n: float(np.median(du[:, i])) for i, n in enumerate(un)}, indent=1))
q = e.debug()[:, 20:25]
qn = ["eq fast path (Householder)", "eq generic path", "R/s to LDS + substitutions", "u, R^-1 rows, slacks"]
dq = np.diff(q, axis=1)
print(json.dumps({n: float(np.median(dq[:, i])) for i, n in enumerate(qn)}, indent=1))
n = e.debug()[:, 25:29]
nn = ["build_normal", "norms", "to_column"]
dn = np.diff(n, axis=1)
print(json.dumps({k: float(np.median(dn[:, i])) for i, k in enumerate(nn)}, indent=1))
