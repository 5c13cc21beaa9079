"""Cycles per stage of the split-mode update kernel (four robots per wave), from the WBC_ISTAMPS
build.  The stamps are written by lane 0 of each wave, so only robots rb % 4 == 0 carry them.
Usage (GPU box): WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so python tools/ustamps.py [config] [B]"""
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
    e.step(STATELESS)  # default split form: update kernel, then solve kernel
e.synchronize()
u = e.debug()[0::4, 8:20]
un = ["inputs+sincos", "stage A (leg chains)", "stage B (bodies)", "Jf + CoM sums", "Ic sum+inv", "stage C (joints)",
      "hb sum, y, zeta, lane0", "Jbar/Mbar/bbar", "Tdot_inv", "bounds, wrench, history",
      "slot Cholesky (presolve) + store"]
du = np.diff(u, axis=1)
ok = (u > 0).all(1)
res = {n: float(np.median(du[ok, i])) for i, n in enumerate(un)}
res["total (stamps 0..11)"] = float(np.median(u[ok, -1] - u[ok, 0]))
# four-contact stance stage inside the presolve slot (stamps 12..14, written before stamp 11)
st = e.debug()[0::4, 20:23]
ok2 = ok & (st > 0).all(1)
s2 = e.debug()[0::4, 27:29]  # stamps 19, 20 inside the first stance stage
if ok2.any() and (s2[ok2] > 0).all():
    res["stance: leg inverses, W"] = float(np.median(s2[ok2, 0] - u[ok2, 10]))
    res["stance: S = I - K W"] = float(np.median(s2[ok2, 1] - s2[ok2, 0]))
    res["stance: S^-1 (Gauss-Jordan)"] = float(np.median(st[ok2, 0] - s2[ok2, 1]))
s3 = e.debug()[0::4, 29:31]  # stamps 21, 22 inside the second stance stage
if ok2.any() and (s3[ok2] > 0).all():
    res["stance: Y, q0"] = float(np.median(s3[ok2, 0] - st[ok2, 0]))
    res["stance: Q = Y^T Y"] = float(np.median(s3[ok2, 1] - s3[ok2, 0]))
    res["stance: H^, H_f row, g_f"] = float(np.median(st[ok2, 1] - s3[ok2, 1]))
f2 = e.debug()[0::4, 31:33]  # stamps 23, 24 inside factor12
if ok2.any() and (f2[ok2] > 0).all():
    res["factor: Cholesky"] = float(np.median(f2[ok2, 0] - st[ok2, 2]))
    res["factor: M = L^-1"] = float(np.median(f2[ok2, 1] - f2[ok2, 0]))
    res["factor: f0"] = float(np.median(u[ok2, 11] - f2[ok2, 1]))
if ok2.any():
    res["stance: Gauss-Jordan"] = float(np.median(st[ok2, 0] - u[ok2, 10]))
    res["stance: H_f row"] = float(np.median(st[ok2, 1] - st[ok2, 0]))
    res["stance: Nt, t0, stores"] = float(np.median(st[ok2, 2] - st[ok2, 1]))
    res["stance: factor H_f + stores"] = float(np.median(u[ok2, 11] - st[ok2, 2]))
# inline stance solve (wbc_update_solve_kernel, stateless all-stance steps): stamps 15..18 after 11
il = e.debug()[0::4, 23:27]
ok3 = ok & (il > 0).all(1)
if ok3.any():
    res["inline: normals + C0"] = float(np.median(il[ok3, 0] - u[ok3, 11]))
    res["inline: active-set loop"] = float(np.median(il[ok3, 1] - il[ok3, 0]))
    res["inline: primal"] = float(np.median(il[ok3, 2] - il[ok3, 1]))
    res["inline: outputs"] = float(np.median(il[ok3, 3] - il[ok3, 2]))
    out = e.outputs()
    wave_iters = out["iters"][: (B // 4) * 4].reshape(-1, 4).max(1)
    res["inline: loop cycles per wave iteration"] = float(np.median((il[ok3, 1] - il[ok3, 0]) /
                                                                   np.maximum(wave_iters[ok3] + 1, 1)))
    res["inline: mean max-over-wave iters"] = float(wave_iters.mean())
    res["inline: mean iters"] = float(out["iters"].mean())
res["robots sampled"] = int(ok.sum())
print(json.dumps(dict(config=cfg, batch=B, split_update_cycles=res), indent=1))
