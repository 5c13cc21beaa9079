"""Cycles per stage of the default step kernel (wbc_update_solve_kernel: four QPs per wave, each
reduced to 12 variables and solved in its 16-lane segment), from the WBC_ISTAMPS build: medians over
waves (lane 0 of each wave writes the stamps, so only QPs qp % 4 == 0 carry them).
Usage (GPU box): WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so python tools/ust16.py [config] [B]
(config: a stateless workloads generator, or trot: configs[2]'s stateful trot, its 60th cycle;
WBC_UST_NOX=1 steps with WBC_NO_X, as bench.py does)"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrupedwholebodycontroller_amd import NO_X, STATELESS, Engine, workloads

cfg = sys.argv[1] if len(sys.argv) > 1 else "stance_cold"
XF = NO_X if os.environ.get("WBC_UST_NOX") else 0
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
e = Engine(B)
if cfg == "trot":  # configs[2]: stateful (history, hotstart), the stamps of its 60th cycle
    for k, s in enumerate(workloads.trot_sequence(B, steps=60, seed=2)):
        e.set_state(s["base_pose"], s["nu"], s["qj"])
        e.set_reference(s["ref"], s["contacts"], s["switching"])
        e.step(XF)
else:
    inp = getattr(workloads, cfg)(B, seed=1 if cfg == "stance_cold" else 3)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    for _ in range(3):
        e.step(STATELESS | XF)
e.synchronize()
D = e.debug()[0::4]
st = lambda i: D[:, 8 + i]  # UST(i)
res = {}
u = np.stack([st(i) for i in range(11)], 1)
ok = (u > 0).all(1)
names = ["inputs+sincos", "stage A (leg chains)", "stage B (bodies)", "Jf + CoM sums", "Ic sum+inv", "stage C (joints)",
         "hb sum, y, zeta, lane0", "Jbar/Mbar/bbar", "Tdot_inv", "bounds, wrench, history"]
for i, n in enumerate(names):
    res[n] = float(np.median(u[ok, i + 1] - u[ok, i]))
t10, t11 = st(10), st(11)
# the stance form stamps 19 (stance_reduce's leg inverses) inside its own reduce; the general form never
stn = ok & (st(19) > t10) & (st(19) < t11)
gen = ok & ~stn & (st(20) > t10)
def med(a, b, m):
    return float(np.median(b[m] - a[m])) if m.any() else None
res["general: R1-R4 (leg inverses, S6, S6^-1, Y, B, v, rho0)"] = med(t10, st(20), gen)
res["general: R5 (V, gamma, o, blk)"] = med(st(20), st(21), gen)
res["general: R6 (H rows, g)"] = med(st(21), st(22), gen)
res["general: R7 factor12 + R8 Nt"] = med(st(22), st(14), gen)
res["general:   R7 factor12"] = med(st(22), st(23), gen)
res["general:   R8 Nt"] = med(st(23), st(14), gen)
res["prologue (kernel entry -> update start: model staging, input loads)"] = float(np.median((st(0) - st(30))[ok]))
res["stance: reduce + rank-6 factor"] = med(t10, t11, stn)
for n, (i0, i1) in (("leg inverses, W", (None, 19)), ("S", (19, 20)), ("S^-1", (20, 12)), ("Y, q0", (12, 21)),
                    ("Q = Y^T Y", (21, 22)), ("H^, g_f", (22, 13)), ("Nt, t0", (13, 14)), ("rank-6 factor", (14, 11))):
    res[f"stance:   {n}"] = med(t10 if i0 is None else st(i0), st(i1), stn)
for tag, m in (("general", gen), ("stance", stn)):
    if not m.any():
        continue
    res[f"{tag}: solve setup (normals, slacks, J)"] = med(t11, st(15), m)
    res[f"{tag}: active-set loop"] = med(st(15), st(16), m)
    res[f"{tag}:   hotstart block (warm re-adds, point, slacks)"] = med(st(15), st(25), m)
    res[f"{tag}:   selection + loop passes"] = med(st(25), st(16), m)
    # the loop's sub-steps summed over its passes (IST slots 0..5, lane 0 of the wave)
    for i, n in enumerate(["normal row", "direction (d, R^-1 d, z)", "slack rates", "step lengths",
                           "select + Householder add", "mirror (+ drop path)"]):
        res[f"{tag}:   loop: {n}"] = float(np.median(D[m, i]))
    res[f"{tag}:   loop: passes, drops (mean per wave)"] = [float(D[m, 6].mean()), float(D[m, 7].mean())]
    res[f"{tag}: primal + outputs"] = med(st(16), st(18), m)
    res[f"{tag}: total"] = med(st(0), st(18), m)
    res[f"{tag}: entry to end"] = med(st(30), st(18), m)
    res[f"{tag}: entry to end, max over waves"] = float(np.max((st(18) - st(30))[m]))
out = e.outputs()
wi = out["iters"][: (B // 4) * 4].reshape(-1, 4).max(1)
res["mean max-over-wave iters"] = float(wi.mean())
res["mean iters"] = float(out["iters"].mean())
loop = st(16) - st(15)
res["loop cycles per pass (passes = max iters + 1)"] = float(np.median(loop[ok] / (wi[ok] + 1)))
res["waves sampled (general, stance)"] = [int(gen.sum()), int(stn.sum())]
print(json.dumps(dict(config=cfg, batch=B, cycles=res), indent=1))
