"""Diagnostic (GPU box): QP status and active-set iteration counts of the HIP engine against the
C oracle (oracle/wbc_ref.c, dense 42 x 70 Goldfarb-Idnani) on the same cold inputs."""
import json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import wbc_ref
from quadrupedwholebodycontroller_amd import STATELESS, Engine, default_params, workloads


def stress(B, seed):
    g = np.random.default_rng(seed)
    inp = workloads.rl_random(B, seed=seed)
    inp["qj"] = workloads.Q0 + g.uniform(-1.2, 1.2, (B, 12))
    inp["nu"] = g.normal(0.0, 2.0, (B, 18))
    inp["ref"][:, 12:18] = g.normal(0.0, 15.0, (B, 6))
    inp["ref"][:, 42:54] = g.normal(0.0, 40.0, (B, 12))
    inp["contacts"] = (np.arange(B) % 16).astype(np.uint8)
    return inp


cases = [("stance", workloads.stance_cold(1024, 1), {}), ("rl_random", workloads.rl_random(2048, 3), {}),
         ("stress80", stress(512, 51), dict(max_torque=80.0)), ("stress20", stress(512, 52), dict(max_torque=20.0)),
         ("stress6", stress(512, 53), dict(max_torque=6.0))]
res = {}
for name, inp, ov in cases:
    B = inp["base_pose"].shape[0]
    p = default_params()
    for k, v in ov.items():
        setattr(p, k, v)
    e = Engine(B, params=p)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    e.step(STATELESS)
    g = e.outputs()
    e.close()
    o = wbc_ref.run_batch(inp, **ov)
    d = g["iters"].astype(int) - o["iters"].astype(int)
    res[name] = dict(B=B, status_equal=int((g["status"] == o["status"]).sum()),
                     gpu_status=np.bincount(g["status"], minlength=4).tolist(),
                     ref_status=np.bincount(o["status"], minlength=4).tolist(),
                     iters_equal=int((d == 0).sum()), iters_diff_hist={int(k): int(v) for k, v in zip(*np.unique(d, return_counts=True))},
                     gpu_mean=float(g["iters"].mean()), ref_mean=float(o["iters"].mean()))
    print(name, json.dumps(res[name]), flush=True)
