"""Generate the committed golden fixtures (tests/golden/*.npz) from the numpy oracle.

The reference repository holds no tests, fixtures or golden vectors, and
neither it nor its un-vendored iDynTree/qpOASES can be built here, so these fixtures come from
oracle/wbc_np.py (the fp64 restatement of src/whole_body_controller.cpp:256-577), after it has
passed the physics-identity checks in tests/test_oracle_physics.py.  They pin the oracle against
regressions and give the GPU tests fixed vectors.  Parity against the reference binary itself
remains unpinned.

Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import wbc_np as W  # noqa: E402
from quadrupedwholebodycontroller_amd import workloads  # noqa: E402

KEYS = ["com", "comvel", "pose", "vc", "M", "Cnu", "Jfeet", "pfeet", "vfeet", "Mbar_b", "Mbar_j", "Jbar", "bbar", "W",
        "r1", "rsw"]


def cold_case(name, inp):
    model, params = W.Model(), W.default_params()
    B = inp["base_pose"].shape[0]
    rec = {k: [] for k in KEYS}
    out = dict(tau=[], grf=[], x=[], status=[], iters=[], H=[], g=[], A=[], lbA=[], ubA=[])
    for b in range(B):
        c = W.ReferenceWBC(model, params)
        c.set_state(inp["base_pose"][b], inp["nu"][b], inp["qj"][b])
        c.set_reference(inp["ref"][b], [(int(inp["contacts"][b]) >> i) & 1 for i in range(4)], bool(inp["switching"][b]))
        tau, grf, x, st, it = c.step()
        d = c.debug_record()
        for k in KEYS:
            rec[k].append(np.asarray(d[k]))
        H, g, A, lb, ub = c.qp
        for k, v in (("tau", tau), ("grf", grf), ("x", x), ("status", st), ("iters", it), ("H", H), ("g", g),
                     ("A", A), ("lbA", lb), ("ubA", ub)):
            out[k].append(np.asarray(v))
    arrs = {f"in_{k}": v for k, v in inp.items()}
    arrs.update({f"dbg_{k}": np.stack(v) for k, v in rec.items()})
    arrs.update({f"out_{k}": np.stack(v) for k, v in out.items()})
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
    print(name, B, "status counts", np.bincount(np.array(out["status"]), minlength=4))


def trajectory_case(name, steps_iter, n_steps, robots):
    """Stateful multi-step case: history (finite differences, Tdot_inv lag, integral error) carried."""
    model, params = W.Model(), W.default_params()
    ctrls = [W.ReferenceWBC(model, params) for _ in robots]
    ins = {k: [] for k in ("base_pose", "nu", "qj", "ref", "contacts", "switching")}
    outs = dict(tau=[], x=[], status=[], bbar=[], r1=[], rsw=[])
    for k, inp in enumerate(steps_iter):
        if k >= n_steps:
            break
        for key in ins:
            ins[key].append(inp[key][robots])
        tr, xr, sr, br, r1r, rsr = [], [], [], [], [], []
        for j, b in enumerate(robots):
            c = ctrls[j]
            c.set_state(inp["base_pose"][b], inp["nu"][b], inp["qj"][b])
            c.set_reference(inp["ref"][b], [(int(inp["contacts"][b]) >> i) & 1 for i in range(4)],
                            bool(inp["switching"][b]))
            tau, grf, x, st, it = c.step()
            tr.append(tau); xr.append(x); sr.append(st); br.append(c.bbar.copy()); r1r.append(c.r1); rsr.append(c.rsw)
        for key, v in (("tau", tr), ("x", xr), ("status", sr), ("bbar", br), ("r1", r1r), ("rsw", rsr)):
            outs[key].append(np.array(v))
    arrs = {f"in_{k}": np.stack(v) for k, v in ins.items()}
    arrs.update({f"out_{k}": np.stack(v) for k, v in outs.items()})
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **arrs)
    print(name, "steps", n_steps, "robots", len(robots), "status counts",
          np.bincount(np.array(outs["status"]).ravel(), minlength=4))


def stance_hold_steps(n):
    """Config 1 stand-in: the reference's start-up (cpp:65-120 pose, base z 0.585) held still;
    the first cycle is the reference's real first cycle (switching false, T_old = I)."""
    B = 1
    for k in range(n):
        pose = np.zeros((B, 7)); pose[:, 2] = 0.585; pose[:, 6] = 1.0
        yield dict(base_pose=pose, nu=np.zeros((B, 18)), qj=np.tile(workloads.Q0, (B, 1)),
                   ref=np.tile(np.r_[workloads.REF_POSE, np.zeros(48)], (B, 1)),
                   contacts=np.full(B, 15, np.uint8), switching=np.zeros(B, np.uint8))


def main():
    cold_case("stance_cold", workloads.stance_cold(16, seed=101))
    cold_case("rl_random", workloads.rl_random(24, seed=103))
    # every contact mask, switching and non-switching
    inp = workloads.rl_random(32, seed=105)
    inp["contacts"] = np.tile(np.arange(16, dtype=np.uint8), 2)
    inp["switching"] = np.r_[np.ones(16, np.uint8), np.zeros(16, np.uint8)]
    cold_case("all_masks", inp)
    trajectory_case("traj_stance_hold", stance_hold_steps(40), 40, [0])
    trajectory_case("traj_trot", workloads.trot_sequence(2, steps=160, seed=2), 160, [0, 1])


if __name__ == "__main__":
    main()
