"""GPU parity: the HIP engine (through the C-ABI) against the numpy oracle of the reference path.

Tolerances (fp64 everywhere; tests/margins.py, tightened in round 4; 6-53x the worst error
measured on MI355X in round 5, profiles/r05/parity_margins.json, well inside BASELINE.md's parity gate):
  intermediates (M, C nu, Jacobians, CoM, Mbar, Jbar, bbar, wrench, bounds): 1e-13 relative to
    max(1, |value|) (W 5e-12, Mbar_b and rsw 1e-12; the kinematics, Jbar and Mbar_j 1e-14) -- the kernel uses closed forms instead of the
    reference's dense LU inverses, so agreement is to rounding, not bitwise;
  x*  within 1e-9 * (1 + |x*|_inf);   tau within 1e-9 * (1 + |tau|_inf);  grf 2e-11;
  QP status identical.
"""
import numpy as np

import margins as M
import pytest

import wbc_np as W
from quadrupedwholebodycontroller_amd import DEBUG, FUSED, SPLIT, STATELESS, Engine, split_debug, workloads

pytestmark = pytest.mark.gpu

MODEL = W.Model()
PARAMS = W.default_params()


def oracle_batch(inp, idx):
    out = []
    for b in idx:
        c = W.ReferenceWBC(MODEL, PARAMS)
        c.set_state(inp["base_pose"][b], inp["nu"][b], inp["qj"][b])
        kap = [(int(inp["contacts"][b]) >> i) & 1 for i in range(4)]
        c.set_reference(inp["ref"][b], kap, bool(inp["switching"][b]))
        c.step()
        out.append(c)
    return out


def run_engine(inp, flags=STATELESS | DEBUG):
    B = inp["base_pose"].shape[0]
    e = Engine(B)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    e.step(flags)
    out = e.outputs()
    out["dbg"] = e.debug()
    e.close()
    return out


def rel_err(a, b):
    return np.max(np.abs(np.asarray(a) - np.asarray(b)) / np.maximum(1.0, np.abs(np.asarray(b))))


def check_robot(ctrl, out, b):
    d = split_debug(out["dbg"][b])
    ref = ctrl.debug_record()
    for k in ("com", "comvel", "pose", "vc", "M", "Cnu", "Jfeet", "pfeet", "vfeet", "Mbar_b", "Mbar_j", "Jbar",
              "W", "r1", "rsw"):
        tol = M.INTERMEDIATE.get(k, 1e-13)
        assert M.record(k, rel_err(d[k], ref[k]), tol) < tol, (b, k, rel_err(d[k], ref[k]))
    assert M.record("bbar", rel_err(d["bbar"][6:], ref["bbar"][6:]), 1e-13) < 1e-13, (b, "bbar")
    assert out["status"][b] == ctrl.qp_status, (b, out["status"][b], ctrl.qp_status)
    if ctrl.qp_status == W.QP_OK:
        assert M.close(out["x"][b], ctrl.qp_solution, M.X, "x"), (b, "x")
        assert M.close(out["tau"][b], ctrl.tau, M.TAU, "tau"), (b, "tau")
        assert M.close(out["grf"][b], ctrl.grf, M.GRF, "grf"), (b, "grf")


def test_stance_cold_parity():
    inp = workloads.stance_cold(256, seed=11)
    out = run_engine(inp)
    ctrls = oracle_batch(inp, range(256))
    for b, c in enumerate(ctrls):
        check_robot(c, out, b)


def test_random_modes_parity():
    inp = workloads.rl_random(256, seed=12)
    out = run_engine(inp)
    ctrls = oracle_batch(inp, range(256))
    for b, c in enumerate(ctrls):
        check_robot(c, out, b)
    # the mix must exercise swing legs, active inequalities and infeasible cases
    assert len(set(int(k) for k in inp["contacts"])) == 16


def test_update_solve_split_equals_fused():
    inp = workloads.rl_random(512, seed=13)
    B = 512
    e = Engine(B)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    e.step(STATELESS | FUSED)  # one fused kernel
    fused = e.outputs()
    e.update(STATELESS)
    e.solve(STATELESS)
    split = e.outputs()
    e.step(STATELESS | SPLIT)  # update kernel + solve kernel
    step = e.outputs()
    e.close()
    # WBC_SPLIT and wbc_update + wbc_solve run the same kernels: bitwise.  The fused kernel (one robot
    # per wave, 2 waves per SIMD) keeps round 3's J-bar / M-bar stage code, whose stores sit inside
    # its loops (the batched form of the 16-lane update spills there), and the compiler fuses that
    # code's multiply-adds differently: general rows agree to rounding, with the same status and
    # working-set changes.  Four-contact stance rows take the force-space solve in the split form
    # and the 24-variable solve in the fused kernel: the same QP, agreement to rounding.
    st = inp["contacts"] == 15
    assert st.any() and (~st).any()
    for k in ("tau", "grf", "x", "status", "iters"):
        assert np.array_equal(step[k], split[k]), k
    assert np.array_equal(fused["status"], split["status"])
    assert M.record("iters mismatch fraction (fused vs split)", np.mean(fused["iters"] != split["iters"]), 0.0) == 0.0
    ok = split["status"] == 0
    for rows, tag, tols in ((~st & ok, "general", (M.BITS * 10, M.BITS, M.BITS)), (st & ok, "stance", (M.BITS, M.BITS, M.BITS))):
        for k, tol in zip(("tau", "grf", "x"), tols):
            assert M.close(fused[k][rows], split[k][rows], tol, f"{k} fused vs split ({tag} rows)"), (k, tag)


def test_half_turn_poses_match_oracle():
    """Base orientations whose rotation matrix has exact zeros where the RPY angles read it: half turns
    about z, x and y and their compositions (quaternions with entries in {0, +-1}, and two tilted
    yaws of pi).  At a half turn atan2 sees (+-0, x < 0): the engine's sign of that zero must give
    the oracle's angle (atan2_br and -fno-signed-zeros), or the pose error flips by 2 pi.
    Checked on the pose intermediate and the whole step."""
    base = workloads.stance_cold(12, seed=31)
    s = np.sqrt(0.5)
    quats = [(0, 0, 1, 0), (1, 0, 0, 0), (0, 1, 0, 0), (0, 0, -1, 0), (-1, 0, 0, 0), (0, -1, 0, 0),
             (0, 0, 0, 1), (0, 0, 0, -1), (0, s, s, 0), (s, 0, 0, s), (0.1, 0, 0.99498743710662, 0),
             (0, 0.1, 0.99498743710662, 0)]  # (no pitch of +-pi/2: roll and yaw are rounding noise there)
    for b, q in enumerate(quats):
        base["base_pose"][b, 3:7] = q
    out = run_engine(base)
    ctrls = oracle_batch(base, range(len(quats)))
    for b, c in enumerate(ctrls):
        check_robot(c, out, b)
