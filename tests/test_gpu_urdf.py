"""GPU: the engine built from a run-time-loaded URDF (wbc_model_from_urdf, a synthetic quadruped
with its own names, fixed links and frames) against the numpy oracle given the same robot through
tools/gen_model.py. Same tolerances as test_gpu_parity.py.
"""
import json
import os
import sys

import numpy as np
import pytest

import wbc_np as W
from quadrupedwholebodycontroller_amd import DEBUG, STATELESS, Engine, model_from_urdf, workloads
from test_gpu_parity import check_robot
from test_urdf_loader import synthetic_urdf

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import gen_model  # noqa: E402

pytestmark = pytest.mark.gpu

LEGS, JOINTS, FOOT = ("FL", "FR", "HL", "HR"), ("hip_roll", "hip_pitch", "knee"), "toe"


def test_engine_on_loaded_urdf_matches_oracle(tmp_path):
    p = str(tmp_path / "q.urdf")
    synthetic_urdf(p, 7, LEGS, JOINTS, FOOT)
    links, js = gen_model.load_urdf(p)
    d = gen_model.build(links, js, leg_order=list(LEGS), joint_suffix=list(JOINTS), foot_suffix=FOOT)
    jp = str(tmp_path / "q.json")
    with open(jp, "w") as fh:
        json.dump(d, fh)
    oracle_model, params = W.Model(jp), W.default_params()

    B = 128
    inp = workloads.rl_random(B, seed=21)
    e = Engine(B, model=model_from_urdf(p, legs=LEGS, joints=JOINTS, foot_suffix=FOOT))
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    e.step(STATELESS | DEBUG)
    out = e.outputs()
    out["dbg"] = e.debug()
    e.close()
    for b in range(B):
        c = W.ReferenceWBC(oracle_model, params)
        c.set_state(inp["base_pose"][b], inp["nu"][b], inp["qj"][b])
        c.set_reference(inp["ref"][b], [(int(inp["contacts"][b]) >> i) & 1 for i in range(4)],
                        bool(inp["switching"][b]))
        c.step()
        check_robot(c, out, b)
    assert np.any(out["status"] == W.QP_OK)
