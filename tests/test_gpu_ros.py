"""GPU: a ROS-bytes control cycle.  Serialized ModelStates / JointState / WbcReferenceMsg in,
libwbc_ros.so decodes them into the engine's inputs, one step, torques out as Float64MultiArray
bytes.  Must equal the step fed with the arrays directly (bit-exact), for robots whose joint
order in JointState is shuffled and whose model is not first in ModelStates.
"""
import numpy as np
import pytest

from quadrupedwholebodycontroller_amd import STATELESS, Engine, workloads
from quadrupedwholebodycontroller_amd import ros_wire as RW
from test_ros_wire import JOINTS, REF_SIZES, f64ma, joint_state, model_states, ref_msg

pytestmark = pytest.mark.gpu


def test_ros_bytes_cycle_equals_array_cycle():
    B = 96
    inp = workloads.rl_random(B, seed=31)
    g = np.random.default_rng(0)
    ms, js, rs = [], [], []
    for b in range(B):
        names = ["ground_plane", "anymalModel"] if b % 2 else ["anymalModel"]
        poses = [np.zeros(7), inp["base_pose"][b]] if b % 2 else [inp["base_pose"][b]]
        tws = [np.zeros(6), inp["nu"][b, :6]] if b % 2 else [inp["nu"][b, :6]]
        ms.append(model_states(names, poses, tws))
        perm = g.permutation(12)
        js.append(joint_state([JOINTS[i] for i in perm], inp["qj"][b, perm], inp["nu"][b, 6 + perm], []))
        fields = np.split(inp["ref"][b], np.cumsum(REF_SIZES)[:-1])
        rs.append(ref_msg(fields, [(int(inp["contacts"][b]) >> i) & 1 for i in range(4)]))
    pose, nu = RW.decode_model_states(ms)
    qj, nu = RW.decode_joint_state(js, nu=nu)
    ref, con = RW.decode_reference(rs)

    e = Engine(B)
    e.set_state(pose, nu, qj)
    e.set_reference(ref, con, inp["switching"])
    e.step(STATELESS)
    via_ros = e.outputs()
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    e.step(STATELESS)
    direct = e.outputs()
    e.close()
    for k in ("tau", "grf", "status"):
        assert np.array_equal(via_ros[k], direct[k]), k
    msgs = RW.encode_float64_array(via_ros["tau"])
    assert all(m == f64ma(t) for m, t in zip(msgs, direct["tau"]))
