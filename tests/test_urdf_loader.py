"""CPU: wbc_model_from_urdf (C++ run-time URDF loader) against the Python
generator tools/gen_model.py on synthetic quadruped URDFs (different names, extra fixed links,
rotated joint frames, off-axis inertials), against the committed ANYmal constants when the
reference URDF is present in this container, and its error paths.
"""
import ctypes as C
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import gen_model  # noqa: E402

from quadrupedwholebodycontroller_amd import WbcError, anymal_model, model_from_urdf  # noqa: E402

REF_URDF = "/root/reference/urdf/anymal.urdf"


def _f(v):
    return " ".join(repr(float(x)) for x in v)


def synthetic_urdf(path, seed, legs=("FL", "FR", "HL", "HR"), joints=("hip_roll", "hip_pitch", "knee"),
                   foot="toe"):
    """A 12-DoF quadruped in URDF: base with a fixed IMU link, per leg 3 revolute links, a fixed
    foot frame and a fixed cover plate on the thigh; random masses, inertias and frames."""
    g = np.random.default_rng(seed)

    def inertial(m):
        A = g.normal(size=(3, 3))
        I = (A @ A.T * 0.01 + np.eye(3) * 0.02).tolist()
        m = float(m)
        return (f'<inertial><origin xyz="{_f(g.uniform(-0.05, 0.05, 3))}" rpy="{_f(g.uniform(-0.3, 0.3, 3))}"/>'
                f'<mass value="{m!r}"/><inertia ixx="{I[0][0]!r}" ixy="{I[0][1]!r}" ixz="{I[0][2]!r}" '
                f'iyy="{I[1][1]!r}" iyz="{I[1][2]!r}" izz="{I[2][2]!r}"/></inertial>')

    out = ['<?xml version="1.0"?>', "<!-- synthetic quadruped for the loader test -->", '<robot name="synth">',
           f'<link name="trunk">{inertial(g.uniform(10, 30))}</link>',
           f'<link name="imu">{inertial(0.2)}</link>',
           f'<joint name="imu_joint" type="fixed"><parent link="trunk"/><child link="imu"/>'
           f'<origin xyz="0.1 0 0.05" rpy="0 0 0.3"/></joint>']
    for i, leg in enumerate(legs):
        sx, sy = (1 if i < 2 else -1), (1 if i % 2 == 0 else -1)
        parent = "trunk"
        for k, jn in enumerate(joints):
            link = f"{leg}_link{k}"
            out.append(f'<link name="{link}">{inertial(g.uniform(0.3, 3))}</link>')
            xyz = [0.3 * sx, 0.1 * sy, 0.0] if k == 0 else ([0.05, 0.0, 0.0] if k == 1 else [0.0, 0.05 * sy, -0.3])
            out.append(f'<joint name="{leg}_{jn}" type="revolute"><parent link="{parent}"/><child link="{link}"/>'
                       f'<origin xyz="{_f(xyz)}" rpy="{_f(g.uniform(-0.2, 0.2, 3))}"/>'
                       f'<axis xyz="{_f([1, 0, 0] if k == 0 else [0, 1, 0])}"/>'
                       f'<limit lower="-3" upper="3" effort="80" velocity="10"/></joint>')
            if k == 1:  # a fixed cover plate on the thigh
                out.append(f'<link name="{leg}_cover">{inertial(0.15)}</link>')
                out.append(f'<joint name="{leg}_cover_joint" type="fixed"><parent link="{link}"/>'
                           f'<child link="{leg}_cover"/><origin xyz="0 0.02 -0.1" rpy="0.1 0 0"/></joint>')
            parent = link
        out.append(f'<link name="{leg}_{foot}"/>')
        out.append(f'<joint name="{leg}_{foot}_joint" type="fixed"><parent link="{parent}"/>'
                   f'<child link="{leg}_{foot}"/><origin xyz="0.01 0 -0.32"/></joint>')
    out.append("</robot>")
    with open(path, "w") as fh:
        fh.write("\n".join(out))


def model_array(m):
    return np.frombuffer(bytes(C.string_at(C.addressof(m), C.sizeof(m))), np.float64)


def python_model_array(d):
    v = [d["base"]["mass"], *d["base"]["com"], *np.ravel(d["base"]["inertia"])]
    for leg in d["legs"]:
        for lk in leg:
            v += [*np.ravel(lk["R"]), *lk["p"], *lk["axis"], lk["mass"], *lk["com"], *np.ravel(lk["inertia"])]
    v += [*np.ravel(d["foot"]), d["total_mass"]]
    return np.array(v)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_loader_matches_python_generator(tmp_path, seed):
    legs, joints, foot = ("FL", "FR", "HL", "HR"), ("hip_roll", "hip_pitch", "knee"), "toe"
    p = str(tmp_path / "q.urdf")
    synthetic_urdf(p, seed, legs, joints, foot)
    links, js = gen_model.load_urdf(p)
    d = gen_model.build(links, js, leg_order=list(legs), joint_suffix=list(joints), foot_suffix=foot)
    m = model_from_urdf(p, legs=legs, joints=joints, foot_suffix=foot)
    a, b = model_array(m), python_model_array(d)
    assert a.shape == b.shape
    assert np.max(np.abs(a - b) / np.maximum(1.0, np.abs(b))) < 1e-13


def test_loader_reproduces_committed_anymal_model():
    if not os.path.exists(REF_URDF):
        pytest.skip("reference URDF not in this container")
    assert np.array_equal(model_array(model_from_urdf(REF_URDF)), model_array(anymal_model()))


def test_loader_errors(tmp_path):
    with pytest.raises(WbcError, match="cannot open"):
        model_from_urdf(str(tmp_path / "missing.urdf"))
    p = str(tmp_path / "q.urdf")
    synthetic_urdf(p, 4)
    with pytest.raises(WbcError, match="does not leave the base"):
        model_from_urdf(p)  # default names LH_HAA ... are not in this robot
    with pytest.raises(WbcError, match="not in the last body"):
        model_from_urdf(p, legs=("FL", "FR", "HL", "HR"), joints=("hip_roll", "hip_pitch", "knee"))  # foot: FOOT
    bad = str(tmp_path / "bad.urdf")
    with open(bad, "w") as fh:
        fh.write('<robot name="x"><link name="a"></robot>')
    with pytest.raises(WbcError):
        model_from_urdf(bad)


def test_loader_rejects_malformed_numbers_and_extra_chains(tmp_path):
    """Malformed attributes are errors, not silent zeros (no exception escapes the C-ABI: the
    process survives and WbcError carries the message); chains the lumped model cannot hold
    (an extra moving joint off the base or mid-leg) are refused instead of dropping their mass."""
    import re

    names = dict(legs=("FL", "FR", "HL", "HR"), joints=("hip_roll", "hip_pitch", "knee"), foot_suffix="toe")
    p = str(tmp_path / "q.urdf")
    synthetic_urdf(p, 5, names["legs"], names["joints"], names["foot_suffix"])
    good = open(p).read()
    model_from_urdf(p, **names)  # the unmodified robot loads

    def bad(text, match):
        q = str(tmp_path / "bad.urdf")
        with open(q, "w") as fh:
            fh.write(text)
        with pytest.raises(WbcError, match=match):
            model_from_urdf(q, **names)

    bad(re.sub(r'<mass value="[^"]*"', '<mass value="abc"', good, count=1), "malformed number")
    bad(re.sub(r'<origin xyz="[^"]*"', '<origin xyz="0.1 0.2"', good, count=1), "must hold 3")
    bad(re.sub(r'rpy="[^"]*"', 'rpy="0 0 0 x"', good, count=1), "malformed number")
    bad(re.sub(r'<axis xyz="[^"]*"', '<axis xyz="0 0 0"', good, count=1), "zero joint axis")
    bad(re.sub(r'<axis xyz="[^"]*"', '<axis xyz="1 0"', good, count=1), "must hold 3")
    m = re.search(r'<joint name="FL_hip_roll".*?</joint>', good, re.S)
    root = re.search(r'<parent link="([^"]+)"', m.group(0)).group(1)
    arm = (f'<link name="arm"><inertial><mass value="2.0"/><inertia ixx="0.1" ixy="0" ixz="0" iyy="0.1" iyz="0" '
           f'izz="0.1"/></inertial></link><joint name="arm_joint" type="revolute"><parent link="{root}"/>'
           f'<child link="arm"/><axis xyz="0 0 1"/></joint></robot>')
    bad(good.replace("</robot>", arm), "moving joints leave the base")
    thigh = re.search(r'<child link="([^"]+)"', re.search(r'<joint name="FL_hip_pitch".*?</joint>', good, re.S)
                      .group(0)).group(1)
    extra = arm.replace(f'<parent link="{root}"/>', f'<parent link="{thigh}"/>')
    bad(good.replace("</robot>", extra), "moving child joints")
