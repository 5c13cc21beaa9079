"""Synthetic inputs for the BASELINE.json configurations, numpy PCG64, fp64.

Arrays are robot-major per quantity, exactly the C-ABI layout (include/wbc.h):
  base_pose [B,7] = (px,py,pz,qx,qy,qz,qw), nu [B,18], qj [B,12], ref [B,54] (WbcReferenceMsg order),
  contacts [B] uint8 bitmask (bit i = leg i, LH,LF,RF,RH), switching [B] uint8.
"""
from __future__ import annotations

import numpy as np

Q0 = np.array([0.0, -0.4, 0.8, 0.0, 0.4, -0.8, 0.0, 0.4, -0.8, 0.0, -0.4, 0.8])  # cpp:81
REF_POSE = np.array([0.0, 0.0, 0.50, 0.0, 0.0, 0.0])  # params_controller.yaml:12
BASE_Z = 0.585
# nominal foot positions at Q0 with the base at (0, 0, 0.585) (FK of the lumped model)
FEET0 = np.array([[-0.506953, 0.31775, 0.0], [0.506953, 0.31775, 0.0], [0.506953, -0.31775, 0.0],
                  [-0.506953, -0.31775, 0.0]])


def rpy_to_quat(rpy):
    """(roll, pitch, yaw) [...,3] -> quaternion (x, y, z, w) [...,4], R = Rz Ry Rx."""
    r, p, y = (np.asarray(rpy)[..., i] / 2 for i in range(3))
    cr, sr, cp, sp, cy, sy = np.cos(r), np.sin(r), np.cos(p), np.sin(p), np.cos(y), np.sin(y)
    return np.stack([sr * cp * cy - cr * sp * sy, cr * sp * cy + sr * cp * sy,
                     cr * cp * sy - sr * sp * cy, cr * cp * cy + sr * sp * sy], axis=-1)


def _ref_nominal(B):
    ref = np.zeros((B, 54))
    ref[:, 0:6] = REF_POSE
    return ref


def stance_cold(B=4096, seed=1):
    """Config 2: 4-contact stance, every solve cold (switching=1: derivative terms 0)."""
    g = np.random.default_rng(seed)
    pose = np.zeros((B, 7))
    pose[:, 0:3] = np.array([0, 0, BASE_Z]) + g.uniform(-0.02, 0.02, (B, 3))
    pose[:, 3:7] = rpy_to_quat(g.uniform(-0.05, 0.05, (B, 3)))
    qj = Q0 + g.uniform(-0.05, 0.05, (B, 12))
    nu = g.normal(0.0, 0.1, (B, 18))
    return dict(base_pose=pose, nu=nu, qj=qj, ref=_ref_nominal(B), contacts=np.full(B, 15, np.uint8),
                switching=np.ones(B, np.uint8))


# Knee angle per leg at which the leg is stretched straight: its 3 x 3 foot Jacobian is singular
# (|det| / max|J|^3 ~ 1e-13, whatever the hip angles; found by bisection on the lumped model).
KNEE_STRAIGHT = np.array([-1.0, 1.0, 1.0, -1.0]) * 0.249494035113


def straight_legs(inp, every=5):
    """A copy of `inp` with one leg (leg b % 4) stretched straight on every `every`-th robot: the
    stance elimination / 12-variable reduction is not usable there (the engine's fallback solve)."""
    out = {k: np.array(v, copy=True) for k, v in inp.items()}
    for b in range(0, len(out["qj"]), every):
        out["qj"][b, 3 * (b % 4) + 2] = KNEE_STRAIGHT[b % 4]
    return out


def rl_random(B=65536, seed=3):
    """Config 4: randomized RL-style batch, contacts uniform over the 16 masks, cold."""
    g = np.random.default_rng(seed)
    pose = np.zeros((B, 7))
    pose[:, 0:2] = g.uniform(-0.02, 0.02, (B, 2))
    pose[:, 2] = g.uniform(0.45, 0.65, B)
    pose[:, 3:7] = rpy_to_quat(g.uniform(-0.3, 0.3, (B, 3)))
    qj = Q0 + g.uniform(-0.4, 0.4, (B, 12))
    nu = g.normal(0.0, 0.5, (B, 18))
    ref = _ref_nominal(B)
    ref[:, 0:3] += g.uniform(-0.02, 0.02, (B, 3))
    ref[:, 6:18] = g.normal(0.0, 0.05, (B, 12))
    ref[:, 18:30] = (FEET0 + np.array([0, 0, 0.03])).ravel() + g.uniform(-0.02, 0.02, (B, 12))
    ref[:, 30:54] = g.normal(0.0, 0.1, (B, 24))
    return dict(base_pose=pose, nu=nu, qj=qj, ref=ref, contacts=g.integers(0, 16, B).astype(np.uint8),
                switching=np.ones(B, np.uint8))


def mode_hypotheses(n_states=8192, seed=4):
    """Config 5: every state solved under all 16 contact masks (state-major, mask fastest)."""
    base = rl_random(n_states, seed)
    rep = {k: np.repeat(v, 16, axis=0) for k, v in base.items()}
    rep["contacts"] = np.tile(np.arange(16, dtype=np.uint8), n_states)
    return rep


def mode_states(n_states=8192, seed=4):
    """Config 5 for wbc_set_modes / wbc_step_modes: the n_states states of mode_hypotheses (one input
    row each) and the 16 contact masks; QP s * 16 + k of the engine equals row s * 16 + k of
    mode_hypotheses(n_states, seed)."""
    return rl_random(n_states, seed), np.arange(16, dtype=np.uint8)


def modes16(B=16384, seed=4):
    """Config 5 shard of B QPs: B // 16 states, each under all 16 contact masks."""
    return mode_hypotheses(B // 16, seed)


TROT_PERIOD_STEPS = 100  # 0.25 s at 400 Hz per half-cycle


def trot_sequence(B=4096, steps=400, seed=2, loop_rate=400.0):
    """Config 3 generator: yields per-step inputs of a trot, with the contact mask alternating
    LH+RF (0b0101) / LF+RH (0b1010) every 0.25 s and swing references lifted 5 cm."""
    g = np.random.default_rng(seed)
    phase = g.uniform(0, 2 * np.pi, B)
    prev = np.full(B, 15, np.uint8)
    for k in range(steps):
        t = k / loop_rate
        w = 2 * np.pi * 2.0
        s = np.sin(w * t + phase)[:, None]
        c = np.cos(w * t + phase)[:, None]
        qj = Q0 + 0.1 * s
        qd = 0.1 * w * c * np.ones((1, 12))
        pose = np.zeros((B, 7))
        pose[:, 2] = BASE_Z + 0.01 * s[:, 0]
        pose[:, 6] = 1.0
        nu = np.zeros((B, 18))
        nu[:, 2] = 0.01 * w * c[:, 0]
        nu[:, 6:] = qd
        half = (k // TROT_PERIOD_STEPS) % 2
        mask = 0b0101 if half == 0 else 0b1010
        contacts = np.full(B, mask, np.uint8)
        sphase = (k % TROT_PERIOD_STEPS) / TROT_PERIOD_STEPS
        ref = _ref_nominal(B)
        feet = FEET0.copy()
        for l in range(4):
            if not (mask >> l) & 1:
                feet[l, 2] += 0.05 * np.sin(np.pi * sphase)
        ref[:, 18:30] = feet.ravel()
        switching = (contacts != prev).astype(np.uint8)
        prev = contacts
        yield dict(base_pose=pose, nu=nu, qj=qj, ref=ref, contacts=contacts, switching=switching)


CONFIGS = {
    "stance_cold_b4096": lambda: stance_cold(4096, 1),
    "rl_random_b65536": lambda: rl_random(65536, 3),
    "modes16_x8192": lambda: mode_hypotheses(8192, 4),
}
