"""GPU parity at the bench's own sizes (BASELINE configs[1], configs[2] as bench.py times it, the
configs[3] shard and its global batch on one GPU, the configs[4] shard).

At B = 4096 and more the solve kernel runs several occupancy passes (8 robots per CU x 256 CUs
per pass); the smaller parity tests fit in one.  Each test runs the full batch once, then:

  * compares a stratified sample of >= 512 rows against the C oracle (oracle/wbc_ref.c): rows
    spread over the whole batch, every pass boundary (multiples of 2048) and the last robot;
    identical QP status (the literal 42 x 70 QP) and iteration counts (the oracle's REDUCED
    method, the 12-variable form the default step solves), x* / tau at the tolerances of
    test_gpu_parity.py;
  * re-runs the sampled rows as a small batch and requires bit-identical outputs (a robot's
    result does not depend on where in the grid, in which pass or next to which robots it ran: each
    QP's form follows from its own mask, and the wave map only decides who shares a wave,
    DESIGN.md 4.11).
"""
import numpy as np
import pytest

import margins as M
import wbc_ref as R
from quadrupedwholebodycontroller_amd import STATELESS, Engine, workloads

pytestmark = pytest.mark.gpu

KEYS = ("tau", "grf", "x", "status", "iters")


def sample_rows(B, n=512):
    rows = set(np.linspace(0, B - 1, n).astype(int).tolist())
    for k in range(0, B, 2048):  # pass boundaries
        rows.update(r for r in (k - 1, k, k + 1) if 0 <= r < B)
    rows.add(B - 1)
    return np.array(sorted(rows))


def run(inp, modes=None):
    S = inp["base_pose"].shape[0]
    K = len(modes) if modes is not None else 1
    e = Engine(S * K)
    if modes is not None:
        e.set_modes(modes)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    (e.step_modes if modes is not None else e.step)(STATELESS)
    out = e.outputs()
    e.close()
    return out


def check_vs_oracle(out, rows, inp_rows):
    o = R.run_batch(inp_rows)
    red = R.run_batch(inp_rows, method=R.REDUCED)
    assert np.array_equal(out["status"][rows], o["status"])
    same_it = out["iters"][rows] == red["iters"]
    # identical counts: near-ties are decided by one rule on both sides (WBC_TIE_BAND)
    assert M.record("iters mismatch fraction", 1.0 - same_it.mean(), 0.0) == 0.0, int((~same_it).sum())
    ok = o["status"] == 0
    for j in np.nonzero(ok)[0]:
        b = rows[j]
        assert M.close(out["x"][b], o["x"][j], M.X, "x"), (b, "x")
        assert M.close(out["tau"][b], o["tau"][j], M.TAU, "tau"), (b, "tau")


@pytest.mark.parametrize("name,B,seed", [("stance_cold", 4096, 1), ("rl_random", 8192, 3), ("rl_random", 65536, 3)])
def test_full_batch_sample_matches_oracle_and_small_batch(name, B, seed):
    inp = getattr(workloads, name)(B, seed=seed)
    out = run(inp)
    rows = sample_rows(B)
    assert len(rows) >= 512 and rows[-1] == B - 1 and (rows >= 2048).sum() > 256
    sub = {k: np.ascontiguousarray(v[rows]) for k, v in inp.items()}
    check_vs_oracle(out, rows, sub)
    small = run(sub)
    for k in KEYS:
        assert np.array_equal(small[k], out[k][rows]), k


@pytest.mark.parametrize("S", [1024, 8192])
def test_modes_full_shard_sample_matches_oracle_and_small_batch(S):
    """S = 1024: the configs[4] shard of one GPU of eight; S = 8192: configs[4]'s global batch
    (131 072 QPs) on one GPU."""
    K = 16
    inp, modes = workloads.mode_states(S, 4)
    out = run(inp, modes)
    # 40 spread states plus the pass boundaries (QP 2048 k = state 128 k) and the last state
    step = 128 if S <= 1024 else 1024
    states = np.unique(np.concatenate([np.linspace(0, S - 1, 40).astype(int), np.arange(step - 1, S, step),
                                       np.arange(step, S, step), [S - 1]]))
    rows = (states[:, None] * K + np.arange(K)[None, :]).ravel()
    assert len(rows) >= 512 and rows[-1] == S * K - 1
    # the oracle sees each hypothesis as its own robot (contacts = modes[k])
    rep = {k: np.repeat(np.ascontiguousarray(v[states]), K, axis=0) for k, v in inp.items()}
    rep["contacts"] = np.tile(modes, len(states))
    check_vs_oracle(out, rows, rep)
    small = run({k: np.ascontiguousarray(v[states]) for k, v in inp.items()}, modes)
    for k in KEYS:
        assert np.array_equal(small[k], out[k][rows]), k


def trot_rows(B, n=256):
    """n robots spread over the batch, both sides of every 1024-robot boundary, every robot of the
    first and last waves, and the last robot."""
    rows = set(np.linspace(0, B - 1, n).astype(int).tolist())
    for k in range(0, B + 1, 1024):
        rows.update(r for r in (k - 2, k - 1, k, k + 1) if 0 <= r < B)
    rows.update(range(4))
    rows.update(range(B - 4, B))
    return np.array(sorted(rows))


def test_trot_bench_path_every_step_matches_stateful_oracle():
    """BASELINE configs[2] exactly as bench.py times it (bench_trot): B = 4096 robots, 400 stateful
    steps, all inputs staged in HBM and bound per step (wbc_bind_device_inputs), WBC_NO_X, the
    history and hotstart carried on the GPU.  At every step >= 256 sampled robots are compared
    with the C oracle's stateful robots (oracle/wbc_ref.c, the REDUCED method: the 12-variable form
    with the same hotstart): identical status and iteration counts, tau / grf at the parity
    tolerances.  The sequence then runs again after wbc_reset(), as bench.py's timed pass does after
    its warm-up pass, and must reproduce the first pass bit for bit."""
    import torch

    from quadrupedwholebodycontroller_amd import NO_X

    B, T = 4096, 400
    seq = list(workloads.trot_sequence(B, steps=T, seed=2))  # bench_trot's inputs
    dev = {k: torch.from_numpy(np.ascontiguousarray(np.stack([s[k] for s in seq]))).cuda() for k in seq[0]}
    rows = trot_rows(B)
    assert len(rows) >= 256 and rows[-1] == B - 1
    e = Engine(B)
    first = []
    for p in range(2):
        e.reset()
        oracle = R.Robots(rows, method=R.REDUCED) if p == 0 else None
        n_ok = n_it = 0
        for t in range(T):
            e.bind_device_inputs(dev["base_pose"][t].data_ptr(), dev["nu"][t].data_ptr(), dev["qj"][t].data_ptr(),
                                 dev["ref"][t].data_ptr(), dev["contacts"][t].data_ptr(), dev["switching"][t].data_ptr())
            e.step(NO_X)
            g = e.outputs()
            if p == 1:
                for k in ("tau", "grf", "status", "iters"):
                    assert np.array_equal(g[k], first[t][k]), (t, k)
                continue
            first.append({k: g[k].copy() for k in ("tau", "grf", "status", "iters")})
            o = oracle.step(seq[t])
            assert np.array_equal(g["status"][rows], o["status"]), (t, rows[g["status"][rows] != o["status"]][:8])
            same = g["iters"][rows] == o["iters"]
            assert M.record("iters mismatch fraction", 1.0 - same.mean(), 0.0) == 0.0, (t, rows[~same][:8])
            ok = o["status"] == 0
            assert M.close(g["tau"][rows][ok], o["tau"][ok], M.TAU, "tau"), t
            assert M.close(g["grf"][rows][ok], o["grf"][ok], M.GRF, "grf"), t
            n_ok += int(ok.sum())
            n_it += int(o["iters"].sum())
        if p == 0:
            assert n_ok > 0.9 * len(rows) * T
    e.close()


@pytest.mark.parametrize("name,B,seed", [("rl_random", 8192, 3), ("stance_cold", 4096, 1)])
def test_split_form_full_batch_matches_literal_oracle(name, B, seed):
    """The reference's updateState() / solveQP() surface at the bench's sizes: WBC_SPLIT (the update
    kernel, the problem through HBM, then the 24-variable solve kernel, one robot per wave, several
    occupancy passes) against the oracle's LITERAL method on the 42 x 70 QP: identical status and
    iteration counts on a stratified sample of >= 512 rows, tau at the parity tolerance."""
    from quadrupedwholebodycontroller_amd import SPLIT

    inp = getattr(workloads, name)(B, seed=seed)
    e = Engine(B)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    e.step(STATELESS | SPLIT)
    out = e.outputs()
    e.close()
    rows = sample_rows(B)
    sub = {k: np.ascontiguousarray(v[rows]) for k, v in inp.items()}
    o = R.run_batch(sub, method=R.LITERAL)
    assert np.array_equal(out["status"][rows], o["status"])
    same = out["iters"][rows] == o["iters"]
    assert M.record("iters mismatch fraction (split)", 1.0 - same.mean(), 0.0) == 0.0, rows[~same][:8]
    ok = o["status"] == 0
    assert M.close(out["tau"][rows][ok], o["tau"][ok], M.TAU, "tau")
    assert M.close(out["x"][rows][ok], o["x"][ok], M.X, "x")
