"""GPU: contact-mode hypotheses (wbc_set_modes / wbc_step_modes, BASELINE configs[4]).

Every state is solved under K contact masks with the dynamics and assembly computed once per
state.  The contract is bit-identity with the per-row path: a
wbc_step over the state replicated K times with contacts = modes[k] must give the same tau, grf,
x, status and iteration counts, bit for bit.  The oracle check reuses test_gpu_parity's
tolerances on a subset.

The default form runs either one hypothesis per 16-lane segment or, with many states, the mode loop
(wbc_modes_kernel: one update per state and wave, then M hypotheses in turn, the engine's choice of
M; WBC_MODES_M forces it): both are checked against the per-row step, fallbacks included.
"""
import os

import numpy as np

import margins as M
import pytest

import wbc_np as W
from quadrupedwholebodycontroller_amd import NO_X, SPLIT, STATELESS, Engine, WbcError, workloads

pytestmark = pytest.mark.gpu

KEYS = ("tau", "grf", "x", "status", "iters")


def replicated(base, modes):
    K = len(modes)
    rep = {k: np.repeat(v, K, axis=0) for k, v in base.items()}
    rep["contacts"] = np.tile(np.asarray(modes, np.uint8), base["base_pose"].shape[0])
    return rep


def per_row(inp, flags=STATELESS):
    B = inp["base_pose"].shape[0]
    e = Engine(B)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    e.step(flags)
    out = e.outputs()
    e.close()
    return out


def hypotheses(base, modes, flags=STATELESS, m=None):
    """wbc_step_modes; m: hypotheses per wave of the mode loop (WBC_MODES_M, read by wbc_set_modes)."""
    S, K = base["base_pose"].shape[0], len(modes)
    e = Engine(S * K)
    old = os.environ.get("WBC_MODES_M")
    if m is not None:
        os.environ["WBC_MODES_M"] = str(m)
    try:
        e.set_modes(modes)
    finally:
        if m is not None:
            if old is None:
                del os.environ["WBC_MODES_M"]
            else:
                os.environ["WBC_MODES_M"] = old
    e.set_state(base["base_pose"], base["nu"], base["qj"])
    e.set_reference(base["ref"], base["contacts"], base["switching"])
    e.step_modes(flags)
    out = e.outputs()
    e.close()
    return out


@pytest.mark.parametrize("m", [None, 2, 4, 16])
@pytest.mark.parametrize("switching", [1, 0])
def test_all_16_modes_bit_identical_to_per_row(switching, m):
    base = workloads.rl_random(96, seed=21)
    base["switching"][:] = switching  # 0: stateless but non-switching, the R1 / swing bounds carry J-dot terms
    modes = list(range(16))
    got = hypotheses(base, modes, m=m)
    want = per_row(replicated(base, modes))
    for k in KEYS:
        assert np.array_equal(got[k], want[k]), k
    assert len(set(want["status"].tolist())) >= 1 and (want["status"] == 0).mean() > 0.5


@pytest.mark.parametrize("split,m", [(False, None), (False, 4), (False, 16), (True, None)])
def test_modes_with_stretched_legs_bit_identical_to_per_row(split, m):
    """A stretched (singular) leg makes the reduction unusable for the hypotheses where that leg is
    in stance: those QPs take the update wave's general fallback from their own
    problem record, in both paths alike (in the mode loop, several per wave, drained after the
    loop); under WBC_SPLIT the split kernels' own forms."""
    base = workloads.straight_legs(workloads.stance_cold(24, seed=25), every=2)
    modes = list(range(16))
    flags = STATELESS | (SPLIT if split else 0)
    got = hypotheses(base, modes, flags, m=m)
    want = per_row(replicated(base, modes), flags)
    for k in KEYS:
        assert np.array_equal(got[k], want[k]), k
    assert (want["status"] == 0).mean() > 0.5


@pytest.mark.parametrize("m", [None, 5])
def test_subset_of_modes_and_repeats(m):
    base = workloads.stance_cold(40, seed=22)
    modes = [15, 10, 5, 15, 0]  # stance, both trot pairs, a repeat, all-swing
    got = hypotheses(base, modes, m=m)
    want = per_row(replicated(base, modes))
    for k in KEYS:
        assert np.array_equal(got[k], want[k]), k


def test_modes_against_oracle():
    base = workloads.rl_random(8, seed=23)
    modes = list(range(16))
    got = hypotheses(base, modes)
    model, params = W.Model(), W.default_params()
    for s in range(8):
        for k in modes:
            r = s * 16 + k
            c = W.ReferenceWBC(model, params)
            c.set_state(base["base_pose"][s], base["nu"][s], base["qj"][s])
            c.set_reference(base["ref"][s], [(k >> i) & 1 for i in range(4)], bool(base["switching"][s]))
            c.step()
            assert got["status"][r] == c.qp_status, (s, k)
            if c.qp_status == W.QP_OK:
                assert M.close(got["x"][r], c.qp_solution, M.X, "x"), (s, k)
                assert M.close(got["tau"][r], c.tau, M.TAU, "tau"), (s, k)


def test_no_x_and_device_outputs():
    base = workloads.rl_random(32, seed=24)
    modes = list(range(16))
    e = Engine(32 * 16)
    e.set_modes(modes)
    e.set_state(base["base_pose"], base["nu"], base["qj"])
    e.set_reference(base["ref"], base["contacts"], base["switching"])
    e.step_modes(STATELESS | NO_X)
    out = e.outputs()
    e.close()
    want = per_row(replicated(base, modes))
    for k in ("tau", "grf", "status", "iters"):
        assert np.array_equal(out[k], want[k]), k


def test_mode_errors():
    e = Engine(48)
    with pytest.raises(WbcError):
        e.set_modes([1] * 5)  # 5 does not divide 48
    with pytest.raises(WbcError):
        e.set_modes([16])  # masks are 4-bit
    with pytest.raises(WbcError):
        e.step_modes(STATELESS)  # no modes set
    e.set_modes([15, 3, 12])
    with pytest.raises(WbcError):
        e.step_modes(0)  # hypotheses are cold steps
    with pytest.raises(WbcError):
        e.step(STATELESS)  # the per-row step is refused while modes are set
    base = workloads.stance_cold(16, seed=25)
    e.set_state(base["base_pose"], base["nu"], base["qj"])
    e.set_reference(base["ref"], base["contacts"], base["switching"])
    e.step_modes(STATELESS)
    e.set_modes(None)  # back to one robot per row
    full = workloads.stance_cold(48, seed=26)
    e.set_state(full["base_pose"], full["nu"], full["qj"])
    e.set_reference(full["ref"], full["contacts"], full["switching"])
    e.step(STATELESS)
    out = e.outputs()
    e.close()
    assert (out["status"] == 0).all()


def test_mode_loop_at_the_bench_size():
    """configs[4]'s shard, 1024 states x 16 masks (bench.py modes16_b16384): the engine picks the mode
    loop (four hypotheses per wave on a 256-CU MI355X); every output bit-identical to the per-row
    step over the 16384 replicated rows."""
    base, modes = workloads.mode_states(1024, 4)
    got = hypotheses(base, modes, NO_X | STATELESS)
    want = per_row(replicated(base, modes), NO_X | STATELESS)
    for k in ("tau", "grf", "status", "iters"):
        assert np.array_equal(got[k], want[k]), k
    assert (want["status"] == 0).mean() > 0.9
