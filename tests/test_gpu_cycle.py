"""GPU: wbc_cycle, the one-call host-to-host control cycle (pinned staging, one H2D copy, the
step, one D2H copy).  It must give exactly what wbc_set_state + wbc_set_reference + wbc_step +
wbc_get_output give, cold and stateful, for odd batch sizes (output block alignment), with and
without x, and leave caller-bound output buffers bound."""
import numpy as np
import pytest

from quadrupedwholebodycontroller_amd import RESIDENT, STATELESS, Engine, WbcError, workloads

pytestmark = pytest.mark.gpu

KEYS = ("tau", "grf", "x", "status", "iters")


def separate_calls(e, inp, flags):
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    e.step(flags)
    return e.outputs()


@pytest.mark.parametrize("B", [1, 33, 256])
def test_cycle_equals_separate_calls_cold(B):
    inp = workloads.rl_random(B, seed=40 + B)
    e1, e2 = Engine(B), Engine(B)
    want = separate_calls(e1, inp, STATELESS)
    got = e2.cycle(inp["base_pose"], inp["nu"], inp["qj"], inp["ref"], inp["contacts"], inp["switching"], STATELESS)
    no_x = e2.cycle(inp["base_pose"], inp["nu"], inp["qj"], inp["ref"], inp["contacts"], inp["switching"], STATELESS,
                    want_x=False)
    e1.close(); e2.close()
    for k in KEYS:
        assert np.array_equal(got[k], want[k]), k
    for k in ("tau", "grf", "status", "iters"):
        assert np.array_equal(no_x[k], want[k]), k


def test_cycle_equals_separate_calls_stateful_trot():
    B, T = 48, 60
    seq = list(workloads.trot_sequence(B, steps=T, seed=5))
    e1, e2 = Engine(B), Engine(B)
    for t, s in enumerate(seq):
        want = separate_calls(e1, s, 0)
        got = e2.cycle(s["base_pose"], s["nu"], s["qj"], s["ref"], s["contacts"], s["switching"], 0)
        for k in KEYS:
            assert np.array_equal(got[k], want[k]), (t, k)
    e1.close(); e2.close()


def test_cycle_keeps_bound_outputs_and_refuses_modes():
    import torch

    B = 16
    inp = workloads.stance_cold(B, seed=41)
    e = Engine(B)
    tau_dev = torch.zeros(B * 12, dtype=torch.float64, device="cuda")
    e.bind_device_outputs(tau=tau_dev.data_ptr())
    got = e.cycle(inp["base_pose"], inp["nu"], inp["qj"], inp["ref"], inp["contacts"], inp["switching"], STATELESS)
    # the cycle returns its own copy; the bound tensor stays bound for the next plain step
    e.step(STATELESS)
    torch.cuda.synchronize()
    assert np.array_equal(tau_dev.cpu().numpy().reshape(B, 12), got["tau"])
    e.set_modes([15, 5])
    with pytest.raises(WbcError):
        e.cycle(inp["base_pose"], inp["nu"], inp["qj"], inp["ref"], inp["contacts"], inp["switching"], STATELESS)
    e.close()


def test_cycle_keeps_bound_inputs():
    """A caller that bound device inputs keeps them across wbc_cycle: the cycle reads its own host
    arrays for that one step, the next plain step reads the bound tensors again."""
    import torch

    B = 24
    a, b = workloads.rl_random(B, seed=61), workloads.rl_random(B, seed=62)
    want_a = separate_calls(Engine(B), a, STATELESS)
    want_b = separate_calls(Engine(B), b, STATELESS)
    d = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in a.items()}
    e = Engine(B)
    e.bind_device_inputs(d["base_pose"].data_ptr(), d["nu"].data_ptr(), d["qj"].data_ptr(), d["ref"].data_ptr(),
                         d["contacts"].data_ptr(), d["switching"].data_ptr())
    got_b = e.cycle(b["base_pose"], b["nu"], b["qj"], b["ref"], b["contacts"], b["switching"], STATELESS)
    e.step(STATELESS)
    got_a = e.outputs()
    e.close()
    for k in KEYS:
        assert np.array_equal(got_b[k], want_b[k]), k
        assert np.array_equal(got_a[k], want_a[k]), k


def test_cycle_zero_copy_across_flag_and_mask_changes():
    """At B <= 64 wbc_cycle runs zero-copy: the step reads the pinned input block and the pinned wave
    map and writes the pinned output block.  Stateful trot with mixed masks every
    sixth cycle (the wave map path) and x switched on and off: every cycle must equal the separate
    calls, history included."""
    B = 8
    seq = list(workloads.trot_sequence(B, steps=24, seed=9))
    e1, e2 = Engine(B), Engine(B)
    g = np.random.default_rng(2)
    for t, s in enumerate(seq):
        s = dict(s)
        if t % 6 == 5:  # mixed masks: the wave map (built at copy time, read through its device address)
            s["contacts"] = g.integers(0, 16, B).astype(np.uint8)
        flags = 0  # stateful throughout; x on / off alternates below
        want = separate_calls(e1, s, flags)
        got = e2.cycle(s["base_pose"], s["nu"], s["qj"], s["ref"], s["contacts"], s["switching"], flags,
                       want_x=(t % 3 != 0))
        for k in ("tau", "grf", "status", "iters"):
            assert np.array_equal(got[k], want[k]), (t, k)
        if t % 3 != 0:
            assert np.array_equal(got["x"], want["x"]), t
    e1.close(); e2.close()


@pytest.mark.parametrize("B", [8, 24])
def test_zero_copy_cycle_then_plain_step_mixed_masks(B):
    """After a zero-copy cycle with mixed masks the engine's own device inputs, outputs and wave map
    are brought up to date lazily (sync_own) before any other call.  outputs() right after the cycle,
    then a plain wbc_step on the cycle's inputs and outputs() again, must give exactly what the
    separate calls give (stateless and stateful)."""
    a = workloads.rl_random(B, seed=70 + B)
    for flags in (STATELESS, 0):
        ref = Engine(B)
        want = separate_calls(ref, a, flags)
        want2 = (ref.step(flags), ref.outputs())[1]  # the second cycle of the same inputs (history)
        ref.close()
        e = Engine(B)
        got = e.cycle(a["base_pose"], a["nu"], a["qj"], a["ref"], a["contacts"], a["switching"], flags)
        after = e.outputs()  # the cycle's outputs, now read from the engine's own buffers
        e.step(flags)  # the cycle's inputs, masks and map from the engine's own buffers
        got2 = e.outputs()
        e.close()
        for k in KEYS:
            assert np.array_equal(got[k], want[k]), (flags, k)
            assert np.array_equal(after[k], want[k]), (flags, k)
            assert np.array_equal(got2[k], want2[k]), (flags, k)


@pytest.mark.parametrize("B", [1, 4])
def test_resident_cycle_equals_separate_calls(B):
    """WBC_RESIDENT (B <= 4): the step stays on the GPU between cycles, polling a pinned mailbox
    (DESIGN.md 4.18).  A stateful trot, every cycle equal to the separate calls, with the resident
    wave stopped and restarted on the way: by a plain wbc_step / wbc_get_output (any other call
    stops it), by a change of flags (x on / off), and by a pause longer than the host's restart
    limit (the wave may have ended by its idle limit)."""
    import time

    seq = list(workloads.trot_sequence(B, steps=40, seed=11))
    e1, e2 = Engine(B), Engine(B)
    for t, s in enumerate(seq):
        want = separate_calls(e1, s, 0)
        got = e2.cycle(s["base_pose"], s["nu"], s["qj"], s["ref"], s["contacts"], s["switching"], RESIDENT,
                       want_x=(t % 10 < 7))
        for k in ("tau", "grf", "status", "iters"):
            assert np.array_equal(got[k], want[k]), (t, k)
        if t % 10 < 7:
            assert np.array_equal(got["x"], want["x"]), t
        if t == 15:  # any other call stops the resident wave and sees the cycle's state
            o = e2.outputs()
            for k in ("tau", "grf", "status", "iters"):
                assert np.array_equal(o[k], want[k]), (t, k)
        if t == 25:
            time.sleep(0.15)  # longer than the wave's idle limit: it has ended; the next cycle restarts it
    e1.close()
    e2.close()


def test_resident_cycle_then_plain_steps():
    """After resident cycles, plain steps on the engine's own buffers continue the same history."""
    B = 1
    seq = list(workloads.trot_sequence(B, steps=20, seed=12))
    e1, e2 = Engine(B), Engine(B)
    for t, s in enumerate(seq):
        want = separate_calls(e1, s, 0)
        if t < 10:
            got = e2.cycle(s["base_pose"], s["nu"], s["qj"], s["ref"], s["contacts"], s["switching"], RESIDENT)
        else:
            got = separate_calls(e2, s, 0)
        for k in KEYS:
            assert np.array_equal(got[k], want[k]), (t, k)
    e1.close()
    e2.close()


@pytest.mark.parametrize("B", [2, 4, 5])
def test_resident_cycle_stateless_and_above_limit(B):
    """WBC_RESIDENT | WBC_STATELESS: cold solves through the resident wave (mixed masks, then all
    stance, then mixed again: the masks change between cycles) equal separate calls bit for bit.
    B = 5 is above the resident limit (B <= 4): the flag falls back to the launch path, same bits."""
    e1, e2 = Engine(B), Engine(B)
    for t in range(6):
        inp = workloads.rl_random(B, seed=70 + t)
        if t in (2, 3):
            inp["contacts"] = np.full(B, 15, np.uint8)
        want = separate_calls(e1, inp, STATELESS)
        got = e2.cycle(inp["base_pose"], inp["nu"], inp["qj"], inp["ref"], inp["contacts"], inp["switching"],
                       RESIDENT | STATELESS)
        for k in KEYS:
            assert np.array_equal(got[k], want[k]), (t, k)
    e1.close()
    e2.close()


def test_two_resident_engines_in_turn():
    """Two B = 1 engines cycled in turn with WBC_RESIDENT: at most one resident wave
    runs per process, and any other engine's call stops it first, so neither engine's work can
    queue behind the other's polling wave on a shared hardware queue (it would wait up to the
    wave's 100 ms idle limit).  Both trajectories equal separate plain steps bit for bit, no cycle
    takes more than 20 ms and the median stays under 2 ms; a large engine's step issued while a
    resident wave runs is not held up either."""
    import time

    seqs = [list(workloads.trot_sequence(1, steps=60, seed=s)) for s in (13, 14)]
    plain = [Engine(1), Engine(1)]
    res = [Engine(1), Engine(1)]
    big = Engine(4096)
    binp = workloads.stance_cold(4096, seed=3)
    big.set_state(binp["base_pose"], binp["nu"], binp["qj"])
    big.set_reference(binp["ref"], binp["contacts"], binp["switching"])
    big.step(STATELESS)
    want_big = big.outputs()
    dts, big_dts = [], []
    for t in range(60):
        for i in (0, 1):
            s = seqs[i][t]
            want = separate_calls(plain[i], s, 0)
            t0 = time.perf_counter()
            got = res[i].cycle(s["base_pose"], s["nu"], s["qj"], s["ref"], s["contacts"], s["switching"], RESIDENT)
            dts.append(time.perf_counter() - t0)
            for k in KEYS:
                assert np.array_equal(got[k], want[k]), (t, i, k)
        if t % 10 == 5:  # a large engine's step while engine 1's resident wave runs
            t0 = time.perf_counter()
            big.step(STATELESS)
            o = big.outputs()
            big_dts.append(time.perf_counter() - t0)
            assert np.array_equal(o["tau"], want_big["tau"])
    for e in plain + res + [big]:
        e.close()
    dts = np.array(dts[2:])  # (the first cycles start the waves)
    assert dts.max() < 0.02 and np.median(dts) < 0.002, (dts.max(), np.median(dts))
    assert max(big_dts) < 0.02, big_dts
