"""GPU: the engine on a caller-owned stream (wbc_set_stream, include/wbc.h).

A bound caller stream is synchronized when it is unbound or the engine is destroyed (no per-launch
event tracks it: that packet cost ~3 us per step).  Steps queued on a torch stream must give the
own-stream results bit for bit, switching back and forth between steps must not race (the switch
drains the old stream), and destroying the engine with a caller stream bound must drain it.
"""
import numpy as np
import pytest

from quadrupedwholebodycontroller_amd import NO_X, STATELESS, Engine, workloads

pytestmark = pytest.mark.gpu

KEYS = ("tau", "grf", "status", "iters")


def _load(e, inp):
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])


def test_caller_stream_matches_own_stream_and_switches_safely():
    torch = pytest.importorskip("torch")
    B = 512
    a, b = workloads.stance_cold(B, seed=31), workloads.rl_random(B, seed=32)
    ref = []
    e = Engine(B)
    for inp in (a, b):
        _load(e, inp)
        e.step(STATELESS | NO_X)
        ref.append(e.outputs())
    e.close()

    s = torch.cuda.Stream()
    e = Engine(B)
    for k, inp in enumerate((a, b, a, b)):
        e.set_stream(s.cuda_stream if k % 2 == 0 else 0)  # caller stream, own stream, caller ...
        _load(e, inp)
        for _ in range(3):  # several steps queued before the outputs are read
            e.step(STATELESS | NO_X)
        out = e.outputs()
        for key in KEYS:
            assert np.array_equal(out[key], ref[k % 2][key]), (k, key)
    e.set_stream(s)  # the stream object: the engine keeps it referenced while bound
    assert e._stream is s
    _load(e, a)
    for _ in range(5):
        e.step(STATELESS | NO_X)
    e.close()  # drains the bound caller stream before freeing, then releases it
    assert e._stream is None
    s.synchronize()
