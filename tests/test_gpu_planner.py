"""GPU: the batched motion planner (include/wbc_planner.h) against the literal CPU restatement of
the reference's plannerLoop (oracle/planner_ref.py), tick by tick, and the planner feeding the WBC
engine directly on the device.

Per tick and robot: `published` identical, contacts and switching identical, the 54-double
message within 1e-12 (absolute + relative; the same fp64 expressions, up to FMA contraction).
"""
import numpy as np
import pytest

import margins as M
import planner_ref as PR
import wbc_ref
from quadrupedwholebodycontroller_amd import Engine, Planner, workloads

pytestmark = pytest.mark.gpu


def command_schedule(B, T, seed=0):
    """Per robot: zero, forward, lateral, turning, mixed; some change mid-cycle."""
    g = np.random.default_rng(seed)
    base = np.zeros((B, 3))
    kinds = np.arange(B) % 5
    base[kinds == 1, 0] = 0.4
    base[kinds == 2, 1] = -0.25
    base[kinds == 3, 2] = 0.5
    base[kinds == 4] = g.uniform(-0.5, 0.5, (int((kinds == 4).sum()), 3))
    sched = np.repeat(base[None], T, axis=0)
    # robots with index % 7 == 0 change command at tick 50 (mid-cycle) and stop at tick 200
    chg = np.arange(B) % 7 == 0
    sched[50:, chg] = g.uniform(-0.4, 0.4, (int(chg.sum()), 3))
    sched[200:, chg] = 0.0
    return sched


def oracle_ticks(sched, b):
    t = [0]
    gen = PR.planner(lambda: tuple(sched[t[0], b]))
    out, last = [], (1, 1, 1, 1)
    for k in range(sched.shape[0]):
        t[0] = k
        o = next(gen)
        if o is None:
            out.append(None)
        else:
            msg, con = o
            out.append((msg, sum(c << i for i, c in enumerate(con)), int(con != last)))
            last = con
    return out


def test_planner_matches_reference_loop():
    B, T = 40, 300
    sched = command_schedule(B, T)
    pl = Planner(B)
    got = []
    for k in range(T):
        pl.set_command(sched[k])
        pl.tick()
        got.append(pl.outputs())
    pl.close()
    for b in range(B):
        ref = oracle_ticks(sched, b)
        for k in range(T):
            o = got[k]
            if ref[k] is None:
                assert o["published"][b] == 0, (b, k)
                continue
            msg, con, sw = ref[k]
            assert o["published"][b] == 1, (b, k)
            assert o["contacts"][b] == con, (b, k)
            assert o["switching"][b] == sw, (b, k)
            err = np.abs(o["ref"][b] - msg)
            assert np.all(err <= 1e-12 * (1 + np.abs(msg))), (b, k, float(err.max()))


def test_planner_drives_engine_on_device():
    """Planner tick every 4 control cycles (100 Hz vs 400 Hz); the engine reads the planner's
    device buffers (no host copies) and matches the same run fed from host copies bit for bit, and
    the C oracle's stateful robots fed the same messages (status and iteration counts equal, tau at
    the parity tolerance) through the planner's contact switches and the hotstart across them."""
    import torch

    B, cycles = 64, 4 * 85  # one full 4-step planner cycle
    pl = Planner(B)
    cmd = np.zeros((B, 3))
    cmd[:, 0] = 0.3
    pl.set_command(cmd)
    dev = pl.device_outputs()
    st = workloads.stance_cold(B, seed=5)
    e_dev, e_host = Engine(B), Engine(B)
    for e in (e_dev, e_host):
        e.set_state(st["base_pose"], st["nu"], st["qj"])
    e_dev.bind_device_inputs(ref=dev["ref"], contacts=dev["contacts"], switching=dev["switching"])
    robots = wbc_ref.Robots(np.arange(B), method=wbc_ref.REDUCED)
    seen = set()
    for c in range(cycles):
        if c % 4 == 0:
            pl.tick()
        o = pl.outputs()
        e_host.set_reference(o["ref"], o["contacts"], o["switching"])
        e_dev.step(0)
        e_host.step(0)
        a, h = e_dev.outputs(), e_host.outputs()
        for k in ("tau", "grf", "status"):
            assert np.array_equal(a[k], h[k]), (c, k)
        r = robots.step(dict(st, ref=o["ref"], contacts=o["contacts"], switching=o["switching"]))
        assert np.array_equal(a["status"], r["status"]) and np.array_equal(a["iters"], r["iters"]), c
        ok = r["status"] == 0
        assert M.close(a["tau"][ok], r["tau"][ok], M.TAU, "tau"), c
        seen.update(int(x) for x in o["contacts"])
    assert {7, 11, 13, 14} <= seen  # every single-swing mode was exercised
    for e in (e_dev, e_host):
        e.close()
    pl.close()
    torch.cuda.synchronize()
