"""Deployment probe (not the bench line): configs[1]'s batch (4096 cold stance QPs) stepped by 1, 2
or 3 engines on their own streams in turn, so that up to that many independent steps are in flight
on the GPU at once.  A step's kernel lasts as long as its hardest QP's wave; with
another step queued on a second stream, SIMDs freed by the first step's early waves start the next
step's waves instead of idling.  Prints solves/s per engine count.
Usage (GPU box): python tools/inflight_probe.py [steps]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from quadrupedwholebodycontroller_amd import NO_X, STATELESS, Engine, workloads  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
B = 4096
inp = workloads.stance_cold(B, seed=1)
res = {}
for n in (1, 2, 3):
    engines, streams = [], []
    for _ in range(n):
        st = torch.cuda.Stream()
        e = Engine(B)
        e.set_stream(st)
        e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
        e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
        engines.append(e)
        streams.append(st)
    for k in range(10 * n):
        engines[k % n].step(STATELESS | NO_X)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        engines[k % n].step(STATELESS | NO_X)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    outs = [e.outputs()["tau"] for e in engines]
    same = all((o == outs[0]).all() for o in outs)
    res[n] = {"solves_per_s": B * steps / dt, "us_per_step": dt / steps * 1e6, "identical_outputs": bool(same)}
    for e in engines:
        e.close()
    print(n, json.dumps(res[n]), flush=True)
print(json.dumps({"batch": B, "steps": steps, "engines_in_flight": res}))
