"""Probe: the headline step replayed from a captured HIP graph (torch.cuda.CUDAGraph around the
engine's launches) against plain stream launches.  Usage (GPU box): python tools/graph_probe.py [B] [steps]"""
import json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from quadrupedwholebodycontroller_amd import NO_X, STATELESS, Engine, workloads

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 50
inp = workloads.stance_cold(B, seed=1)
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
e = Engine(B)
e.set_stream(st.cuda_stream)
e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
F = STATELESS | NO_X
for _ in range(5):
    e.step(F)
torch.cuda.synchronize()


def timed(fn, reps):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(st)
    for _ in range(reps):
        fn()
    b.record(st)
    torch.cuda.synchronize()
    return a.elapsed_time(b)


res = {}
for rep in range(2):
    ms = timed(lambda: e.step(F), steps) / steps
    res[f"stream#{rep}"] = dict(ms=ms, solves_per_s=B / ms * 1e3)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=st):
        for _ in range(steps):
            e.step(F)
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    ms = timed(g.replay, 1) / steps
    res[f"graph#{rep}"] = dict(ms=ms, solves_per_s=B / ms * 1e3)
o = e.outputs()
res["tau_sum"] = float(abs(o["tau"]).sum())
print(json.dumps(res))
e.close()
