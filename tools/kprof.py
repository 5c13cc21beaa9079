"""Run one bench workload for a few steps (for rocprofv3 --kernel-trace --stats per-kernel times).
Usage (GPU box): [WBC_LIB=...] python tools/kprof.py <config> [steps]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
import bench
from quadrupedwholebodycontroller_amd import NO_X, STATELESS

name = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cfg = bench.CONFIGS[name]
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
e, step, _ = bench.make_engine(cfg, cfg["batch"], cfg["seed"], 0, st)
for _ in range(steps):
    step(STATELESS | NO_X)
torch.cuda.synchronize()
o = e.outputs()
print(name, "status", [int((o["status"] == k).sum()) for k in range(4)], "mean iters", float(o["iters"].mean()))
e.close()
