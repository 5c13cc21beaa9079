"""Time the occupancy variants (libwbc_hip_w{N}.so) side by side; each in its own process.
Usage (GPU box): python tools/variants.py [steps]"""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys, time
sys.path.insert(0, %r)
import torch
from quadrupedwholebodycontroller_amd import NO_X, STATELESS, Engine, workloads
steps = int(sys.argv[1])
res = {}
for name, gen, B in (("stance_cold_b4096", workloads.stance_cold, 4096), ("rl_random_b8192", workloads.rl_random, 8192),
                     ("stance_cold_b16384", workloads.stance_cold, 16384)):
    inp = gen(B, seed=1)
    e = Engine(B)
    st = torch.cuda.Stream(); torch.cuda.set_stream(st); e.set_stream(st.cuda_stream)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"]); e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    F = STATELESS | NO_X
    for _ in range(3): e.step(F)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(st)
    for _ in range(steps): e.step(F)
    ev1.record(st); torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    o = e.outputs()
    res[name] = dict(ms=ms, solves_per_s=B / ms * 1e3, status=[int(x) for x in __import__("numpy").bincount(o["status"], minlength=4)],
                     tau_sum=float(abs(o["tau"]).sum()))
    e.close()
S = 1024  # configs[4] shard: 1024 states x 16 contact masks through wbc_step_modes
inp, modes = workloads.mode_states(S, 4)
e = Engine(S * 16)
st = torch.cuda.Stream(); torch.cuda.set_stream(st); e.set_stream(st.cuda_stream)
e.set_modes(modes)
e.set_state(inp["base_pose"], inp["nu"], inp["qj"]); e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
for _ in range(3): e.step_modes(STATELESS | NO_X)
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record(st)
for _ in range(steps): e.step_modes(STATELESS | NO_X)
ev1.record(st); torch.cuda.synchronize()
ms = ev0.elapsed_time(ev1) / steps
o = e.outputs()
res["modes16_b16384"] = dict(ms=ms, solves_per_s=S * 16 / ms * 1e3, status=[int(x) for x in __import__("numpy").bincount(o["status"], minlength=4)],
                             tau_sum=float(abs(o["tau"]).sum()))
e.close()
import bench  # configs[2]: stateful trot (history + hotstart), 100 cycles
r = bench.bench_trot(torch, st, 0, STATELESS, T=100)
res["trot_b4096"] = dict(ms=r["ms_per_step"], solves_per_s=r["solves_per_s"], status=r["status_counts_last"],
                         mean_iters=r["mean_iters_last"])
print(json.dumps(res))
''' % ROOT
steps = sys.argv[1] if len(sys.argv) > 1 else "30"
names = sys.argv[2].split(",") if len(sys.argv) > 2 else ["w2", "w3", "w4", "w5"]
out = {}
for rep in range(2):  # two passes, interleaved, to expose box-to-box / run-to-run drift
    for n in names:
        lib = os.path.join(ROOT, "quadrupedwholebodycontroller_amd", f"libwbc_hip_{n}.so")
        r = subprocess.run([sys.executable, "-c", CHILD, steps], env=dict(os.environ, WBC_LIB=lib), capture_output=True,
                           text=True, timeout=300)
        res = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else dict(error=r.stderr[-500:])
        print(f"{n}#{rep}", json.dumps(res), flush=True)
