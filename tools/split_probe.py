"""A/B: fused wbc_step vs split wbc_update + wbc_solve, per library variant (each in its own process).
Usage (GPU box): python tools/split_probe.py steps lib1,lib2,...  (names of quadrupedwholebodycontroller_amd/libwbc_hip_<name>.so)"""
import json, os, subprocess, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, sys
sys.path.insert(0, %r)
import numpy as np, torch
from quadrupedwholebodycontroller_amd import FUSED, NO_X, STATELESS, Engine, workloads
steps = int(sys.argv[1]); F = STATELESS | NO_X
res = {}
for name, gen, B in (("stance_cold_b4096", workloads.stance_cold, 4096), ("rl_random_b8192", workloads.rl_random, 8192)):
    inp = gen(B, seed=1); e = Engine(B)
    st = torch.cuda.Stream(); torch.cuda.set_stream(st); e.set_stream(st.cuda_stream)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"]); e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    def t(fn):
        for _ in range(3): fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        for _ in range(steps): fn()
        b.record(st); torch.cuda.synchronize(); return a.elapsed_time(b) / steps
    fused = t(lambda: e.step(F | FUSED)); o1 = e.outputs()
    upd = t(lambda: e.update(F))
    split = t(lambda: (e.update(F), e.solve(F))); o2 = e.outputs()
    res[name] = dict(fused_ms=fused, update_ms=upd, split_ms=split, same=bool(np.array_equal(o1["tau"], o2["tau"])))
    e.close()
print(json.dumps(res))
''' % ROOT
steps = sys.argv[1] if len(sys.argv) > 1 else "30"
for n in sys.argv[2].split(","):
    lib = os.path.join(ROOT, "quadrupedwholebodycontroller_amd", f"libwbc_hip_{n}.so")
    r = subprocess.run([sys.executable, "-c", CHILD, steps], env=dict(os.environ, WBC_LIB=lib), capture_output=True, text=True, timeout=300)
    print(n, r.stdout.strip().splitlines()[-1] if r.returncode == 0 else r.stderr[-800:], flush=True)
