"""Diagnostic: robots on which the split form (WBC_SPLIT, the 24-variable QP) and the C oracle's
LITERAL method (the 42 x 70 QP) count different working-set changes on the stress inputs of
tests/test_gpu_iters.py.  Writes the robots' inputs and both counts to gpurun_out/split_diverge.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import wbc_ref as R  # noqa: E402
from test_gpu_iters import CASES, engine_cold  # noqa: E402

from quadrupedwholebodycontroller_amd import SPLIT  # noqa: E402

out = {}
for case in ("stress6", "stress20", "stress80", "rl_random"):
    gen, ov, _ = CASES[case]
    inp = gen()
    g = engine_cold(inp, SPLIT, **ov)
    o = R.run_batch(inp, method=R.LITERAL, **ov)
    bad = np.nonzero(g["iters"] != o["iters"])[0]
    print(case, "mismatched robots", bad.tolist(), "engine", g["iters"][bad].tolist(), "oracle", o["iters"][bad].tolist(),
          "status", g["status"][bad].tolist(), flush=True)
    out[case + "_rows"] = bad
    out[case + "_g_iters"] = g["iters"]
    out[case + "_o_iters"] = o["iters"]
    if os.environ.get("WBC_QTRACE"):
        out[case + "_dbg"] = g.get("dbg", np.zeros(0))
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", "split_diverge.npz"), **out)
