"""configs[4]'s shard (1024 states x 16 contact masks, wbc_step_modes) against the mode loop's
hypotheses per wave (WBC_MODES_M: 1 = one hypothesis per segment, wbc_update_solve_kernel; M > 1 =
wbc_modes_kernel, one update per state and wave), and the engine's own choice.  DESIGN.md 4.14.
Usage (GPU box): python tools/modes_sweep.py [steps]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from quadrupedwholebodycontroller_amd import NO_X, STATELESS, Engine, workloads  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
S = int(os.environ.get("SWEEP_STATES", "1024"))
inp, modes = workloads.mode_states(S, 4)
ref = None
for m in (None, 1, 2, 4, 8, 16):
    if m is None:
        os.environ.pop("WBC_MODES_M", None)
    else:
        os.environ["WBC_MODES_M"] = str(m)
    e = Engine(S * 16)
    st = torch.cuda.Stream()
    torch.cuda.set_stream(st)
    e.set_stream(st)
    e.set_modes(modes)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    F = STATELESS | NO_X
    for _ in range(3):
        e.step_modes(F)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record(st)
    for _ in range(steps):
        e.step_modes(F)
    ev1.record(st)
    torch.cuda.synchronize()
    ms = ev0.elapsed_time(ev1) / steps
    o = e.outputs()
    e.close()
    if ref is None:
        ref = o
    same = all(np.array_equal(o[k], ref[k]) for k in ("tau", "grf", "status", "iters"))
    print(json.dumps(dict(M="auto" if m is None else m, ms=round(ms, 4), solves_per_s_M=round(S * 16 / ms / 1e3, 2),
                          bit_identical_to_auto=same)), flush=True)
os.environ.pop("WBC_MODES_M", None)
