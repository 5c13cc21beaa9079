"""GPU probe: the device-built wave map under WBC_GROUP against no map, for device-bound
contact masks (the RL-environment case), on the rl_random batch at B = 8192 and 65536.

Per batch it times back-to-back wbc_step(STATELESS | NO_X [| GROUP]) with HIP events on the engine
stream and prints one JSON line: ms per step and M solves/s with and without the map, and the two
paths' outputs compared (they must be identical: the map only changes which QPs share a wave).
The map kernel's own duration comes from a rocprofv3 kernel trace of the same command
(wbc_qmap_kernel in kernel_stats.csv).

Usage (GPU box): python tools/qmap_probe.py [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from quadrupedwholebodycontroller_amd import GROUP, NO_X, STATELESS, Engine, workloads  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    for B in (8192, 65536):
        inp = workloads.rl_random(B, seed=3)
        d = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in inp.items()}
        st = torch.cuda.Stream()
        torch.cuda.set_stream(st)
        res = dict(batch=B)
        outs = {}
        for name, fl in (("no_map", STATELESS | NO_X), ("group", STATELESS | NO_X | GROUP)):
            e = Engine(B)
            e.set_stream(st.cuda_stream)
            e.bind_device_inputs(d["base_pose"].data_ptr(), d["nu"].data_ptr(), d["qj"].data_ptr(), d["ref"].data_ptr(),
                                 d["contacts"].data_ptr(), d["switching"].data_ptr())
            for _ in range(3):
                e.step(fl)
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(st)
            for _ in range(steps):
                e.step(fl)
            ev1.record(st)
            torch.cuda.synchronize()
            ms = ev0.elapsed_time(ev1) / steps
            res[name] = dict(ms=round(ms, 4), msolves_per_s=round(B / ms * 1e-3, 2))
            outs[name] = e.outputs()
            e.close()
        res["identical"] = all(np.array_equal(outs["no_map"][k], outs["group"][k]) for k in ("tau", "grf", "status", "iters"))
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
