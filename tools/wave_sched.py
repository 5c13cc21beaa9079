"""Wave-schedule probe: where and when every wave of the default step ran (WBC_ISTAMPS build, which
records per wave the constant clock at entry and end, HW_ID, XCC_ID and the workgroup index).

For one launch it reports the kernel's span, the busy time per SIMD, the SIMDs' idle tail, and what
an ideal balance (total busy / SIMDs) and a longest-first list schedule of the measured durations
would give: the headroom a better wave order could reach.
Usage (GPU box): WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so python tools/wave_sched.py [config] [B]"""
import heapq
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quadrupedwholebodycontroller_amd import STATELESS, Engine, workloads  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "rl_random"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
out = sys.argv[3] if len(sys.argv) > 3 else None
e = Engine(B)
if cfg == "trot":
    for s in workloads.trot_sequence(B, steps=60, seed=2):
        e.set_state(s["base_pose"], s["nu"], s["qj"])
        e.set_reference(s["ref"], s["contacts"], s["switching"])
        e.step(0)
else:
    inp = getattr(workloads, cfg)(B, seed=1 if cfg == "stance_cold" else 3)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    for _ in range(3):
        e.step(STATELESS)
e.synchronize()
D = e.debug()
t0 = D[:, 39]
ok = t0 > 0
D = D[ok]
t_in, hw, xcc, t_out, blk = D[:, 39], D[:, 40].astype(np.int64), D[:, 41].astype(np.int64), D[:, 42], D[:, 44]
# one record per workgroup (lane 0 of segment 0 writes its QP's row): keep one row per blk
_, first = np.unique(blk, return_index=True)
t_in, hw, xcc, t_out, blk = t_in[first], hw[first], xcc[first], t_out[first], blk[first].astype(np.int64)
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
sh = (hw >> 12) & 1
se = (hw >> 13) & 7
slot = (((xcc & 15) * 8 + se) * 2 + sh) * 16 * 4 + cu * 4 + simd
base = t_in.min()
t_in = (t_in - base) * 10.0 / 1000.0  # 100 MHz ticks -> us
t_out = (t_out - base) * 10.0 / 1000.0
dur = t_out - t_in
span = t_out.max()
slots = np.unique(slot)
busy = np.zeros(len(slots))
last = np.zeros(len(slots))
cnt = np.zeros(len(slots), dtype=int)
idx = {s: i for i, s in enumerate(slots)}
for s_, d_, o_ in zip(slot, dur, t_out):
    i = idx[s_]
    busy[i] += d_
    last[i] = max(last[i], o_)
    cnt[i] += 1


def list_schedule(durs, n):
    h = [0.0] * n
    heapq.heapify(h)
    for d_ in durs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + d_)
    return max(h)


order = np.argsort(blk)
res = {
    "config": cfg, "batch": B, "waves": int(len(blk)), "simds_used": int(len(slots)),
    "waves_per_simd": np.bincount(cnt).tolist(),
    "span_us": float(span),
    "wave_us": {"mean": float(dur.mean()), "p50": float(np.median(dur)), "p99": float(np.percentile(dur, 99)), "max": float(dur.max())},
    "busy_per_simd_us": {"mean": float(busy.mean()), "max": float(busy.max())},
    "idle_tail_us_mean": float((span - last).mean()),
    "ideal_balance_us": float(busy.sum() / len(slots)),
    "list_schedule_map_order_us": float(list_schedule(dur[order], len(slots))),
    "list_schedule_longest_first_us": float(list_schedule(np.sort(dur)[::-1], len(slots))),
    "start_us_by_dispatch_index": {"first": float(t_in[order][0]), "1024th": float(t_in[order][min(1023, len(order) - 1)]),
                                    "last": float(t_in[order][-1])},
    "xcc_ids": np.unique(xcc).tolist(),
}
print(json.dumps(res, indent=1))
if out:
    np.savez(out, t_in=t_in, t_out=t_out, slot=slot, blk=blk, xcc=xcc)
