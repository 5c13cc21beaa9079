"""GPU: the multi-rank step on the HIP engine, rehearsed with two ranks sharing
cuda:0 over gloo: each rank runs the engine (wbc_step) on its contiguous shard of the batch, packs
tau | status | iters into its StepOutputs block and the blocks are gathered
(sharding.gather_step_outputs, the code bench.py runs over RCCL).  Rank 0 checks the gathered batch
against one full-batch engine run on the same device (bit-identical on both batches: the step groups
its QPs by contact mask, so a robot's result does not depend on the shard boundary) and against the C oracle (status equal,
tau to 1e-9, tests/margins.py TAU) for a batch over all 16 contact masks.  The reference's own step is per robot
(cpp:650-652), so sharding robots across ranks is exact."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = r"""
import os, sys
import numpy as np
import torch, torch.distributed as dist
sys.path.insert(0, {root!r}); sys.path.insert(0, os.path.join({root!r}, "oracle"))
from quadrupedwholebodycontroller_amd import STATELESS, Engine, workloads
from quadrupedwholebodycontroller_amd.sharding import (StepOutputs, gather_step_outputs, shard_bounds, shard_capacity,
                                                       unpack_gathered)
import wbc_ref
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()

def engine_run(inp):
    B = inp["base_pose"].shape[0]
    e = Engine(B, device=0)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    e.step(STATELESS)
    o = e.outputs()
    e.close()
    return o

for name, inp in (("stance", workloads.stance_cold(1031, seed=5)), ("rl_random", workloads.rl_random(515, seed=6))):
    B = inp["base_pose"].shape[0]
    lo, hi = shard_bounds(B, world, rank)
    out = engine_run({{k: v[lo:hi] for k, v in inp.items()}})
    blk = StepOutputs(shard_capacity(B, world))
    blk.fill(out["tau"], out["status"], out["iters"])
    g = gather_step_outputs(blk, world)
    tau, st, it = unpack_gathered(g, B, world)
    if rank == 0:
        full = engine_run(inp)
        # bit-identical for every batch: waves hold one contact mask each, so a robot's result does
        # not depend on where the shard boundary falls
        assert np.array_equal(tau, full["tau"]), ("gathered torques differ from the full-batch step", name)
        assert np.array_equal(st, full["status"]) and np.array_equal(it, full["iters"]), name
        o = wbc_ref.run_batch(inp)
        assert np.array_equal(st, o["status"]), name
        ok = st == 0
        err = np.max(np.abs(tau[ok] - o["tau"][ok])) / (1.0 + np.max(np.abs(o["tau"][ok])))
        assert err < 1e-9, (name, err)
        print("CHECKED", name, B, float(err), flush=True)
print("DIST_OK", rank, flush=True)
dist.destroy_process_group()
"""


def test_two_rank_engine_shards_gather_to_the_full_batch(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29533", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-3000:])
    assert "DIST_OK 0" in r.stdout and "DIST_OK 1" in r.stdout
    assert "CHECKED stance" in r.stdout and "CHECKED rl_random" in r.stdout
