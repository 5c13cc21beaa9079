"""GPU: the RCCL branch of the multi-rank step, executed on a one-GPU box.

bench.py on N > 1 GPUs initialises `init_process_group("nccl", device_id=cuda:<local rank>)` (nccl is
RCCL on ROCm) and gathers every step's packed tau | status | iters block with
`all_gather_into_tensor` on a second stream (sharding.StepPipeline).  Two ranks cannot
share one GPU under RCCL, so the multi-rank tests rehearse that loop over gloo; this test runs the
RCCL calls themselves on a one-rank process group, launched as bench.py is (torch.distributed.run,
a fresh child process before anything touches the GPU):

  * the nccl process group with `device_id`, as bench.py creates it;
  * sharding.gather_step_outputs through its RCCL branch (collective=True bypasses the one-rank
    short-cut): the gathered block equals the engine's outputs bit for bit;
  * StepPipeline with a real `comm` stream and collective=True over 8 steps with changing inputs
    bound in HBM: each step's gathered outputs equal a separate engine's step on the same inputs;
  * bench.py's barrier and the max-over-ranks all_reduce of the elapsed time."""
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
sys.path.insert(0, {root!r})
from quadrupedwholebodycontroller_amd import NO_X, STATELESS, Engine, workloads
from quadrupedwholebodycontroller_amd.sharding import StepOutputs, StepPipeline, gather_step_outputs, unpack_gathered
local_rank = int(os.environ["LOCAL_RANK"])
torch.cuda.set_device(local_rank)
dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))  # bench.py's call
world = dist.get_world_size()
assert dist.get_backend() == "nccl" and world == 1
FLAGS = STATELESS | NO_X
KEYS = ("base_pose", "nu", "qj", "ref", "contacts", "switching")
B, STEPS = 1337, 8

def step_inputs(inp, k):
    s = {{kk: v.copy() for kk, v in inp.items()}}
    s["qj"] = s["qj"] + 0.003 * np.sin(k + np.arange(s["qj"].size).reshape(s["qj"].shape))
    s["nu"] = s["nu"] * (1.0 + 0.05 * k)
    return s

def engine_step(s):
    e = Engine(B, device=local_rank)
    e.set_state(s["base_pose"], s["nu"], s["qj"])
    e.set_reference(s["ref"], s["contacts"], s["switching"])
    e.step(FLAGS)
    o = e.outputs()
    e.close()
    return o

seq = [step_inputs(workloads.rl_random(B, seed=61), k) for k in range(STEPS)]
ref = [engine_step(s) for s in seq]

# 1. the gather alone: the block the engine wrote, through all_gather_into_tensor
blk = StepOutputs(B, device="cuda")
blk.fill(ref[0]["tau"], ref[0]["status"], ref[0]["iters"])
g = gather_step_outputs(blk, world, collective=True)
torch.cuda.synchronize()
assert g.data_ptr() != blk.buf.data_ptr()
tau, st, it = unpack_gathered(g, B, world)
assert np.array_equal(tau, ref[0]["tau"]) and np.array_equal(st, ref[0]["status"]) and np.array_equal(it, ref[0]["iters"])
print("GATHER_OK", flush=True)

# 2. bench.py's step loop: outputs bound into the packed blocks, the gather on `comm`
stream, comm = torch.cuda.Stream(), torch.cuda.Stream()
torch.cuda.set_stream(stream)
dev = {{kk: torch.from_numpy(np.ascontiguousarray(np.stack([s[kk] for s in seq]))).cuda() for kk in KEYS}}
e = Engine(B, device=local_rank)
e.set_stream(stream)
pipe = StepPipeline(e, e.step, FLAGS, world, B, stream, comm, collective=True)
results = []
dist.barrier()
for k in range(STEPS):
    e.bind_device_inputs(*[dev[kk][k].data_ptr() for kk in KEYS])
    slot = pipe.step()
    if k >= 1:  # the previous step's gather, read while this step runs
        results.append(pipe.result(pipe.prev_slot(slot), B))
results.append(pipe.result(pipe.last_slot, B))
torch.cuda.synchronize()
dist.barrier()
tt = torch.tensor([0.25], dtype=torch.float64, device="cuda")
dist.all_reduce(tt, op=dist.ReduceOp.MAX)
assert float(tt.item()) == 0.25
e.close()
for k in range(STEPS):
    tau, st, it = results[k]
    assert np.array_equal(tau, ref[k]["tau"]), (k, "tau")
    assert np.array_equal(st, ref[k]["status"]) and np.array_equal(it, ref[k]["iters"]), k
print("PIPE_OK", flush=True)
dist.destroy_process_group()
"""


def test_rccl_gather_and_step_pipeline_on_one_rank(tmp_path):
    script = tmp_path / "worker.py"
    script.write_text(WORKER.format(root=ROOT))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", "--master-port=29547", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-1000:], r.stderr[-3000:])
    assert "GATHER_OK" in r.stdout and "PIPE_OK" in r.stdout
