"""Batch sharding across GPUs (one process per GPU, torch.distributed over RCCL/xGMI).

Robots are independent (the reference runs one robot per controller object,
src/whole_body_controller.cpp:678-683): rank g owns the contiguous range [lo_g, hi_g) of
`shard_bounds` and keeps its history resident, so the data path has no collective.  The one
exchange is the all-gather of a step's published outputs, so that every rank holds the whole
batch: tau (12 fp64 per robot, cpp:565-576) plus the QP status and the iteration count
(cpp:654) as an int32 pair.

`StepOutputs` is the per-rank buffer the engine writes into (wbc_bind_device_outputs) and
`gather_step_outputs` is the single collective of a step.  bench.py calls exactly these on
RCCL; tests/test_capi_and_dist.py drives the same functions on gloo with CPU tensors.

Packed layout of one rank's block (`cap` robots, the largest shard, so every rank contributes
the same number of bytes, as all_gather_into_tensor requires):

    [ tau: cap x 12 fp64 | status: cap int32 | iters: cap int32 ]    = 13 cap doubles

Rows past a rank's own shard are padding and are dropped by `unpack_gathered`.
"""
from __future__ import annotations

TAU_W = 12            # doubles of tau per robot
ROW_DOUBLES = 13      # tau (12 fp64) + status and iters (2 int32 = 1 double's worth)


def shard_bounds(total: int, world: int, rank: int):
    """Contiguous, balanced [lo, hi) robot range of `rank` (first total % world ranks get one more)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def shard_capacity(total: int, world: int) -> int:
    """Rows every rank's packed block holds: the largest shard."""
    return -(-total // world)


class StepOutputs:
    """One rank's packed output block (torch tensor on the rank's device, or CPU under gloo).

    tau / status / iters are views into `buf`; their data_ptr()s are what the engine binds as
    its output buffers, so a step writes the block in place and the gather reads it directly."""

    def __init__(self, cap: int, device=None):
        import torch

        self.cap = int(cap)
        self.buf = torch.zeros(self.cap * ROW_DOUBLES, dtype=torch.float64, device=device)
        self.tau = self.buf[: self.cap * TAU_W]
        ints = self.buf[self.cap * TAU_W:].view(torch.int32)
        self.status = ints[: self.cap]
        self.iters = ints[self.cap: 2 * self.cap]

    def fill(self, tau, status, iters):
        """Copy host results of n <= cap robots into the block (CPU stand-in for a step)."""
        import torch

        n = len(status)
        self.tau[: n * TAU_W].copy_(torch.as_tensor(tau, dtype=torch.float64).reshape(-1))
        self.status[:n].copy_(torch.as_tensor(status, dtype=torch.int32))
        self.iters[:n].copy_(torch.as_tensor(iters, dtype=torch.int32))


def gather_step_outputs(block: StepOutputs, world: int, out=None, group=None, collective=None):
    """The step's one collective: every rank's packed block, concatenated in rank order
    (RCCL all_gather_into_tensor on GPU tensors; the list form on gloo / CPU).  `out` is an
    optional preallocated [world * 13 cap] fp64 tensor.  With one rank there is nothing to gather
    and the block is returned (copied into `out`) unless `collective` is True: then the collective
    runs anyway (a one-rank process group), which is how tests/test_gpu_rccl.py executes the RCCL
    branch on a one-GPU box."""
    import torch
    import torch.distributed as dist

    local = block.buf
    if collective is None:
        collective = world > 1
    if not collective:
        if out is not None:
            out.copy_(local)
            return out
        return local
    if out is None:
        out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
    if local.is_cuda and dist.get_backend(group) != "gloo":
        dist.all_gather_into_tensor(out, local, group=group)
    elif local.is_cuda:  # gloo rehearsal of the GPU path (several ranks on one device): via host
        host = torch.empty(out.numel(), dtype=out.dtype)
        dist.all_gather(list(host.view(world, local.numel()).unbind(0)), local.cpu(), group=group)
        out.copy_(host)
    else:
        parts = list(out.view(world, local.numel()).unbind(0))
        dist.all_gather(parts, local, group=group)
    return out


def unpack_gathered(gathered, total: int, world: int, unit: int = 1):
    """Gathered blocks -> (tau [total, 12], status [total], iters [total]) as numpy arrays, in
    global robot order (padding rows of the shorter shards dropped).  Shards are whole groups of
    `unit` rows (mode hypotheses: the K QPs of one state), cap = shard_capacity(total / unit) unit."""
    import numpy as np
    import torch

    units = total // unit
    cap = shard_capacity(units, world) * unit
    g = gathered.detach().to("cpu").view(world, cap * ROW_DOUBLES)
    taus, sts, its = [], [], []
    for r in range(world):
        lo, hi = shard_bounds(units, world, r)
        n = (hi - lo) * unit
        blk = g[r]
        taus.append(blk[: cap * TAU_W].reshape(cap, TAU_W)[:n])
        ints = blk[cap * TAU_W:].contiguous().view(torch.int32)
        sts.append(ints[:n])
        its.append(ints[cap: cap + n])
    return (torch.cat(taus).numpy(), torch.cat(sts).numpy().astype(np.int32),
            torch.cat(its).numpy().astype(np.int32))


def all_gather_rows(local, world: int, group=None):
    """Concatenate every rank's equal-length 1-D block (RCCL all_gather_into_tensor on GPU tensors;
    the list form on gloo/CPU)."""
    import torch
    import torch.distributed as dist

    if world == 1:
        return local
    if local.is_cuda:
        out = torch.empty(world * local.numel(), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, local.contiguous(), group=group)
        return out
    parts = [torch.empty_like(local) for _ in range(world)]
    dist.all_gather(parts, local.contiguous(), group=group)
    return torch.cat(parts)


class StepPipeline:
    """The per-step loop of bench.py on N ranks: every step writes the rank's outputs straight into a
    packed block (StepOutputs, bound as the engine's output buffers) and the step's one collective
    gathers the blocks on a second stream, overlapped with the next steps.  `nbuf` blocks rotate: step
    k + nbuf waits for the gather of step k (an event on `comm`) before the engine overwrites its block.

    engine: the rank's Engine (on `stream`); step(flags) runs one step (Engine.step or step_modes);
    cap: rows of a block (the largest shard).  With world == 1 there is no gather (the block is the
    whole batch's output).  tests/test_gpu_pipeline.py runs this class with two gloo ranks on one GPU
    and checks every step's gathered outputs against a one-rank step."""

    def __init__(self, engine, step, flags, world, cap, stream, comm=None, device="cuda", group=None, collective=None,
                 nbuf=3):
        """collective: gather every step (default: world > 1); True with world == 1 runs the gather
        path on a one-rank process group (tests/test_gpu_rccl.py).  nbuf: output blocks in rotation,
        so that a gather may take up to nbuf - 1 steps before the compute stream waits for it (three:
        one RCCL all-gather of an 8-rank step is about as long as the step itself)."""
        import torch

        self.torch = torch
        self.e, self.step_fn, self.flags, self.world = engine, step, flags, world
        self.coll = (world > 1) if collective is None else bool(collective)
        self.stream, self.comm, self.group = stream, comm, group
        self.cap = cap
        self.nbuf = max(2, int(nbuf))
        self.blocks = [StepOutputs(cap, device=device) for _ in range(self.nbuf)]
        self.gathered = ([torch.empty(world * cap * ROW_DOUBLES, dtype=torch.float64, device=device)
                          for _ in range(self.nbuf)] if self.coll else None)
        self.ev_step = [torch.cuda.Event() for _ in range(self.nbuf)]
        self.ev_gath = [torch.cuda.Event() for _ in range(self.nbuf)]
        self.used = [False] * self.nbuf
        self.k = 0

    def bind(self, slot):
        b = self.blocks[slot]
        self.e.bind_device_outputs(tau=b.tau.data_ptr(), status=b.status.data_ptr(), iters=b.iters.data_ptr())

    def step(self):
        """Queue one step (and, N > 1, its gather); returns the slot its outputs land in."""
        torch = self.torch
        slot = self.k % self.nbuf
        if self.coll and self.used[slot]:
            self.stream.wait_event(self.ev_gath[slot])  # the gather of step k - nbuf has read this block
        self.bind(slot)
        self.step_fn(self.flags)
        if self.coll:
            self.ev_step[slot].record(self.stream)
            with torch.cuda.stream(self.comm):
                self.comm.wait_event(self.ev_step[slot])
                gather_step_outputs(self.blocks[slot], self.world, out=self.gathered[slot], group=self.group,
                                    collective=True)
                self.ev_gath[slot].record(self.comm)
            self.used[slot] = True
        self.k += 1
        return slot

    @property
    def last_slot(self):
        return (self.k - 1) % self.nbuf

    def prev_slot(self, slot):
        """The slot of the step queued before the one in `slot`."""
        return (slot - 1) % self.nbuf

    def result(self, slot, total, unit=1):
        """(tau, status, iters) of the step in `slot` for the whole batch (numpy, global order) once its
        gather is done; `total` QPs overall (N > 1) or this rank's (N = 1)."""
        import numpy as np

        if self.coll:
            self.ev_gath[slot].synchronize()
            return unpack_gathered(self.gathered[slot], total, self.world, unit=unit)
        self.ev_step[slot].record(self.stream)
        self.ev_step[slot].synchronize()
        b = self.blocks[slot]
        return (b.tau[: total * TAU_W].cpu().numpy().reshape(total, TAU_W),
                b.status[:total].cpu().numpy().astype(np.int32), b.iters[:total].cpu().numpy().astype(np.int32))
