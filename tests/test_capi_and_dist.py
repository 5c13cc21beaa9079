"""CPU-side checks of the boundary and of the multi-rank path.

  * libwbc_hip.so loads and exports every entry point declared in include/wbc.h;
  * the ctypes mirrors of wbc_model / wbc_params have the C layout (gcc sizeof/offsetof);
  * without a GPU the product path fails loudly (no CPU fallback);
  * world_size-2 gloo: each rank solves its shard (C restatement standing in for the HIP step on
    CPU), the torque blocks are all-gathered, and the result equals the single-process batch.
"""
import os
import re
import subprocess
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "wbc.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|const char\*)\s+(wbc_\w+)\s*\(", txt, re.M)))


def test_library_exports_every_declared_symbol():
    from quadrupedwholebodycontroller_amd import _capi

    lib = _capi.load_library()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(_capi.C_API_SYMBOLS) == syms
    out = subprocess.run(["nm", "-D", "--defined-only", _capi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r" T (wbc_\w+)", out))
    assert set(syms) <= exported


def test_struct_layout_matches_c():
    import ctypes as C

    from quadrupedwholebodycontroller_amd import _capi

    src = r"""
#include <stddef.h>
#include <stdio.h>
#include "wbc.h"
int main(void){ printf("%zu %zu %zu %zu %zu %zu\n", sizeof(wbc_model), sizeof(wbc_params), sizeof(wbc_link),
  offsetof(wbc_model, foot), offsetof(wbc_model, total_mass), offsetof(wbc_params, max_wsr)); return 0; }
"""
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "s.c")
        exe = os.path.join(d, "s")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        vals = [int(v) for v in subprocess.run([exe], capture_output=True, text=True).stdout.split()]
    assert vals == [C.sizeof(_capi.WbcModel), C.sizeof(_capi.WbcParams), C.sizeof(_capi.WbcLink),
                    _capi.WbcModel.foot.offset, _capi.WbcModel.total_mass.offset, _capi.WbcParams.max_wsr.offset]


def test_generated_model_header_matches_json():
    """The C initializer (include/wbc_anymal_model.h) and the JSON hold the same constants."""
    import ctypes as C

    import wbc_ref

    m, _ = wbc_ref.model_params()
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "m.c")
        exe = os.path.join(d, "m")
        open(c, "w").write('#include <stdio.h>\n#include "wbc_anymal_model.h"\nint main(void){ fwrite(&WBC_ANYMAL_MODEL, '
                           'sizeof(wbc_model), 1, stdout); return 0; }\n')
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        raw = subprocess.run([exe], capture_output=True).stdout
    assert raw == bytes(C.string_at(C.addressof(m), C.sizeof(m)))


def test_no_silent_cpu_fallback():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from quadrupedwholebodycontroller_amd import Engine, WbcError

    with pytest.raises(WbcError):
        Engine(8)


def test_controller_shim_builds_and_fails_loudly_without_gpu():
    """The C++ WholeBodyController shim (include/wbc_controller.hpp) exports the reference's
    method names, and its node stand-in refuses to run without a HIP device."""
    import torch

    lib = os.path.join(ROOT, "quadrupedwholebodycontroller_amd", "libwbc_controller.so")
    exe = os.path.join(ROOT, "quadrupedwholebodycontroller_amd", "wbc_control_loop")
    assert os.path.exists(lib) and os.path.exists(exe)
    out = subprocess.run(["nm", "-DC", "--defined-only", lib], capture_output=True, text=True).stdout
    for m in ("floatingBaseStateCallback", "jointStateCallback", "referenceCallback", "updateState",
              "setInitialState", "solveQP", "computeJointTorques", "controlLoop", "terminate"):
        assert f"wbc_mi355x::WholeBodyController::{m}(" in out, m
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    r = subprocess.run([exe, "stance", "5"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and "no HIP device" in r.stderr


def test_shard_bounds():
    from quadrupedwholebodycontroller_amd.sharding import shard_bounds

    for total in (1, 7, 4096, 65536, 65537):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [h - l for l, h in spans]
            assert max(sizes) - min(sizes) <= 1


DIST_WORKER = r"""
import os, sys
import numpy as np
import torch, torch.distributed as dist
sys.path.insert(0, {root!r}); sys.path.insert(0, os.path.join({root!r}, "oracle"))
from quadrupedwholebodycontroller_amd import workloads
from quadrupedwholebodycontroller_amd.sharding import (StepOutputs, gather_step_outputs, shard_bounds, shard_capacity,
                                                       unpack_gathered)
import wbc_ref
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
# the collective bench.py runs over RCCL each step (sharding.gather_step_outputs on the packed
# tau | status | iters block), here on CPU tensors: strong shards of an odd-sized batch (padding
# rows), then mode-hypothesis shards in whole states (unit = K rows)
for B, unit in ((67, 1), (5 * 4, 4)):
    inp = workloads.rl_random(B // unit, seed=77 + unit)
    if unit > 1:  # K = unit hypotheses per state, state-major
        inp = {{k: np.repeat(v, unit, axis=0) for k, v in inp.items()}}
        inp["contacts"] = np.tile(np.array([15, 5, 10, 3], np.uint8), B // unit)
    lo, hi = shard_bounds(B // unit, world, rank)
    lo, hi = lo * unit, hi * unit
    out = wbc_ref.run_batch({{k: v[lo:hi] for k, v in inp.items()}}, max_torque=20.0)
    blk = StepOutputs(shard_capacity(B // unit, world) * unit)
    blk.fill(out["tau"], out["status"], out["iters"])
    g = gather_step_outputs(blk, world)
    tau, st, it = unpack_gathered(g, B, world, unit=unit)
    if rank == 0:
        full = wbc_ref.run_batch(inp, max_torque=20.0)
        assert np.array_equal(tau, full["tau"]), "gathered torques differ"
        assert np.array_equal(st, full["status"]) and np.array_equal(it, full["iters"])
print("DIST_OK", rank)
dist.destroy_process_group()
"""


@pytest.mark.parametrize("world", [2, 4])
def test_two_rank_gloo_shard_and_gather(tmp_path, world):
    """world_size 2 (the required rehearsal) and 4 (uneven shards of the odd batches, closer to the
    8-GPU node): shard, gather, unpack, bit-identical to one full-batch run."""
    script = tmp_path / "worker.py"
    script.write_text(DIST_WORKER.format(root=ROOT))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr=127.0.0.1", f"--master-port={29531 + world}", str(script)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert all(f"DIST_OK {k}" in r.stdout for k in range(world))


def test_bench_world_mismatch_exits_nonzero():
    """bench.py --gpus N inside a torch.distributed environment of another size refuses to run
    (it never reports n_gpus different from what was asked)."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


def test_bench_strong_shards_cover_the_global_batch():
    """Strong scaling: the ranks' input shards concatenate to the global batch of the config (so
    the gathered outputs are the same for every N); mode hypotheses shard by whole state."""
    sys.path.insert(0, ROOT)
    import bench

    for name in ("rl_random_b65536", "modes16_x8192"):
        cfg = dict(bench.CONFIGS[name])
        K = cfg.get("modes", 0) or 1
        cfg["batch"] = 96 * K  # small stand-in of the same generator
        _, _, ref, _, tot = bench.shard_inputs(cfg, "strong", 1, 0)
        for world in (2, 3, 8):
            parts = [bench.shard_inputs(cfg, "strong", world, r) for r in range(world)]
            assert sum(p[0] for p in parts) == tot == 96 * K
            for k in ref:
                assert np.array_equal(np.concatenate([p[2][k] for p in parts]), ref[k]), (name, world, k)
