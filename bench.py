#!/usr/bin/env python3
"""Benchmark: batched ANYmal WBC QP solves/s on MI355X (BASELINE.json metric).

One step = one wbc_step over the rank's batch (dynamics + centroidal assembly + QP + torques: one
kernel, wbc_update_solve_kernel, four QPs per wave, each reduced exactly to 12 variables and
solved in place; a QP whose reduction is not usable is solved by the same wave's general method;
mode hypotheses with many states: wbc_modes_kernel, one update per state and wave), plus for N > 1 the RCCL all-gather of the torque block.  Inputs are
resident in HBM before the timed region.  Default workload: configs[1] of BASELINE.json,
B = 4096 four-contact stance states, cold solves, per GPU (weak scaling).

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under torch.distributed.run.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6   # MI355X fp64 dense peak (vector = matrix on gfx950; AMD spec, = 1/2 of 157.3 TF fp32)
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s
# algorithmic flops per solve F(k) = F_dyn + F_asm + F_tau + F_fact + k F_iter
F_DYN, F_ASM, F_TAU, F_FACT, F_ITER = 9000, 14000, 600, 24696, 12936
BYTES_COLD = 929          # 729 B in + 200 B out per cold solve
BYTES_IN, BYTES_OUT = 729, 200  # per state read / per QP written (mode hypotheses share the state read)
# configs[2] (stateful): SURVEY.md 8(d)'s 11 457 B per solve (the reference's per-robot history read and
# written each cycle, hpp:154-161); the engine's own compact history (wbc_layout.h HistOff, 350 doubles)
# read and written once per step: 729 B in + 200 B out + 2 x 2 800 B = 6 529 B per solve
BYTES_TROT_SURVEY = 11457
BYTES_TROT_ENGINE = BYTES_IN + BYTES_OUT + 2 * 350 * 8

CONFIGS = {
    "stance_cold_b4096": dict(gen="stance_cold", batch=4096, seed=1, scaling="weak",
                              desc="BASELINE configs[1]: B=4096 4-contact stance QPs, fp64, cold start"),
    "rl_random_b8192": dict(gen="rl_random", batch=8192, seed=3, scaling="weak",
                            desc="BASELINE configs[3] per-GPU shard: randomized q/qd, 16 contact masks, cold"),
    "modes16_b16384": dict(gen="modes16", batch=16384, seed=4, modes=16, scaling="weak",
                           desc="BASELINE configs[4] per-GPU shard: 1024 states x all 16 contact masks, cold; "
                                "wbc_step_modes (the mode loop: one update per state and wave, then four "
                                "hypotheses in turn, wbc_modes_kernel)"),
    # the two multi-GPU configurations at their global sizes (strong scaling: total work fixed)
    "rl_random_b65536": dict(gen="rl_random", batch=65536, seed=3, scaling="strong",
                             desc="BASELINE configs[3]: global B=65536 randomized q/qd (16 contact masks, cold), "
                                  "contiguous robot shards per GPU"),
    "modes16_x8192": dict(gen="modes16", batch=131072, seed=4, modes=16, scaling="strong",
                          desc="BASELINE configs[4]: 8192 states x 16 contact masks = 131072 QPs, sharded by state "
                               "(a state's 16 hypotheses on one GPU)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def _native_baseline_lib():
    """Build the CPU baseline with -march=native for this host into a temp dir; the
    portable x86-64-v3 build (oracle/_build/libwbc_ref.so) if that fails.  Returns (path or None, note)."""
    import tempfile

    out = os.path.join(tempfile.gettempdir(), f"wbc_cpu_native_{os.getpid()}.so")
    try:
        r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native", f"NATIVE_OUT={out}"],
                           capture_output=True, text=True, timeout=120)
        if r.returncode == 0 and os.path.exists(out):
            return out, "-O3 -march=native -fopenmp (built on this host)"
        return None, "-O3 -march=x86-64-v3 -fopenmp (native build failed: %s)" % r.stderr.strip()[-200:]
    except (OSError, subprocess.SubprocessError) as ex:
        return None, "-O3 -march=x86-64-v3 -fopenmp (native build failed: %s)" % ex


def cpu_baseline(inp, budget_s=15.0, threads=None):
    """Time the CPU restatements on a bounded sample of the same inputs (inputs cycled), one robot
    per OpenMP thread (static schedule), as SURVEY.md 8d prescribes, in two variants:
      * structure-exploiting (oracle/wbc_fast.c): the GPU engine's algorithm (closed-form
        centroidal transform, reduced QP, stance elimination) -> the reported `value`;
      * reference-faithful (oracle/wbc_ref.c): dense 18x18 LU inverses, dense 42 x 70 active set.
    Each on `threads` threads (default min(16, nproc): the GPU box's CPU share, OMP_NUM_THREADS
    there) and on one thread."""
    lib_path = os.path.join(ROOT, "oracle", "_build", "libwbc_ref.so")
    B = inp["base_pose"].shape[0]
    if not os.path.exists(lib_path):
        return _cpu_baseline_numpy(inp, budget_s)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wbc_ref  # ctypes wrapper of the C restatements

    T = threads or max(1, min(16, os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16") or 16)))
    native, build_note = _native_baseline_lib()

    def sample(n):
        idx = np.arange(n) % B
        return {k: np.ascontiguousarray(v[idx]) for k, v in inp.items()}

    def run(variant, n, nthreads, budget):
        t_used = 0.0
        while True:
            sub = sample(n)
            t0 = time.perf_counter()
            wbc_ref.cpu_run_batch(sub, variant, nthreads, native)
            dt = time.perf_counter() - t0
            t_used += dt
            if dt >= 0.8 * budget or t_used >= 2.5 * budget:
                return n, dt
            n = int(n * max(2.0, min(10.0, budget / max(dt, 1e-6))))

    res = {}
    for variant, share in (("fast", 0.5), ("dense", 0.5)):
        b = budget_s * share
        n1, dt1 = run(variant, 64, 1, b / 4)
        nT, dtT = run(variant, 64 * T, T, 3 * b / 4)
        res[variant] = dict(value=nT / dtT, unit="solves/s", cores=T, kind="port",
                            sample=f"{nT} cold solves of the same workload (inputs cycled), {T} OpenMP threads, "
                                   f"{dtT:.2f} s",
                            single_core=dict(value=n1 / dt1, cores=1, sample=f"{n1} cold solves, 1 thread, {dt1:.2f} s"))
    if native:
        try:
            os.remove(native)
        except OSError:
            pass
    out = dict(res["fast"])
    out["variant"] = ("structure-exploiting (oracle/wbc_fast.c: the engine's algorithm - closed-form centroidal "
                      "transform, reduced QP, four-contact equality elimination - dense Goldfarb-Idnani per robot)")
    out["build"] = build_note
    out["reference_faithful"] = dict(res["dense"], variant="oracle/wbc_ref.c: seven dense 18x18 LU inverses, dense "
                                                         "42 x 70 Goldfarb-Idnani (src/whole_body_controller.cpp:256-542)")
    out["note"] = (f"{T} threads is the GPU box's CPU share (OMP_NUM_THREADS); the box's other cores belong to "
                   f"other jobs, so the all-core figure is not taken")
    return out


def _cpu_baseline_numpy(inp, budget_s):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import wbc_np as W

    B = inp["base_pose"].shape[0]
    model, params = W.Model(), W.default_params()
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < budget_s and n < B:
        c = W.ReferenceWBC(model, params)
        c.set_state(inp["base_pose"][n], inp["nu"][n], inp["qj"][n])
        c.set_reference(inp["ref"][n], [(int(inp["contacts"][n]) >> i) & 1 for i in range(4)], True)
        c.step()
        n += 1
    dt = time.perf_counter() - t0
    return dict(value=n / dt, unit="solves/s", cores=1, kind="port",
                sample=f"{n} cold solves through oracle/wbc_np.py (numpy restatement), 1 thread, {dt:.2f} s")


def committed_pmc(workload, batch):
    """The committed PMC summary (tools/pmc_summary.py) taken on this exact kernel source, workload and
    batch, and its path; (None, None) if none."""
    import glob

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from pmc_summary import kernel_source_hash

    want = kernel_source_hash()
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "pmc_*.json")), reverse=True):
        try:
            rec = json.load(open(f))
        except (OSError, ValueError):
            continue
        if (rec.get("kernel_source_sha256") == want and rec.get("workload") == workload and
                rec.get("batch") == batch and "traffic" in rec):
            return rec, os.path.relpath(f, ROOT)
    return None, None


def committed_traffic(workload, batch):
    """HBM bytes per launch, per kernel and per step, from the committed PMC summary; {} if none."""
    rec, src = committed_pmc(workload, batch)
    return (rec["traffic"], src) if rec else ({}, None)


def executed_fp64(workload, batch, kernel, kernel_ms):
    """The fp64 VALU work the kernel actually issued (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 x 64 lanes, an
    FMA counted twice, every lane of an issued instruction counted) per launch, from the committed PMC
    summary, over this run's kernel time: TFLOP/s and the fraction of the fp64 peak; None without it."""
    rec, src = committed_pmc(workload, batch)
    f = (rec or {}).get("fp64_executed_flops", {}).get(kernel)
    if not f:
        return None
    tf = f / (kernel_ms * 1e-3) / 1e12
    return {"flops_per_launch": f, "achieved": tf, "frac": tf / FP64_PEAK_TFLOPS, "source": src,
            "note": "issued fp64 VALU lane-operations (64 lanes per instruction, masked lanes included) from the "
                    "PMC counters, beside the reference-equivalent flops of SURVEY 8(d) used for frac"}


def step_flops(S, iters):
    """SURVEY 8(d) algorithmic flops of one step: F_dyn + F_asm per state (mode hypotheses share
    their state's dynamics), F_fact + F_tau + k F_iter per QP with k = iters[] (the working-set
    changes of the form the engine solved)."""
    iters = np.asarray(iters, np.int64)
    return float(S * (F_DYN + F_ASM) + np.sum(F_FACT + F_TAU + F_ITER * iters))


def step_kernel(e):
    """The one kernel of the engine's default step: wbc_modes_kernel under the mode loop (mode
    hypotheses, many states), wbc_update_solve_kernel otherwise."""
    return "wbc_modes_kernel" if e.modes_per_wave() > 1 else "wbc_update_solve_kernel"


def kernel_instance(e, config):
    """Which instance of the step kernel ran, and its translation unit (each under its own
    schedule): the engine launches the stance-only instance for a stateless
    step whose masks are all 15, the mixed-form instance for any other stateless step."""
    if e.modes_per_wave() > 1:
        return "wbc_modes_kernel (wbc_kernel_modes.hip)"
    if config.startswith("stance"):
        return "wbc_update_solve_kernel<0, true> (stance-only: wbc_kernel_stance.hip)"
    return "wbc_update_solve_kernel<0, false> (every contact mask: wbc_kernel_step0.hip)"


def roofline_of(flops, kernel_ms, traffic=None, traffic_src=None, kernel="wbc_update_solve_kernel"):
    tf = flops / (kernel_ms * 1e-3) / 1e12
    return {"bound": "fp64_valu", "achieved": tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": tf / FP64_PEAK_TFLOPS, "traffic": traffic, "traffic_source": traffic_src,
            "kernel": kernel, "kernel_ms": kernel_ms, "flops_per_launch": flops}


def make_engine(cfg, B, seed, device, stream):
    """Engine for a bench config on `stream`, inputs loaded; returns (engine, step flags fn, inputs).
    Mode-hypothesis configs hold B / K states and step with wbc_step_modes."""
    from quadrupedwholebodycontroller_amd import Engine, workloads

    K = cfg.get("modes", 0)
    e = Engine(B, device=device)
    e.set_stream(stream)
    if K:
        inp, modes = workloads.mode_states(B // K, seed)
        e.set_modes(modes)
    else:
        inp = getattr(workloads, cfg["gen"])(B, seed=seed)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    return e, (e.step_modes if K else e.step), inp


def bench_trot(torch, stream, device, STATELESS, B=4096, T=400, seed=2):
    """BASELINE configs[2]: B robots trotting for T cycles (1 s at 400 Hz), alternating 2-contact
    modes, history carried across steps (stateful path: finite differences, Tdot_inv lag, integral
    error).  All T steps of inputs are staged in HBM first and bound per step (no copies timed)."""
    from quadrupedwholebodycontroller_amd import NO_X, Engine, workloads

    seq = list(workloads.trot_sequence(B, steps=T, seed=seed))
    dev = {k: torch.from_numpy(np.ascontiguousarray(np.stack([s[k] for s in seq]))).to(f"cuda:{device}")
           for k in seq[0]}
    e = Engine(B, device=device)
    e.set_stream(stream)

    def run(iters_out=None):
        e.reset()
        for t in range(T):
            e.bind_device_inputs(dev["base_pose"][t].data_ptr(), dev["nu"][t].data_ptr(), dev["qj"][t].data_ptr(),
                                 dev["ref"][t].data_ptr(), dev["contacts"][t].data_ptr(),
                                 dev["switching"][t].data_ptr())
            e.step(NO_X)  # stateful
            if iters_out is not None:
                iters_out.append(e.outputs()["iters"].astype(np.int64))

    its = []
    run(its)  # warm-up pass; its iteration counts (the same inputs every pass) for the flop count
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    run()
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    ms = ev0.elapsed_time(ev1)
    o = e.outputs()
    e.close()
    its = np.stack(its)
    tr, tr_src = committed_traffic("trot_stateful_b4096", B)
    rl = roofline_of(step_flops(B * T, its) / T, ms / T, tr.get("step"), tr_src)
    rl["note"] = "per step (one wbc_update_solve_kernel launch): flops of the 400-step " \
                 "sequence / 400 over the sequence's HIP-event time / 400"
    rl["executed_fp64"] = executed_fp64("trot_stateful_b4096", B, "wbc_update_solve_kernel", ms / T)
    step_s = ms / T * 1e-3
    hbm = {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "achieved": B * BYTES_TROT_ENGINE / step_s / 1e9,
           "frac": B * BYTES_TROT_ENGINE / step_s / 1e9 / HBM_PEAK_GBS,
           "achieved_survey_bytes": B * BYTES_TROT_SURVEY / step_s / 1e9,
           "frac_survey_bytes": B * BYTES_TROT_SURVEY / step_s / 1e9 / HBM_PEAK_GBS,
           "traffic": tr.get("step"), "traffic_source": tr_src,
           "traffic_achieved": (tr["step"] / step_s / 1e9) if tr.get("step") else None,
           "note": "algorithmic bytes per solve: the engine's (729 B inputs + 200 B outputs + its 350-double "
                   "history read and written) = %d B; SURVEY 8(d)'s (the reference's per-robot history) = %d B; "
                   "traffic = PMC bytes per launch (profiles/*/pmc_trot_stateful_b4096.json)"
                   % (BYTES_TROT_ENGINE, BYTES_TROT_SURVEY)}
    return dict(batch=B, steps=T, ms_total=ms, ms_per_step=ms / T, solves_per_s=B * T / (ms * 1e-3),
                wall_solves_per_s=B * T / wall, status_counts_last=np.bincount(o["status"], minlength=4).tolist(),
                mean_iters_last=float(o["iters"].mean()), mean_iters=float(its.mean()), roofline=rl,
                roofline_hbm=hbm, traffic_per_step=tr.get("step"), traffic_source=tr_src,
                algorithmic_bytes_per_step=dict(engine=float(B * BYTES_TROT_ENGINE), survey=float(B * BYTES_TROT_SURVEY)),
                desc="BASELINE configs[2]: trot, alternating 2-contact modes, stateful history, inputs staged in HBM")


def _self_launch(n):
    """`--gpus N` without a torch.distributed environment: run this same command as N ranks under
    torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) as a child process and
    return its exit code.  Nothing here has touched the GPU yet."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd, env=env).returncode


def shard_inputs(cfg, scaling, world, rank):
    """Inputs of this rank: (B_rank QPs, S_rank input rows, inputs, modes or None, global QPs).
    weak: a full per-GPU batch, seed + 1000 rank; strong: the rank's contiguous shard of the
    global batch (mode hypotheses shard by state, so a state's 16 QPs stay on one rank)."""
    from quadrupedwholebodycontroller_amd import workloads
    from quadrupedwholebodycontroller_amd.sharding import shard_bounds

    K = cfg.get("modes", 0)
    B = cfg["batch"]
    S = B // K if K else B
    if scaling == "weak":
        seed = cfg["seed"] + 1000 * rank
        lo, hi, S_tot = 0, S, S * world
    else:
        seed = cfg["seed"]
        lo, hi = shard_bounds(S, world, rank)
        S_tot = S
    if K:
        inp, modes = workloads.mode_states(S if scaling == "strong" else S, seed)
    else:
        inp, modes = getattr(workloads, cfg["gen"])(S, seed=seed), None
    if scaling == "strong":
        inp = {k: np.ascontiguousarray(v[lo:hi]) for k, v in inp.items()}
    S_rank = hi - lo
    return S_rank * (K or 1), S_rank, inp, modes, S_tot * (K or 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="stance_cold_b4096", choices=sorted(CONFIGS) + ["trot_stateful_b4096"],
                    help="trot_stateful_b4096 (configs[2]) runs only the stateful trot sequence, as --extra times "
                         "it (for tools/pmc.sh)")
    ap.add_argument("--scaling", choices=("weak", "strong"), default=None,
                    help="weak: the config's batch per GPU; strong: the config's batch in total, sharded "
                         "(default: the config's own)")
    ap.add_argument("--batch", type=int, default=0, help="override the config's batch")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--extra", action="store_true", help="also time the other configs (reported under 'extra')")
    ap.add_argument("--breakdown", action="store_true", help="also time the update and solve kernels separately")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}")
        sys.exit(2)

    import torch

    # WBC_DIST_BACKEND=gloo rehearses the N-rank path on a box with fewer GPUs (ranks share
    # devices, the gather goes through the host); the measured path is nccl (= RCCL over xGMI)
    backend = os.environ.get("WBC_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local_rank %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist

        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group(backend)

    from quadrupedwholebodycontroller_amd import FUSED, NO_X, SPLIT, STATELESS, Engine

    if args.config == "trot_stateful_b4096":  # configs[2] alone: one JSON line of the trot's record
        if world > 1:
            log("bench.py: trot_stateful_b4096 runs on one GPU")
            sys.exit(2)
        stream = torch.cuda.Stream()
        torch.cuda.set_stream(stream)
        r = bench_trot(torch, stream, local_rank, STATELESS)
        print(json.dumps(dict(metric="WBC QP solves/sec, configs[2] trot (stateful)", value=r["solves_per_s"],
                              unit="solves/s", n_gpus=1, config={"workload": args.config}, trot=r)), flush=True)
        return
    from quadrupedwholebodycontroller_amd.sharding import StepPipeline, shard_capacity

    STEP_FLAGS = STATELESS | NO_X  # cold solves; outputs tau, grf, status, iters (the published ones)

    cfg = dict(CONFIGS[args.config])
    if args.batch:
        cfg["batch"] = args.batch
    scaling = args.scaling or cfg.get("scaling", "weak")
    K = cfg.get("modes", 0)
    B, S, inp, modes, B_total = shard_inputs(cfg, scaling, world, rank)

    # a dedicated (non-null) stream: the engine launches on it and the HIP events below time it (the
    # legacy null stream would be handle 0 = "engine default"); the all-gather runs on `comm`
    stream = torch.cuda.Stream()
    comm = torch.cuda.Stream() if world > 1 else None
    torch.cuda.set_stream(stream)
    e = Engine(B, device=local_rank)
    e.set_stream(stream)
    if K:
        e.set_modes(modes)
    e.set_state(inp["base_pose"], inp["nu"], inp["qj"])
    e.set_reference(inp["ref"], inp["contacts"], inp["switching"])
    step = e.step_modes if K else e.step

    # Step outputs go straight into packed blocks (tau | status | iters) that the step's one
    # collective gathers on `comm`, overlapped with the next step (sharding.StepPipeline, the class
    # tests/test_gpu_pipeline.py runs on two ranks).
    cap = shard_capacity(B_total // (K or 1), world) * (K or 1) if scaling == "strong" else B
    pipe = StepPipeline(e, step, STEP_FLAGS, world, cap, stream, comm)

    for k in range(args.warmup):
        pipe.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        pipe.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    # whole-batch outputs of the last timed step, as every rank holds them after the gather
    g_tau, g_status, g_iters = pipe.result(pipe.last_slot, (B * world if scaling == "weak" else B_total)
                                           if world > 1 else B, unit=K or 1)
    pipe.bind(0)

    # Kernel duration for the roofline: HIP events on the launch stream around K back-to-back
    # launches (this includes the few-us dispatch gap between launches, which rocprofv3's
    # per-dispatch average in profiles/ excludes).
    def timed(fn):
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for _ in range(args.steps):
            fn()
        ev1.record(stream)
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1) / args.steps

    # A step is one kernel (wbc_update_solve_kernel, or wbc_modes_kernel for mode hypotheses under
    # the mode loop: dynamics, the QP reduced to 12 variables and solved in the same wave, torques;
    # the rare unusable reduction solved there too by the general method): the step's time is that
    # kernel's.  It owns all of SURVEY 8(d)'s flops.
    step_ms = timed(lambda: step(STEP_FLAGS))
    out = e.outputs()
    iters = out["iters"].astype(np.int64)
    status = out["status"]
    dom, dom_ms = step_kernel(e), step_ms
    kernels = {dom: step_ms}
    flops_step = step_flops(S, iters)
    tf_dom = flops_step / (dom_ms * 1e-3) / 1e12
    bytes_step = S * BYTES_IN + B * BYTES_OUT
    hbm_gbs = bytes_step / (step_ms * 1e-3) / 1e9

    breakdown = None
    if args.breakdown and not K:  # the general method's forms of the same step, for comparison
        breakdown = dict(step_ms=step_ms, fused64_step_ms=timed(lambda: e.step(STEP_FLAGS | FUSED)),
                         split_step_ms=timed(lambda: e.step(STEP_FLAGS | SPLIT)))

    extra = {}
    if args.extra and rank == 0:
        extra["trot_stateful_b4096"] = bench_trot(torch, stream, local_rank, STATELESS)
        for name, c2 in CONFIGS.items():
            if name == args.config or c2.get("scaling") == "strong":
                continue
            B2 = c2["batch"]
            e2, step2, _ = make_engine(c2, B2, c2["seed"], local_rank, stream)
            for _ in range(args.warmup):
                step2(STEP_FLAGS)
            ms2 = timed(lambda: step2(STEP_FLAGS))
            o2 = e2.outputs()
            tr2, tr2_src = committed_traffic(name, B2)
            S2 = B2 // (c2.get("modes") or 1)
            extra[name] = dict(batch=B2, ms_per_step=ms2, solves_per_s=B2 / (ms2 * 1e-3),
                               status_counts=np.bincount(o2["status"], minlength=4).tolist(),
                               mean_iters=float(o2["iters"].mean()), desc=c2["desc"],
                               roofline=roofline_of(step_flops(S2, o2["iters"]), ms2, tr2.get("step"), tr2_src,
                                                    step_kernel(e2)),
                               traffic_per_step=tr2.get("step"), traffic_source=tr2_src,
                               algorithmic_bytes_per_step=float(S2 * BYTES_IN + B2 * BYTES_OUT))
            extra[name]["roofline"]["executed_fp64"] = executed_fp64(name, B2, step_kernel(e2), ms2)
            e2.close()

    traffic, traffic_src = committed_traffic(args.config, B)
    pmc_rec, _ = committed_pmc(args.config, B)
    total = (B * world if scaling == "weak" else B_total) * args.steps
    value = total / elapsed
    result = {
        "metric": "WBC QP solves/sec (ANYmal 18-DoF, 4-contact) at 1/2/4/8 GPUs; % HBM roofline",
        "value": value,
        "unit": "solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (SURVEY.md 8d generators, numpy PCG64 seed %d%s)"
                % (cfg["seed"], " + 1000*rank" if scaling == "weak" else ", global batch sharded by rank"),
        "config": {"workload": args.config, "description": cfg["desc"], "batch_per_gpu": B,
                   "global_batch": B * world if scaling == "weak" else B_total,
                   "parallelism": f"dp{world}" + (" (robot shards; RCCL all-gather of tau|status|iters per step, "
                                                  "overlapped with the next step)" if world > 1 else "")},
        "roofline": {"bound": "fp64_valu", "achieved": tf_dom, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": tf_dom / FP64_PEAK_TFLOPS, "traffic": traffic.get(dom),
                     "traffic_source": traffic_src, "kernel": dom, "kernel_ms": dom_ms,
                     "kernels_ms": kernels, "step_kernels_ms": step_ms,
                     "instance": kernel_instance(e, args.config),
                     "note": f"the step's one kernel ({dom}; its kernel_ms is the step's, HIP events "
                             "around back-to-back launches); fp64 VALU roof (no MFMA on this path; gfx950 fp64 "
                             "vector peak); SURVEY 8(d) algorithmic flops: F_dyn + F_asm per state, F_fact + F_tau + "
                             "k F_iter per QP, k = iters[] (working-set changes of the 12-variable form the engine "
                             "solves); latency/issue-bound small dense linear algebra",
                     "flops_per_launch": flops_step,
                     "traffic_calibration": (pmc_rec or {}).get("calibration"),
                     "traffic_split": (pmc_rec or {}).get("traffic_split"),
                     "executed_fp64": executed_fp64(args.config, B, dom, dom_ms)},
        "roofline_hbm": {"bound": "hbm", "achieved": hbm_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": hbm_gbs / HBM_PEAK_GBS, "bytes_per_solve": bytes_step / B,
                         "traffic": sum(traffic.get(k, 0) for k in kernels) if traffic else None,
                         "note": "algorithmic bytes over the step (all its kernels): 729 B read per state + 200 B "
                                 "written per QP (929 B/solve one QP per state); traffic = PMC bytes per step "
                                 "(all its kernels, incl. any problem hand-off between them)"},
        "qp_status_counts": np.bincount(status, minlength=4).tolist(),
        "mean_iters": float(iters.mean()),
        "gathered": {"robots": int(len(g_status)), "status_counts": np.bincount(g_status, minlength=4).tolist(),
                     "mean_iters": float(np.mean(g_iters)), "tau_abs_sum": float(np.abs(g_tau).sum())},
    }
    if extra:
        result["extra"] = extra
    if breakdown:
        result["breakdown"] = breakdown
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(inp, args.cpu_budget)
        import multiprocessing

        result["cpu_baseline"]["host"] = dict(nproc=multiprocessing.cpu_count(), model=_cpu_model())
    elif world > 1:
        result["cpu_baseline_note"] = "timed at N=1 only (rank 0), per the bench contract"
    e.close()
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
