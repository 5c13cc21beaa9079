"""CPU: the gfx950 kernels compile scratch-free at the shipped occupancy (a spill or a dynamically
indexed private array turns into per-lane scratch traffic through L2/HBM: PMC WRITE_SIZE went from
1.0 to 7.4 MB per launch for one 6-vector).  The one exception is the elimination
fallback kernel, the rare path (near-singular legs) whose loop over an unknown-length list keeps
the kernel arguments live through the solve."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "quadrupedwholebodycontroller_amd", "csrc")


def test_step_kernels_scratch_free():
    """Every kernel's own code is free of scratch (spill) instructions.  Exceptions, the rare paths:
    the fallback kernel (its list loop keeps the arguments live through the solve) and
    drain_fallbacks, the call in which the default step's wave (and the mode loop's,
    wbc_modes_kernel, and the resident control cycle's, wbc_resident_kernel) solves its own
    fallbacks (only the callee touches the stack; the kernel body stays scratch-free).  The
    resident kernel's loop keeps its state in LDS and re-derives the arguments every cycle: held in
    registers across the step body they were spilled (309 scratch instructions)."""
    mk = open(os.path.join(CSRC, "Makefile")).read()
    waves = re.search(r"^WAVES \?= (\d+)", mk, re.M).group(1)
    kflags = re.search(r"^KFLAGS := (.*)$", mk, re.M).group(1).split()  # the kernel's own flags
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "include"),
                        "-I", CSRC, f"-DWBC_WAVES_PER_SIMD={waves}", *kflags, "-S", "--offload-device-only",
                        os.path.join(CSRC, "wbc_kernel.hip"), "-o", "-"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.split("\n")
    starts = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\w+:", l)]
    ends = [i for i, l in enumerate(lines) if l.startswith(".Lfunc_end")]
    names = []
    for i, n in starts:
        e = min(x for x in ends if x > i)
        body = lines[i:e]
        names.append(n)
        if "fallback" in n:
            continue
        spill = [l for l in body if "scratch_" in l]
        assert not spill, (n, spill[:3])
        calls = [l for l in body if "s_swappc" in l]
        assert not calls or "update_solve" in n or "modes_kernel" in n or "resident_kernel" in n, (n, calls)
    assert any("solve_stance" in n for n in names)
    # the default step's instances, the mode loop and the resident cycle live in their own units (the
    # test below); this one holds the split and one-robot-per-wave forms, the map and reset kernels
    assert not any(k in n for n in names for k in ("update_solve_kernel", "modes_kernel", "resident_kernel")), names
    assert any("wbc_update_kernel" in n for n in names) and any("step_kernel" in n for n in names), names


UNITS = {  # one-kernel translation unit -> (its Makefile flags variable, its kernels' mangled names)
    "stance": ("STANCE_KFLAGS", ["wbc_update_solve_kernelILi0ELb1E"]),
    "step0": ("STEP0_KFLAGS", ["wbc_update_solve_kernelILi0ELb0E"]),
    "step1": ("STEP1_KFLAGS", ["wbc_update_solve_kernelILi1ELb0E"]),
    "modes": ("MODES_KFLAGS", ["wbc_modes_kernel"]),
    "resident": ("RESIDENT_KFLAGS", ["wbc_resident_kernelILi0E", "wbc_resident_kernelILi1E"]),
}


@pytest.mark.parametrize("unit", sorted(UNITS))
def test_one_kernel_units_scratch_free(unit):
    """The one-kernel units (wbc_kernel_<unit>.hip, each under its own Makefile flags, DESIGN.md
    4.22 / 4.24) compile scratch-free too, and each holds only its kernel (the resident unit: the
    two instances of its kernel) and the fallback call of each."""
    var, knames = UNITS[unit]
    mk = open(os.path.join(CSRC, "Makefile")).read()
    waves = re.search(r"^WAVES \?= (\d+)", mk, re.M).group(1)
    kflags = re.search(r"^KFLAGS := (.*)$", mk, re.M).group(1).split()
    sflags = re.search(rf"^{var} := (.*)$", mk, re.M).group(1).split()
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "include"),
                        "-I", CSRC, f"-DWBC_WAVES_PER_SIMD={waves}", *kflags, *sflags, "-S", "--offload-device-only",
                        os.path.join(CSRC, f"wbc_kernel_{unit}.hip"), "-o", "-"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.split("\n")
    starts = [(i, l.split(":")[0]) for i, l in enumerate(lines) if re.match(r"^_Z\w+:", l)]
    ends = [i for i, l in enumerate(lines) if l.startswith(".Lfunc_end")]
    names = [n for _, n in starts]
    kernels = [n for n in names if "drain_fallbacks" not in n]
    assert len(kernels) == len(knames) and all(any(k in n for n in kernels) for k in knames), names
    assert len(names) == 2 * len(knames), names  # one fallback callee per kernel
    for i, n in starts:
        if "drain_fallbacks" in n:
            continue
        body = lines[i:min(x for x in ends if x > i)]
        assert not [l for l in body if "scratch_" in l], n
