"""CPU: the gfx950 kernels compile scratch-free at the shipped occupancy (a spill or a dynamically
indexed private array turns into per-lane scratch traffic through L2/HBM: PMC WRITE_SIZE went from
1.0 to 7.4 MB per launch for one 6-vector).  The one exception is the elimination
fallback kernel, the rare path (near-singular legs) whose loop over an unknown-length list keeps
the kernel arguments live through the solve."""
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "quadrupedwholebodycontroller_amd", "csrc")


def test_step_kernels_scratch_free():
    waves = re.search(r"^WAVES \?= (\d+)", open(os.path.join(CSRC, "Makefile")).read(), re.M).group(1)
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "include"),
                        "-I", CSRC, f"-DWBC_WAVES_PER_SIMD={waves}", "-c", os.path.join(CSRC, "wbc_kernel.hip"),
                        "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    names = re.findall(r"Function Name: (\S+)", r.stderr)
    scratch = [int(x) for x in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", r.stderr)]
    assert len(names) == len(scratch) >= 4
    for n, sc in zip(names, scratch):
        if "fallback" in n:
            continue
        assert sc == 0, (n, sc)
    assert any("solve_stance" in n for n in names)
