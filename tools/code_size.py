"""Code sizes of the gfx950 kernels in an ELF (a HIP shared library or executable): the offload
bundles are extracted with llvm-objdump --offloading into a scratch directory and the kernels' symbol
sizes read with llvm-readelf.  Instruction fetch is real HBM traffic: each XCD's L2 misses a
kernel's code once per launch (measured by tools/micro/calib.hip calib_code).

Usage: python tools/code_size.py <elf> [name_substring]"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
XCDS = 8  # MI355X: 8 XCDs, each with its own L2


def kernel_code_sizes(elf):
    """{mangled symbol: code bytes} over every gfx950 code object in `elf`."""
    sizes = {}
    with tempfile.TemporaryDirectory() as d:
        local = os.path.join(d, os.path.basename(elf))
        shutil.copy(elf, local)
        subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", local], cwd=d, capture_output=True,
                       check=False)
        for f in sorted(os.listdir(d)):
            if "gfx950" not in f:
                continue
            r = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-sW", os.path.join(d, f)], capture_output=True,
                               text=True, check=False)
            for line in r.stdout.splitlines():
                p = line.split()
                if len(p) >= 8 and p[3] == "FUNC" and p[2].isdigit():
                    sizes[p[7]] = max(sizes.get(p[7], 0), int(p[2]))
    return sizes


def code_size(elf, pattern):
    """Code bytes of the one kernel whose mangled name matches the regex `pattern` (None if none)."""
    hits = {k: v for k, v in kernel_code_sizes(elf).items() if re.search(pattern, k)}
    return max(hits.values()) if hits else None


if __name__ == "__main__":
    for k, v in sorted(kernel_code_sizes(sys.argv[1]).items(), key=lambda kv: kv[1]):
        if len(sys.argv) < 3 or sys.argv[2] in k:
            print(v, k)
