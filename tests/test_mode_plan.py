"""CPU: the mode loop's plan (wbc_layout.h mode_loop_plan, wbc_set_modes), compiled for the host from
the engine's own header.  For K hypotheses over `groups` four-state groups on `simds` SIMDs
(DESIGN.md 4.14):

* M is the largest divisor of K with groups * K / M >= simds, else 1; an override that divides K
  replaces it, anything else is ignored;
* the order is a permutation of 0..K-1, cut into K / M chunks of M;
* chunks are filled longest first (LPT on 30 + 3 * passes(popcount)), so their estimated loads
  differ by at most one hypothesis' cost.

The kernel's results do not depend on the plan (tests/test_gpu_modes.py checks bit-identity for
every M); the plan only decides the grid and the balance."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "quadrupedwholebodycontroller_amd", "csrc")
PASSES = [0.3, 2.3, 4.5, 6.7, 8.9]

PROG = r"""
#include <cstdio>
#include "wbc_layout.h"
int main() {
    int K; long long groups, simds; int ov;
    while (std::scanf("%d %lld %lld %d", &K, &groups, &simds, &ov) == 4) {
        uint8_t modes[16], order[16];
        for (int k = 0; k < K; ++k) { int v; std::scanf("%d", &v); modes[k] = (uint8_t)v; }
        const int M = wbc::mode_loop_plan(modes, K, groups, simds, ov, order);
        std::printf("%d", M);
        for (int k = 0; k < K; ++k) std::printf(" %d", order[k]);
        std::printf("\n");
    }
}
"""


@pytest.fixture(scope="module")
def plan_bin(tmp_path_factory):
    d = tmp_path_factory.mktemp("plan")
    src = d / "p.cpp"
    src.write_text(PROG)
    exe = d / "p"
    subprocess.run(["g++", "-O1", "-Wno-unused-result", "-std=c++17", "-I", os.path.join(ROOT, "include"), "-I", CSRC,
                    str(src), "-o", str(exe)], check=True)
    return str(exe)


def run_plans(exe, cases):
    text = "".join(f"{len(m)} {g} {s} {ov} " + " ".join(str(int(v)) for v in m) + "\n" for m, g, s, ov in cases)
    out = subprocess.run([exe], input=text, capture_output=True, text=True, check=True).stdout.splitlines()
    return [(int(l.split()[0]), [int(t) for t in l.split()[1:]]) for l in out]


def expected_m(K, groups, simds, ov):
    if 1 <= ov <= K and K % ov == 0:
        return ov
    for m in range(K, 1, -1):
        if K % m == 0 and groups * (K // m) >= simds:
            return m
    return 1


def cost(mask):
    return 30.0 + 3.0 * PASSES[bin(mask & 15).count("1")]


def test_mode_loop_plan(plan_bin):
    g = np.random.default_rng(5)
    cases = [(list(range(16)), 256, 1024, 0),    # configs[4]'s shard on a 256-CU MI355X: M = 4
             (list(range(16)), 2048, 1024, 0),   # its global size on one GPU: M = 16
             (list(range(16)), 1024, 1024, 0),   # 4096 states per rank on 2 GPUs: M = 16
             (list(range(16)), 64, 1024, 0),     # few states: one hypothesis per segment
             (list(range(16)), 256, 1024, 2), (list(range(16)), 256, 1024, 3),  # override; 3 ignored
             ([15, 10, 5, 15, 0], 10, 1024, 5), ([15, 10, 5, 15, 0], 1000, 1024, 0),
             ([3, 3, 3, 3, 12, 12], 700, 1024, 0), ([7], 5, 1024, 0)]
    for _ in range(20):
        K = int(g.integers(1, 17))
        cases.append((g.integers(0, 16, K).tolist(), int(g.integers(1, 4096)), 1024, 0))
    for (modes, groups, simds, ov), (M, order) in zip(cases, run_plans(plan_bin, cases)):
        K = len(modes)
        assert M == expected_m(K, groups, simds, ov), (modes, groups, ov, M)
        assert sorted(order) == list(range(K)), "a permutation of the hypotheses"
        chunks = [order[c * M:(c + 1) * M] for c in range(K // M)]
        loads = [sum(cost(modes[k]) for k in ch) for ch in chunks]
        assert max(loads) - min(loads) <= max(cost(m) for m in modes) + 1e-9, (modes, M, loads)
    # configs[4]'s shard: four chunks of four, their estimated loads within one mask class apart
    (M, order), = run_plans(plan_bin, [(list(range(16)), 256, 1024, 0)])
    assert M == 4
    loads = [sum(cost(k) for k in order[4 * c:4 * c + 4]) for c in range(4)]
    assert max(loads) - min(loads) <= cost(15) - cost(7) + 1e-9, loads
