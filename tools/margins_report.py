"""The GPU suite's parity margins by bound (tests/margins.py), from a parity_margins.json that the
suite wrote (conftest.py): for every bound constant, the worst achieved value over the tests that
use it and the margin bound / worst; then the overall margin range.  Used to keep the "worst"
comments of tests/margins.py and the margin range quoted in README / DESIGN / BASELINE in step with
the evidence.

Usage: python tools/margins_report.py [profiles/r05/parity_margins.json]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import margins as M  # noqa: E402


def constant(test, q, bound):
    """The tests/margins.py constant a record's bound came from."""
    name = q.split(" ")[0]
    if "replays_golden" in test:
        return "REPLAY"
    if name in M.INTERMEDIATE and bound == M.INTERMEDIATE[name]:
        return "INTERMEDIATE[%s]" % (name if bound > 1e-14 else "few-ulps blocks")
    if bound == M.GOLD and name == "tau":
        return "GOLD"
    if bound == M.TAU and name == "tau":
        return "TAU"
    if bound == M.X and name == "x":
        return "X"
    if bound == M.GRF and name == "grf":
        return "GRF"
    if bound == M.BITS and name in ("tau", "x", "grf"):
        return "BITS"
    return "INTERMEDIATE[others]" if bound == 1e-13 else "bound %.0e" % bound


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r05", "parity_margins.json")
    d = json.load(open(path))
    by_const = {}
    for test, qs in d.items():
        for q, r in qs.items():
            if "mismatch" in q:
                continue
            key = constant(test, q, r["bound"])
            w = by_const.get(key)
            if w is None or r["achieved"] >= w[1]:
                by_const[key] = [r["bound"], r["achieved"], q, test.split("::")[-1][:60]]
    margins = []
    print(f"{'constant':28s} {'bound':>9} {'worst':>10} {'margin':>7}  quantity / test")
    for key, (bound, worst, q, test) in sorted(by_const.items()):
        m = bound / worst if worst > 0 else float("inf")
        if m != float("inf"):
            margins.append(m)
        print(f"{key:28s} {bound:9.1e} {worst:10.2e} {m:7.1f}  {q[:30]} / {test}")
    print(f"margin range over the bounds: {min(margins):.1f} - {max(margins):.0f} x")
    mism = [(t.split('::')[-1][:60], q, r["achieved"], r["bound"]) for t, qs in d.items() for q, r in qs.items()
            if "mismatch" in q and r["achieved"] > 0]
    print("non-zero mismatch fractions:", mism if mism else "none")


if __name__ == "__main__":
    main()
