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


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "profiles", "r05", "parity_margins.json")
    d = json.load(open(path))
    by_bound = {}
    for test, qs in d.items():
        for q, r in qs.items():
            if "mismatch" in q:
                continue
            key = (r["bound"], q.split(" ")[0])
            w = by_bound.setdefault(key, [0.0, None])
            if r["achieved"] >= w[0]:
                by_bound[key] = [r["achieved"], test.split("::")[-1][:60]]
    named = {}
    margins = []
    print(f"{'bound':>9} {'quantity':28s} {'worst':>10} {'margin':>9}  test")
    for (bound, q), (worst, test) in sorted(by_bound.items()):
        m = bound / worst if worst > 0 else float("inf")
        margins.append(m)
        print(f"{bound:9.1e} {q[:28]:28s} {worst:10.2e} {m:9.1f}  {test}")
    fin = [m for m in margins if m != float("inf")]
    print(f"margin range over the bounds: {min(fin):.1f} - {max(fin):.0f} x")
    mism = [(t.split('::')[-1][:60], q, r["achieved"], r["bound"]) for t, qs in d.items() for q, r in qs.items()
            if "mismatch" in q and r["achieved"] > 0]
    print("non-zero mismatch fractions:", mism if mism else "none")


if __name__ == "__main__":
    main()
