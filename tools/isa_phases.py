"""Static instruction mix of wbc_solve_kernel per solve phase (source-line ranges of solve_phase).

Usage: python tools/isa_phases.py <kernel.s built with -gline-tables-only> [start:name ...]
Instructions of inlined helpers are charged to the phase of the last solve_phase line seen.
"""
import collections
import re
import sys

DEFAULT = [(1260, "setup"), (1371, "normals"), (1420, "eq"), (1607, "warm"), (1636, "loop"), (1789, "recovery"),
           (1824, "outputs"), (1946, "kernel")]


def main():
    path = sys.argv[1]
    bounds = [(int(a.split(":")[0]), a.split(":")[1]) for a in sys.argv[2:]] or DEFAULT
    lo, hi = bounds[0][0], bounds[-1][0] + 20
    s = open(path).read().split("\n")
    st = [i for i, l in enumerate(s) if l.startswith("_ZN3wbc16wbc_solve_kernel")][0]
    files = {}
    for l in s:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[m.group(1)] = (m.group(3) or m.group(2)).split("/")[-1]

    def phase(ln):
        p = "pre"
        for b, n in bounds:
            if ln >= b:
                p = n
        return p

    cur = "pre"
    c = collections.defaultdict(collections.Counter)
    for l in s[st + 1:]:
        t = l.strip()
        if t.startswith("s_endpgm"):
            break
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if m:
            ln = int(m.group(2))
            if files.get(m.group(1)) == "wbc_kernel.hip" and lo <= ln <= hi:
                cur = phase(ln)
            continue
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        op = t.split()[0]
        k = "valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") else "other"
        c[cur][k] += 1
        for tag, pred in (("readlane", op.startswith("v_readlane")), ("dpp", "dpp" in op),
                          ("cndmask", op.startswith("v_cndmask")), ("f64", "f64" in op)):
            if pred:
                c[cur][tag] += 1
    for p, v in c.items():
        print(f"{p:10s}", dict(v))


if __name__ == "__main__":
    main()
