"""Static instruction counts of the active-set loops of wbc_update_solve_kernel<0> (the stateless
default step, wbc_kernel_step0.hip), per basic block, from the `make listing` output (hipcc -S
-gline-tables-only; the stance-only step: build/wbc_kernel_stance.s with --sym of its instance).

A loop is the set of blocks the listing marks "in Loop: Header=BB..": the stance form's and the
general form's loops.  For each, prints every block (instructions, VALU / DPP / LDS / SALU / waits /
nops / branches, the wbc_kernel.hip source lines it came from) and the totals of the blocks outside
the Givens drop path (source lines of the drop branch), i.e. the static length of an add pass.

Usage: python tools/isa_loop.py [listing.s] [--sym NAME] [--quiet]"""
import collections
import re
import sys

SYM = "_ZN3wbc23wbc_update_solve_kernelILi0ELb0EEEvNS_10KernelArgsE"


def drop_lines(src):
    """Source lines of solve16's drop branch (from the `// drop slot l1` comment to the mirror call)."""
    lines = src.split("\n")
    sv = next(i for i, l in enumerate(lines) if re.match(r"^__device__ void solve16\(", l))
    a = next(i for i in range(sv, len(lines)) if "drop slot l1" in lines[i]) + 1
    b = next(i for i in range(a, len(lines)) if re.match(r"\s*mirror\(\);", lines[i])) + 1
    return a, b


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    path = args[0] if args else "quadrupedwholebodycontroller_amd/csrc/build/wbc_kernel_step0.s"
    sym = SYM
    if "--sym" in sys.argv:
        sym = sys.argv[sys.argv.index("--sym") + 1]
    quiet = "--quiet" in sys.argv
    src = open("quadrupedwholebodycontroller_amd/csrc/wbc_kernel.hip").read()
    d0, d1 = drop_lines(src)
    lines = open(path).read().split("\n")
    st = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    en = next(i for i in range(st, len(lines)) if lines[i].startswith(".Lfunc_end"))
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[int(m.group(1))] = m.group(3) or m.group(2)
    blocks, blk, cur, curf = [], None, 0, ""
    for l in lines[st:en]:
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            curf, cur = files.get(int(m.group(1)), ""), int(m.group(2))
            continue
        s = l.strip()
        if (s.startswith(".LBB") and s.endswith(":")) or (s.startswith(".LBB") and ":" in s) or s.startswith("; %bb."):
            hdr = re.search(r"Header=(BB\d+_\d+)", s)
            me = re.search(r"(BB\d+_\d+)", s.replace("%bb.", "BB_"))
            blk = dict(name=s.split()[0] if not s.startswith(";") else s[2:].split()[0], loop=hdr.group(1) if hdr else None,
                       c=collections.Counter(), src=set(), n=0)
            if "=>This Inner Loop Header" in s:
                blk["loop"] = "BB" + s.split(":")[0][4:]
            blocks.append(blk)
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        if blk is None:
            continue
        op = s.split()[0]
        blk["n"] += 1
        if curf.endswith("wbc_kernel.hip") and cur > 700:
            blk["src"].add(cur)
        c = blk["c"]
        if "_dpp" in op or "row_" in s or "quad_perm" in s:
            c["dpp"] += 1
        elif op.startswith("v_") and "accvgpr" not in op:
            c["valu"] += 1
        if "accvgpr" in op:
            c["agpr"] += 1
        if op.startswith("s_nop"):
            c["nop"] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
        elif op.startswith("s_waitcnt"):
            c["wait"] += 1
        elif "branch" in op:
            c["branch"] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
    loops = collections.OrderedDict()
    for b in blocks:
        if b["loop"]:
            loops.setdefault(b["loop"], []).append(b)
    for name, bl in loops.items():
        tot, add = collections.Counter(), collections.Counter()
        for b in bl:
            tot.update(b["c"])
            tot["instr"] += b["n"]
            indrop = bool(b["src"]) and all(d0 <= x <= d1 for x in b["src"])
            if not indrop:
                add.update(b["c"])
                add["instr"] += b["n"]
            if not quiet:
                rng = (min(b["src"]), max(b["src"])) if b["src"] else None
                print(f"  {b['name']:14s} {b['n']:4d} {dict(b['c'])} src {rng}{'  [drop]' if indrop else ''}")
        print(f"loop {name}: {len(bl)} blocks, all {dict(tot)}")
        print(f"loop {name}: outside the drop path {dict(add)}")


if __name__ == "__main__":
    main()
