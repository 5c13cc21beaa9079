"""Static instruction mix of wbc_update_solve_kernel per stage of the step (the stage stamps of the
WBC_ISTAMPS build, tools/ust16.py), from a `hipcc -S -gline-tables-only` listing.  An instruction is
charged to the stage of the last wbc_kernel.hip source line seen inside a stage range, so the
instructions of inlined helpers (cross3, mv3, fast_rsq ...) go to the stage that called them.
Dividing a stage's measured ticks (ust16.py) by its VALU count separates issue-bound stages (~7 ticks
per VALU instruction at one wave per SIMD) from latency-bound ones.

Usage: python tools/isa_stages.py listing.s  (make -C quadrupedwholebodycontroller_amd/csrc listing)"""
import collections
import re
import sys

SYM = "_ZN3wbc23wbc_update_solve_kernelILi0EEEvNS_10KernelArgsE"  # the stateless instance


def stage_ranges(src):
    """Stage -> (first, last) source line, found from the stamp comments of wbc_kernel.hip."""
    lines = src.split("\n")

    def find(pat, start=0):
        for i in range(start, len(lines)):
            if re.search(pat, lines[i]):
                return i + 1
        raise KeyError(pat)

    up = find(r"^__device__ bool update_phase\(")
    u = [find(r"UST\(a, rb, %d\);" % k, up) for k in range(11)]
    sr = find(r"^__device__ bool stance_reduce\(")
    s19, s20, s12 = find(r"UST\(ka, rb, 19\)", sr), find(r"UST\(ka, rb, 20\)", sr), find(r"UST\(ka, rb, 12\)", sr)
    s21, s22, s13 = find(r"UST\(ka, rb, 21\)", sr), find(r"UST\(ka, rb, 22\)", sr), find(r"UST\(ka, rb, 13\)", sr)
    s14 = find(r"UST\(ka, rb, 14\)", sr)
    r6 = find(r"^__device__ (__forceinline__ )?bool rank6_factor\(")
    rg = find(r"^__device__ bool reduce_general\(")
    g20, g21, g22 = find(r"UST\(ka, rb, 20\)", rg), find(r"UST\(ka, rb, 21\)", rg), find(r"UST\(ka, rb, 22\)", rg)
    g14 = find(r"UST\(ka, rb, 14\)", rg)
    sv = find(r"^__device__ void solve16\(")
    s15, s16, s18 = find(r"UST\(a, rb, 15\)", sv), find(r"UST\(a, rb, 16\)", sv), find(r"UST\(a, rb, 18\)", sv)
    kern = find(r"void wbc_update_solve_kernel\(KernelArgs a\)")
    names = ["inputs+sincos", "stage A", "stage B", "Jf + CoM", "Ic", "stage C", "hb, y, zeta", "Jbar/Mbar/bbar",
             "Tdot_inv", "bounds, wrench, history"]
    r = collections.OrderedDict()
    r["prologue (kernel)"] = (kern, kern + 60)
    r["update entry"] = (up, u[0])
    for k, n in enumerate(names):
        r[n] = (u[k], u[k + 1])
    r["debug + form choice"] = (u[10], u[10] + 160)
    r["stance: legs, W"] = (sr, s19)
    r["stance: S"] = (s19, s20)
    r["stance: S^-1"] = (s20, s12)
    r["stance: Y, q0"] = (s12, s21)
    r["stance: Q"] = (s21, s22)
    r["stance: H^, g_f"] = (s22, s13)
    r["stance: Nt, t0"] = (s13, s14)
    r["stance: rank-6 factor"] = (r6, rg - 1)
    r["general: R1-R4"] = (rg, g20)
    r["general: R5"] = (g20, g21)
    r["general: R6"] = (g21, g22)
    r["general: R7-R8"] = (g22, g14)
    r["solve setup"] = (sv, s15)
    r["active-set loop"] = (s15, s16)
    r["outputs"] = (s16, s18)
    return r


def main():
    path = sys.argv[1]
    src_path = sys.argv[2] if len(sys.argv) > 2 else "quadrupedwholebodycontroller_amd/csrc/wbc_kernel.hip"
    ranges = stage_ranges(open(src_path).read())
    lines = open(path).read().split("\n")
    st = [i for i, l in enumerate(lines) if l.startswith(SYM + ":")][0]
    en = [i for i, l in enumerate(lines[st:]) if l.startswith(".Lfunc_end")][0] + st
    files = {}
    for l in lines:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', l)
        if m:
            files[int(m.group(1))] = m.group(3) or m.group(2)
    cur = "?"
    acc = collections.defaultdict(collections.Counter)
    for l in lines[st:en]:
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            f, ln = int(m.group(1)), int(m.group(2))
            if "wbc_kernel" in files.get(f, ""):
                for n, (a, b) in ranges.items():
                    if a <= ln < b:
                        cur = n
                        break
            continue
        t = l.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        c = acc[cur]
        c["instr"] += 1
        if t.startswith("v_"):
            c["valu"] += 1
        if t.startswith("v_accvgpr"):
            c["agpr_mov"] += 1
        if t.startswith("ds_"):
            c["lds"] += 1
        if t.startswith("s_waitcnt"):
            c["waitcnt"] += 1
        if "dpp" in t or "row_" in t or "quad_perm" in t:
            c["dpp"] += 1
        if t.startswith("s_nop"):
            c["s_nop"] += 1
        if t.startswith(("global_", "buffer_", "flat_", "scratch_")):
            c["vmem"] += 1
    order = list(ranges) + ["?"]
    for n in order:
        if n in acc:
            print("%-28s %s" % (n, dict(acc[n])))


if __name__ == "__main__":
    main()
