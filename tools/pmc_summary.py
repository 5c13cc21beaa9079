"""Summarise the rocprofv3 PMC passes of tools/pmc.sh for one kernel into a JSON record.

Usage: python tools/pmc_summary.py <pmc_dir> <out.json> [kernel_substring] [workload] [batch]

Per-launch means over every dispatch of the kernel in the passes.  HBM traffic follows
/opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE and WRITE_SIZE are
in KiB; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads, so the read side is
doubled; WRITE_SIZE is taken as is.  Other access widths are uncalibrated (the guide says so),
which this record states next to the number.
"""
import collections
import csv
import glob
import json
import os
import sys


def kernel_source_hash():
    """Hash of the HIP source the counters were taken on (bench.py only uses a matching record)."""
    import hashlib

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    h = hashlib.sha256()
    csrc = os.path.join(root, "quadrupedwholebodycontroller_amd", "csrc")
    # the code, not its comments: a comment edit leaves the counters valid
    import re

    units = sorted(f for f in os.listdir(csrc) if f.startswith("wbc_kernel_") and f.endswith(".hip"))
    for f in ["wbc_kernel.hip"] + units + ["wbc_layout.h"]:
        text = open(os.path.join(csrc, f)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        text = "\n".join(l.rstrip() for l in text.split("\n") if l.strip())
        h.update(text.encode())
    # the kernels' own compile flags (the one-kernel units' schedulers among them)
    for line in open(os.path.join(csrc, "Makefile")):
        if line.startswith("KFLAGS :=") or (line.split(" ", 1)[0].endswith("_KFLAGS") and ":=" in line):
            h.update(line.encode())
    return h.hexdigest()


def summarise(pmc_dir, prefix="wbc::wbc_"):
    """Per-kernel mean of every counter over its dispatches (kernels whose name starts with prefix)."""
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(pmc_dir, "pass*_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if name.startswith("void "):  # a template instance: "void wbc::wbc_update_solve_kernel<0>(...)"
                name = name[len("void "):]
            if name.startswith(prefix):
                short = name[len("wbc::"):].split("(")[0].split("<")[0]  # instances of one kernel share a name
                vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()}, \
           {k: {c: len(v) for c, v in d.items()} for k, d in vals.items()}


def traffic_bytes(mean, read_factor=2.0, write_factor=1.0):
    """HBM bytes per launch: FETCH_SIZE x read_factor + WRITE_SIZE x write_factor, KiB -> bytes.
    The defaults are the guide's figures for 16 B/lane streams (FETCH_SIZE counts half); the step's
    own patterns have measured factors (calibration below)."""
    if "FETCH_SIZE" not in mean or "WRITE_SIZE" not in mean:
        return None
    return read_factor * mean["FETCH_SIZE"] * 1024.0 + write_factor * mean["WRITE_SIZE"] * 1024.0


# the calibration kernel (tools/micro/calib.hip) that reproduces each bench workload's access pattern
CALIB_PATTERN = {"stance_cold": "calib_rows_stance", "rl_random": "calib_rows_rl", "modes16": "calib_rows_modes",
                 "trot": "calib_rows_stance"}


def calibration(workload):
    """(read_factor, write_factor, source) measured on the workload's access pattern by the newest
    committed calibration record (profiles/*/calib/calib_summary.json, tools/calib.sh), or None."""
    import glob

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    pat = next((v for k, v in CALIB_PATTERN.items() if workload.startswith(k)), None)
    for f in sorted(glob.glob(os.path.join(root, "profiles", "*", "calib", "calib_summary.json")), reverse=True):
        k = json.load(open(f))["kernels"].get(pat or "", {})
        if "read_factor" in k and "write_factor" in k:
            return k["read_factor"], k["write_factor"], os.path.relpath(f, root) + ":" + pat
    return None


# the step kernel instance each bench workload launches (its code is what the L2s fetch)
STEP_INSTANCE = {"stance_cold": r"wbc_update_solve_kernelILi0ELb1E", "rl_random": r"wbc_update_solve_kernelILi0ELb0E",
                 "trot": r"wbc_update_solve_kernelILi1ELb0E", "modes16": r"wbc_modes_kernel"}


def code_calibration():
    """(code_factor, source): how FETCH_SIZE counts instruction fetch, from the newest calibration
    record with a calib_code entry (tools/micro/calib.hip), or None."""
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for f in sorted(glob.glob(os.path.join(root, "profiles", "*", "calib", "calib_summary.json")), reverse=True):
        k = json.load(open(f))["kernels"].get("calib_code", {})
        if "code_factor" in k:
            return k["code_factor"], os.path.relpath(f, root) + ":calib_code"
    return None


def step_code_bytes(workload, lib=None):
    """HBM bytes of instruction fetch per launch of the workload's step kernel: 8 XCD L2s x its code
    size in the engine library (tools/code_size.py), or None."""
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from code_size import XCDS, code_size

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = lib or os.path.join(root, "quadrupedwholebodycontroller_amd", "libwbc_hip.so")
    pat = next((v for k, v in STEP_INSTANCE.items() if workload.startswith(k)), None)
    if not pat or not os.path.exists(lib):
        return None
    cs = code_size(lib, pat)
    return XCDS * cs if cs else None


def main():
    pmc_dir, out = sys.argv[1], sys.argv[2]
    workload = sys.argv[3] if len(sys.argv) > 3 else "stance_cold_b4096"
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
    step_kernels = (sys.argv[5] if len(sys.argv) > 5 else "wbc_step_kernel").split(",")
    mean, n = summarise(pmc_dir)
    rec = {"workload": workload, "batch": batch, "dispatches": n, "per_launch": mean,
           "kernel_source_sha256": kernel_source_hash()}
    cal = calibration(workload)
    rf, wf = (cal[0], cal[1]) if cal else (2.0, 1.0)
    rec["calibration"] = ({"read_factor": rf, "write_factor": wf, "source": cal[2]} if cal else None)
    rec["traffic_note"] = (("HBM bytes per launch = FETCH_SIZE x %.3f + WRITE_SIZE x %.3f, KiB -> B: factors measured "
                            "on this workload's own access pattern (%s); separate --pmc passes with --kernel-trace "
                            "only" % (rf, wf, cal[2])) if cal else
                           ("HBM bytes per launch = FETCH_SIZE x 2 (gfx950: half of wide coalesced reads counted) "
                            "+ WRITE_SIZE, KiB -> B; separate --pmc passes with --kernel-trace only; widths other "
                            "than 16 B/lane are uncalibrated (MI355X_MICROARCH.md)"))
    traffic = {k: traffic_bytes(m, rf, wf) for k, m in mean.items()}
    rec["traffic_uncalibrated"] = {k: traffic_bytes(m) for k, m in mean.items()}
    # executed fp64 VALU lane-operations per launch (an FMA counts 2), when the F64 counters ran
    for k, m in mean.items():
        if all(c in m for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64")):
            rec.setdefault("fp64_executed_flops", {})[k] = 64.0 * (m["SQ_INSTS_VALU_ADD_F64"] + m["SQ_INSTS_VALU_MUL_F64"] +
                                                                  2.0 * m["SQ_INSTS_VALU_FMA_F64"] +
                                                                  m.get("SQ_INSTS_VALU_TRANS_F64", 0.0))
    # the step's kernels that ran (the default step runs one of them: wbc_update_solve_kernel, or
    # wbc_modes_kernel for mode hypotheses under the mode loop)
    ran = [k for k in step_kernels if traffic.get(k) is not None]
    # instruction fetch: FETCH_SIZE also counts the step kernel's code, fetched from
    # HBM once per XCD and counted with its own factor (calib_code), not the data pattern's; split it
    # off so the data bytes are scaled by the data factor only, and add the code bytes back as is
    cc, code = code_calibration(), step_code_bytes(workload)
    if cal and cc and code and len(ran) == 1 and "FETCH_SIZE" in mean[ran[0]]:
        m = mean[ran[0]]
        code_counted = code / cc[0]
        data = rf * (m["FETCH_SIZE"] * 1024.0 - code_counted) + wf * m["WRITE_SIZE"] * 1024.0
        traffic[ran[0]] = data + code
        rec["traffic_split"] = {"data": data, "code_fetch": code, "code_factor": cc[0], "code_source": cc[1],
                                "note": "code_fetch = 8 XCD L2s x the step kernel's code size (tools/code_size.py); "
                                        "data = (FETCH_SIZE - code_fetch / code_factor) x read_factor + "
                                        "WRITE_SIZE x write_factor"}
    if ran:
        traffic["step"] = sum(traffic[k] for k in ran)
    rec["traffic"] = traffic
    rec["per_wave"] = {k: {c: v / m["SQ_WAVES"] for c, v in m.items() if c.startswith("SQ_INSTS")}
                       for k, m in mean.items() if m.get("SQ_WAVES")}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
