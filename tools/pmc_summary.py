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
    for f in ("wbc_kernel.hip", "wbc_layout.h"):
        h.update(open(os.path.join(root, "quadrupedwholebodycontroller_amd", "csrc", f), "rb").read())
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


def traffic_bytes(mean):
    """HBM bytes per launch: FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE, KiB -> bytes."""
    if "FETCH_SIZE" not in mean or "WRITE_SIZE" not in mean:
        return None
    return 2.0 * mean["FETCH_SIZE"] * 1024.0 + mean["WRITE_SIZE"] * 1024.0


def main():
    pmc_dir, out = sys.argv[1], sys.argv[2]
    workload = sys.argv[3] if len(sys.argv) > 3 else "stance_cold_b4096"
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else 4096
    step_kernels = (sys.argv[5] if len(sys.argv) > 5 else "wbc_step_kernel").split(",")
    mean, n = summarise(pmc_dir)
    rec = {"workload": workload, "batch": batch, "dispatches": n, "per_launch": mean,
           "kernel_source_sha256": kernel_source_hash(),
           "traffic_note": ("HBM bytes per launch = FETCH_SIZE x 2 (gfx950: half of wide coalesced reads counted) "
                            "+ WRITE_SIZE, KiB -> B; separate --pmc passes with --kernel-trace only; widths other "
                            "than 16 B/lane are uncalibrated (MI355X_MICROARCH.md)")}
    traffic = {k: traffic_bytes(m) for k, m in mean.items()}
    # the step's kernels that ran (the default step runs one of them: wbc_update_solve_kernel, or
    # wbc_modes_kernel for mode hypotheses under the mode loop)
    ran = [k for k in step_kernels if traffic.get(k) is not None]
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
