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


def summarise(pmc_dir, kernel="wbc_step_kernel"):
    vals = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(pmc_dir, "pass*_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    pmc_dir, out = sys.argv[1], sys.argv[2]
    kernel = sys.argv[3] if len(sys.argv) > 3 else "wbc_step_kernel"
    workload = sys.argv[4] if len(sys.argv) > 4 else "stance_cold_b4096"
    batch = int(sys.argv[5]) if len(sys.argv) > 5 else 4096
    mean, n = summarise(pmc_dir, kernel)
    rec = {"kernel": kernel, "workload": workload, "batch": batch, "dispatches": n, "per_launch": mean,
           "kernel_source_sha256": kernel_source_hash()}
    if "FETCH_SIZE" in mean and "WRITE_SIZE" in mean:
        rd = 2.0 * mean["FETCH_SIZE"] * 1024.0
        wr = mean["WRITE_SIZE"] * 1024.0
        rec["traffic_bytes_per_launch"] = rd + wr
        rec["traffic_read_bytes"] = rd
        rec["traffic_write_bytes"] = wr
        rec["traffic_note"] = ("HBM bytes per launch from FETCH_SIZE (x2, gfx950 correction) + WRITE_SIZE, KiB -> B; "
                               "separate --pmc passes with --kernel-trace only")
    if "SQ_WAVES" in mean:
        w = mean["SQ_WAVES"]
        rec["per_wave"] = {k: v / w for k, v in mean.items() if k.startswith("SQ_INSTS")}
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
