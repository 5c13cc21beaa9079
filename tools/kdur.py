"""Per-kernel dispatch durations (mean, count) by grid size from a rocprofv3 output: a rocpd
SQLite database (run_results.db, rocprofv3's default format here) or a *_kernel_trace.csv.
Usage: python tools/kdur.py <file> [name substring ...]"""
import collections
import csv
import sqlite3
import sys


def rows(path):
    if path.endswith(".db"):
        db = sqlite3.connect(path)
        for name, gx, dur in db.execute("select name, grid_x, duration from kernels"):
            yield name, int(gx), float(dur)
    else:
        for r in csv.DictReader(open(path)):
            yield r["Kernel_Name"], int(r.get("Grid_Size_X", r.get("Grid_Size", 0))), \
                float(r["End_Timestamp"]) - float(r["Start_Timestamp"])


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    d = collections.defaultdict(list)
    for name, gx, dur in rows(path):
        if not pats or any(p in name for p in pats):
            d[(name.split("(")[0].replace("void ", ""), gx)].append(dur / 1000.0)
    for (name, gx), v in sorted(d.items()):
        print(f"{name:45s} grid {gx:9d}  n {len(v):4d}  mean {sum(v) / len(v):9.2f} us  min {min(v):9.2f} us")


if __name__ == "__main__":
    main()
