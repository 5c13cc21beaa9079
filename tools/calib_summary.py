"""Factors that turn rocprofv3 FETCH_SIZE / WRITE_SIZE into HBM bytes for the step kernel's access
patterns (tools/micro/calib.hip, run by tools/calib.sh).

For every calibration kernel: the mean FETCH_SIZE / WRITE_SIZE per launch (KiB -> B) against the bytes
it is known to move; read_factor = known read / FETCH bytes (2.0 is the guide's figure for 16 B/lane
streams), write_factor = known write / WRITE bytes.  calib_image gives what the per-workgroup model
image staging adds to the counters (bytes per launch of 1024 workgroups); calib_code gives
code_factor = (8 XCDs x its code size) / FETCH bytes, the counting of instruction fetch.

Usage: python tools/calib_summary.py <dir with known.json and pass*_counter_collection.csv>"""
import collections
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    known = json.load(open(os.path.join(d, "known.json")))
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, "pass*_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("::")[-1]
            if name.startswith("calib_"):
                vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, --kernel-trace), mean per launch over "
                     f"{known['launches']} launches; KiB -> B", "kernels": {}}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) * 1024.0 for c, v in cs.items()}
        kn = known.get(k, {})
        rec = {"fetch_bytes": m.get("FETCH_SIZE"), "write_bytes": m.get("WRITE_SIZE"), "known": kn}
        if kn.get("read") and m.get("FETCH_SIZE"):
            rec["read_factor"] = kn["read"] / m["FETCH_SIZE"]
        if kn.get("write") and m.get("WRITE_SIZE"):
            rec["write_factor"] = kn["write"] / m["WRITE_SIZE"]
        if "read_per_workgroup" in kn and m.get("FETCH_SIZE"):
            rec["image_fetch_bytes_per_launch"] = m["FETCH_SIZE"]
        if k == "calib_code" and m.get("FETCH_SIZE"):
            # instruction fetch: 8 XCD L2s each miss the kernel's code once (tools/code_size.py)
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            from code_size import XCDS, code_size

            cs = code_size(os.path.join(os.path.dirname(os.path.abspath(__file__)), "micro", "calib"), "calib_code")
            if cs:
                rec["known"] = dict(kn, code_bytes=cs, read=XCDS * cs)
                rec["code_factor"] = XCDS * cs / m["FETCH_SIZE"]
        out["kernels"][k] = rec
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
