#!/bin/bash
# Per-kernel rocprofv3 stats for each (library, workload) pair: LIBS="new old" CONFIGS="..." bash tools/kprof.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/kprof_${TAG:-x}
mkdir -p $O
for lib in ${LIBS:-new}; do
  for c in ${CONFIGS:-stance_cold_b4096 rl_random_b8192 modes16_b16384}; do
    so=quadrupedwholebodycontroller_amd/libwbc_hip.so
    [ "$lib" != "new" ] && so=quadrupedwholebodycontroller_amd/libwbc_hip_$lib.so
    WBC_LIB=$(pwd)/$so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$lib.$c -o k --output-format csv -- python3 tools/kprof.py $c 20 > $O/$lib.$c.log 2>&1
    rc=$?
    echo "$lib $c rc=$rc" >> $O/runs.txt
    if [ $rc -ne 0 ]; then tail -5 $O/$lib.$c.log; exit $rc; fi
  done
done
python3 - "$O" <<'PY'
import csv, glob, os, sys
O = sys.argv[1]
for f in sorted(glob.glob(os.path.join(O, "*", "**", "*kernel_stats.csv"), recursive=True)):
    tag = os.path.relpath(f, O).split(os.sep)[0]
    for r in csv.DictReader(open(f)):
        if "wbc" in r["Name"]:
            print(f"{tag:40s} {r['Name'][:40]:40s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs'])/1e3:9.2f}")
PY
