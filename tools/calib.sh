#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on the step kernel's access patterns (tools/micro/calib.hip):
# separate --pmc passes with --kernel-trace only (MI355X_MICROARCH.md), then tools/calib_summary.py.
# OUT=gpurun_out/calib bash tools/calib.sh   (the binary is built on the CPU side beforehand)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/calib}
mkdir -p $OUT
BIN=$PWD/tools/micro/calib
timeout -k 10 60 $BIN 20 > $OUT/known.json || { echo "calib run failed"; exit 1; }
i=0
for set in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT -o pass$i -- $BIN 20 > $OUT/pass$i.log 2>&1
  rc=$?
  echo "pass$i [$set] rc=$rc" >> $OUT/passes.txt
  if [ $rc -ne 0 ]; then echo "pmc pass $i failed rc=$rc"; tail -5 $OUT/pass$i.log; exit $rc; fi
done
python3 tools/calib_summary.py $OUT > $OUT/calib_summary.json && cat $OUT/calib_summary.json
