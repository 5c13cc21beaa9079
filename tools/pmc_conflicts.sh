#!/bin/bash
# LDS bank conflicts / LDS and VALU instructions / wait per wave of the headline step for each
# library variant (VARIANTS="prev new"; product library if empty): one --pmc pass each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-pmcc}
mkdir -p $O
for v in ${VARIANTS:-product}; do
  lib=quadrupedwholebodycontroller_amd/libwbc_hip_$v.so; [ "$v" = product ] && lib=quadrupedwholebodycontroller_amd/libwbc_hip.so
  WBC_LIB=$lib timeout -k 10 90 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d $O/pmc_$v -o p -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc_$v.log 2>&1 || { tail -3 $O/pmc_$v.log; exit 1; }
  python3 - "$O" "$v" <<'PY'
import sys, csv, glob, collections
O, v = sys.argv[1], sys.argv[2]
f = glob.glob(f"{O}/pmc_{v}/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(float)
for row in csv.DictReader(open(f[0])):
    if 'update_solve' in row['Kernel_Name']: acc[row['Counter_Name']] += float(row['Counter_Value'])
w = acc['SQ_WAVES']
print(v, {k: round(acc[k] / w, 1) for k in acc if k != 'SQ_WAVES'})
PY
done
