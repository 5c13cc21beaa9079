# LDS bank conflicts / LDS instructions / VALU per wave of diagnostic variants (not product code)
cd $GRAFT_REPO_ROOT
O=gpurun_out/diagv
mkdir -p $O
for v in "" _diag_NOLOOP _diag_NOSOLVE; do
  lib=quadrupedwholebodycontroller_amd/libwbc_hip$v.so
  WBC_LIB=$lib timeout -k 10 60 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d $O/pmc$v -o p -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc$v.log 2>&1 || { tail -3 $O/pmc$v.log; exit 1; }
  python3 - "$O" "$v" <<'PY'
import sys, csv, glob, collections
O, v = sys.argv[1], sys.argv[2]
f = glob.glob(f"{O}/pmc{v}/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(float)
for row in csv.DictReader(open(f[0])):
    if 'update_solve' in row['Kernel_Name']: acc[row['Counter_Name']] += float(row['Counter_Value'])
w = acc['SQ_WAVES']
print(v or 'base', {k: round(acc[k] / w, 1) for k in acc if k != 'SQ_WAVES'})
PY
done
