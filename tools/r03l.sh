# full GPU suite, bench (+extras), conflict / instruction counters on the headline
export TAG=${TAG:-r03l}
cd $GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r03l}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --extra --no-cpu-baseline > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
TAG=${TAG:-r03l} python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/'+__import__("os").environ.get("TAG","r03l")+'/bench.log').read().strip().splitlines()[-1])
print('headline', d['value']/1e6, d['ms_per_step'])
for k,v in d['extra'].items(): print(k, round(v.get('solves_per_s',0)/1e6,2), v.get('ms_per_step'))
PY
timeout -k 10 60 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --kernel-trace --output-format csv -d $O/pmc -o p -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $O/pmc.log 2>&1 || { tail -3 $O/pmc.log; exit 1; }
TAG=${TAG:-r03l} python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/"+__import__("os").environ.get("TAG","r03l")+"/pmc/**/*counter_collection.csv", recursive=True)
acc = collections.defaultdict(float)
for row in csv.DictReader(open(f[0])):
    if 'update_solve' in row['Kernel_Name']: acc[row['Counter_Name']] += float(row['Counter_Value'])
w = acc['SQ_WAVES']
print({k: round(acc[k] / w, 1) for k in acc if k != 'SQ_WAVES'})
PY
