# modes16 traffic + time with the XCD block remap
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_modes.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python bench.py --config modes16_b16384 --steps 50 --warmup 5 --no-cpu-baseline > $O/b.log 2>&1 || exit 1
python3 -c "import json;d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]);print('modes16', d['value']/1e6, d['ms_per_step'])"
for set in FETCH_SIZE WRITE_SIZE; do
timeout -k 10 60 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $O/p_$set -o p -- python3 bench.py --config modes16_b16384 --steps 5 --warmup 1 --no-cpu-baseline > $O/p_$set.log 2>&1 || exit 1
done
python3 - <<'PY'
import csv, glob, collections
for s in ('FETCH_SIZE','WRITE_SIZE'):
    f=glob.glob(f'gpurun_out/r03k/p_{s}/**/*counter_collection.csv', recursive=True)[0]
    v=collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'update_solve' in r['Kernel_Name']: v[r['Dispatch_Id']].append(float(r['Counter_Value']))
    tot=[sum(x) for x in v.values()]
    print(s, 'KB per launch (raw, before gfx950 correction)', sum(tot)/len(tot))
PY
