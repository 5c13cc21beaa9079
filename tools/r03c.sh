cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r03c.pytest.log 2>&1
echo "pytest rc=$?"
grep -E "FAILED|ERROR" gpurun_out/r03c.pytest.log | head -40
tail -2 gpurun_out/r03c.pytest.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --extra --no-cpu-baseline > gpurun_out/r03c.extra.log 2>&1
echo "bench rc=$?"
tail -1 gpurun_out/r03c.extra.log | python3 -c "
import json,sys;d=json.loads(sys.stdin.read())
print('headline', d['value']/1e6, d['ms_per_step'])
for k,v in d['extra'].items(): print(k, v.get('solves_per_s',0)/1e6, v.get('ms_per_step'), v.get('mean_iters', v.get('mean_iters_last')))"
