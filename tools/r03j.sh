# full GPU suite, bench (+extras), headline kernel stats
cd $GRAFT_REPO_ROOT
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --extra --no-cpu-baseline > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/r03j/bench.log').read().strip().splitlines()[-1])
print('headline', d['value']/1e6, d['ms_per_step'], d['roofline']['kernel_ms'])
for k,v in d['extra'].items(): print(k, round(v.get('solves_per_s',0)/1e6,2), v.get('ms_per_step'))
PY
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o p --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 && cut -c1-120 $O/prof/p_kernel_stats.csv | head -4
