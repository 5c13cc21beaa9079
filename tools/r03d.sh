cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03d
O=gpurun_out/r03d
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; if [ $rc -ne 0 ]; then tail -20 $O/$name.log; exit $rc; fi; }
step bench 300 python bench.py --steps 50 --warmup 5 --extra --breakdown --no-cpu-baseline
step b1_fused 120 quadrupedwholebodycontroller_amd/wbc_control_loop stance 3000 0 fused
step b1_default 120 quadrupedwholebodycontroller_amd/wbc_control_loop stance 3000 0 default
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline --extra
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/r03d/bench.log').read().strip().splitlines()[-1])
print('headline', d['value']/1e6, d['ms_per_step'], d['roofline']['frac'], d.get('breakdown'))
for k,v in d['extra'].items(): print(k, v.get('solves_per_s',0)/1e6, v.get('ms_per_step'), v.get('mean_iters'), v['roofline']['frac'])
for n in ('b1_fused','b1_default'):
    print(n, open('gpurun_out/r03d/%s.log'%n).read().strip().splitlines()[-1][:200])
PY
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs head -12
