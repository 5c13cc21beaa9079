# stage cycles of both forms (stance_cold headline, rl_random general) + bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03h
O=gpurun_out/r03h
timeout -k 10 300 python -u -m pytest tests/test_gpu_iters.py tests/test_gpu_parity.py tests/test_gpu_stateful.py tests/test_gpu_modes.py tests/test_gpu_fallback_sequence.py tests/test_gpu_stream.py tests/test_gpu_controller.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --extra --no-cpu-baseline > $O/bench.log 2>&1 || { tail $O/bench.log; exit 1; }
python3 - <<'PY'
import json
d=json.loads(open('gpurun_out/r03h/bench.log').read().strip().splitlines()[-1])
print('headline', d['value']/1e6, d['ms_per_step'])
for k,v in d['extra'].items(): print(k, round(v.get('solves_per_s',0)/1e6,2), v.get('ms_per_step'))
PY
WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so timeout -k 10 120 python tools/ust16.py stance_cold 4096 > $O/ust_st.log 2>&1 && grep -E "stance|loop|total|iters" $O/ust_st.log
WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so timeout -k 10 120 python tools/ust16.py rl_random 8192 > $O/ust_rl.log 2>&1 && grep -E "general|loop|total" $O/ust_rl.log
for c in "stance_cold 4096" "rl_random 8192"; do
WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so timeout -k 10 120 python tools/ist16.py $c > $O/ist_${c%% *}.log 2>&1 || { tail $O/ist_${c%% *}.log; exit 1; }
grep -A7 cycles_per $O/ist_${c%% *}.log
done
