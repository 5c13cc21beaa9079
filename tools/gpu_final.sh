# Round evidence on one GPU box: GPU tests, smoke, PMC passes for the bench workloads (separate
# runs; their summaries under profiles/$ROUND/ are what bench.py reads for roofline.traffic), the
# default bench line (with the CPU baseline), the --extra configs, and a rocprofv3 kernel-trace
# summary of the same bench command.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-final}
ROUND=${ROUND:-r06}
O=gpurun_out/$TAG
mkdir -p $O profiles/$ROUND
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$name.log; exit $rc; fi; }
PART=${PART:-all}  # 1: calibration, tests, smoke, PMC passes; 2: bench lines, profiles, probes
if [ $PART != 2 ]; then
step calib 300 env OUT=$O/calib bash tools/calib.sh
mkdir -p profiles/$ROUND/calib && cp $O/calib/calib_summary.json $O/calib/known.json $O/calib/pass*_counter_collection.csv profiles/$ROUND/calib/
step pytest 400 env WBC_MARGINS_OUT=$O/parity_margins.json python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
cp $O/parity_margins.json profiles/$ROUND/parity_margins.json
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
for cb in stance_cold_b4096:4096 rl_random_b8192:8192 modes16_b16384:16384 trot_stateful_b4096:4096; do
  c=${cb%%:*}; b=${cb##*:}
  step pmc_$c 600 env TAG=${TAG}_$c CONFIG=$c BATCH=$b bash tools/pmc.sh
  cp gpurun_out/pmc_${TAG}_$c/pmc_summary.json $O/pmc_$c.json
  cp $O/pmc_$c.json profiles/$ROUND/pmc_$c.json  # read by bench.py below
done
fi
if [ $PART = 1 ]; then echo part1 done; exit 0; fi
step bench 300 python bench.py --steps 50 --warmup 5
step bench_extra 300 python bench.py --steps 20 --warmup 3 --extra --breakdown --no-cpu-baseline
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline
for cb in rl_random_b8192 modes16_b16384; do
  step prof_$cb 300 rocprofv3 --kernel-trace --stats -d $O/prof_$cb -o prof --output-format csv -- python3 bench.py --config $cb --steps 200 --warmup 20 --no-cpu-baseline
done
step b1_fused 120 quadrupedwholebodycontroller_amd/wbc_control_loop stance 3000 0 fused
step b1_launch 120 quadrupedwholebodycontroller_amd/wbc_control_loop stance 3000 0 launch
step b1_default 120 quadrupedwholebodycontroller_amd/wbc_control_loop stance 3000 0 default
step qmap_probe 200 python tools/qmap_probe.py 30
step b1_probe 120 python tools/b1_probe.py 2000
step batch_sweep 180 python tools/batch_sweep.py 50
step ust_stance 120 env WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so python tools/ust16.py stance_cold 4096
step ust_rl 120 env WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so python tools/ust16.py rl_random 8192
step ust_trot 120 env WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so python tools/ust16.py trot 4096
step modes_sweep 180 python tools/modes_sweep.py 50
tail -1 $O/bench.log
echo final done
