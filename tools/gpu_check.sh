#!/bin/bash
# One GPU-box session: each GPU step under its own timeout; stop at the first crash / timeout.
# Exit codes 0 (pass) and 1 (Python test/assert failure) continue; anything else ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-run}
step() {
  local name=$1 t=$2; shift 2
  echo "== $name (timeout $t s) $(date +%T)" >> gpurun_out/steps.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$TAG.$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc $(date +%T)" >> gpurun_out/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name rc=$rc"; exit $rc; fi
  return 0
}
for s in ${STEPS:-smoke pytest bench prof}; do
  case $s in
    smoke)  step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" ;;
    pytest) step pytest 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    bench)  step bench 400 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 ${BENCH_ARGS:-} ;;
    stamps) step stamps 300 env WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_stamps.so python tools/stamps.py stance_cold 4096 ;;
    istamps) step istamps 300 env WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so python tools/istamps.py stance_cold 4096 ;;
    stamps2) step stamps2 300 env WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_stamps.so python tools/stamps.py rl_random 8192 ;;
    split) step split 600 python tools/split_probe.py 30 ${VARIANTS:-uw2,uw3,uw4} ;;
    variants) step variants 600 python tools/variants.py 30 ${VARIANTS:-w2,w3,w4,w5} ;;
    dist)   step dist 400 env WBC_DIST_BACKEND=gloo python bench.py --gpus 2 --config rl_random_b65536 --steps 10 --warmup 2 ;;
    strong1) step strong1 400 python bench.py --config rl_random_b65536 --steps 10 --warmup 2 --no-cpu-baseline ;;
    extra)  step extra 400 python bench.py --steps 20 --warmup 3 --extra --no-cpu-baseline ;;
    counters) step counters 120 rocprofv3 -L ;;
    pmc)    step pmc 1200 bash tools/pmc.sh ;;
    prof)   step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o $TAG --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
  esac
done
echo done
