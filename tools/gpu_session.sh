#!/bin/bash
# One GPU-box session of round 5: each step under its own timeout, stop at the first failure.
# STEPS="tests ab qmap calib" VARIANTS=a,b TAG=x bash tools/gpu_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-s}
O=gpurun_out/$TAG
mkdir -p $O
for s in ${STEPS:-tests ab}; do
  echo "== $s $(date +%T)"
  case $s in
    tests) timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
           rc=$?; tail -3 $O/pytest.log ;;
    ab) timeout -k 10 700 python tools/variants.py ${AB_STEPS:-50} ${VARIANTS} > $O/variants.log 2>&1; rc=$?
        python3 - $O/variants.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if '#' not in l.split(' ')[0]: continue
    n, d = l.split(' ', 1)
    d = json.loads(d)
    print(n, {k: round(v['solves_per_s'] / 1e6, 2) for k, v in d.items() if isinstance(v, dict) and 'solves_per_s' in v})
PY
        ;;
    qmap) timeout -k 10 200 python tools/qmap_probe.py 30 > $O/qmap_probe.log 2>&1; rc=$?; cat $O/qmap_probe.log
          if [ $rc -eq 0 ]; then
            (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/qmap_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/qmap_probe.py 10 > $GRAFT_REPO_ROOT/$O/qmap_prof.log 2>&1); rc=$?
          fi ;;
    calib) OUT=$O/calib bash tools/calib.sh > $O/calib.log 2>&1; rc=$?; tail -40 $O/calib.log ;;
    bench) timeout -k 10 400 python bench.py --steps ${BENCH_STEPS:-20} --warmup 3 > $O/bench.log 2>&1; rc=$?; tail -1 $O/bench.log ;;
    extra) timeout -k 10 400 python bench.py --steps 20 --warmup 3 --extra --no-cpu-baseline > $O/bench_extra.log 2>&1; rc=$?; grep '^{' $O/bench_extra.log | cut -c1-200 ;;
    ust) for c in ${UST_CFGS:-stance_cold trot rl_random}; do
           B=4096; [ $c = rl_random ] && B=8192
           WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so timeout -k 10 200 python tools/ust16.py $c $B > $O/ust_$c.log 2>&1; rc=$?
           [ $rc -ne 0 ] && break
         done; grep -h "loop\|hotstart\|entry to end" $O/ust_*.log | head -40 ;;
    b1) for m in default launch default launch; do
          timeout -k 10 120 quadrupedwholebodycontroller_amd/wbc_control_loop stance 3000 0 $m >> $O/b1_$m.log 2>&1; rc=$?
          [ $rc -ne 0 ] && break
        done; tail -n 2 $O/b1_default.log $O/b1_launch.log | cut -c1-200 ;;
    listc) timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1; rc=$?; grep -o "SQ_INSTS_VALU[A-Z0-9_]*F64[A-Z0-9_]*" $O/counters.txt | sort -u ;;
    pmc) CONFIG=${PMC_CONFIG:-stance_cold_b4096} BATCH=${PMC_BATCH:-4096} TAG=${TAG}_$PMC_CONFIG bash tools/pmc.sh > $O/pmc_$PMC_CONFIG.log 2>&1; rc=$?; tail -3 $O/pmc_$PMC_CONFIG.log ;;
    *) echo "unknown step $s"; rc=2 ;;
  esac
  echo "== $s rc=$rc $(date +%T)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
