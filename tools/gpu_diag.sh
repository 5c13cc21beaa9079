# Stamp diagnostics (per-phase and per-loop-step cycles) for the stance and random workloads.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
L=quadrupedwholebodycontroller_amd
for cfg in "stance_cold 4096" "rl_random 8192"; do
  set -- $cfg
  timeout -k 10 120 env WBC_LIB=$L/libwbc_hip_istamps.so python tools/istamps.py $1 $2 > gpurun_out/diag.istamps.$1.log 2>&1 || { echo "istamps $1 rc=$?"; tail gpurun_out/diag.istamps.$1.log; exit 1; }
  timeout -k 10 120 env WBC_LIB=$L/libwbc_hip_stamps.so python tools/stamps.py $1 $2 > gpurun_out/diag.stamps.$1.log 2>&1 || { echo "stamps $1 rc=$?"; tail gpurun_out/diag.stamps.$1.log; exit 1; }
done
echo diag done
