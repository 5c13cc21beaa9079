cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03e
for c in stance_cold:4096 rl_random:8192; do
  n=${c%%:*}; b=${c##*:}
  WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so timeout -k 10 120 python tools/ust16.py $n $b > gpurun_out/r03e/ust_$n.log 2>&1 || { echo "fail $n"; tail gpurun_out/r03e/ust_$n.log; exit 1; }
  cat gpurun_out/r03e/ust_$n.log
done
