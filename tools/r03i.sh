cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03i
O=gpurun_out/r03i
for c in "stance_cold 4096" "rl_random 8192"; do
WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so timeout -k 10 120 python tools/ist16.py $c > $O/ist_${c%% *}.log 2>&1 || { tail $O/ist_${c%% *}.log; exit 1; }
tail -12 $O/ist_${c%% *}.log
done
