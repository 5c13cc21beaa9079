# update-kernel stage stamps (istamps build) for one workload
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so timeout -k 10 120 python tools/ustamps.py ${UST_CFG:-stance_cold} 4096 > gpurun_out/ust_${UST_CFG:-stance_cold}.log 2>&1
