# phase stamps of the update kernel (istamps build) and the stance solve (stamps build), all-stance B=4096
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_istamps.so timeout -k 10 120 python tools/ustamps.py stance_cold 4096 > gpurun_out/ust_stance_cold.log 2>&1 &&
WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_stamps.so timeout -k 10 120 python tools/sstamps.py 4096 > gpurun_out/sst_stance_cold.log 2>&1
