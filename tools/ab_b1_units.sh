set -e
cd $GRAFT_REPO_ROOT
Q=quadrupedwholebodycontroller_amd
mkdir -p gpurun_out/unit2
timeout -k 10 500 python tools/variants.py 40 cur,alldef,allit > gpurun_out/unit2/variants.log 2>&1
for r in 0 1; do for v in cur alldef allit; do
  d=/tmp/b1v_$v; mkdir -p $d; cp $Q/wbc_control_loop $Q/libwbc_controller.so $d/; cp $Q/libwbc_hip_$v.so $d/libwbc_hip.so
  timeout -k 10 120 $d/wbc_control_loop stance 3000 0 default > gpurun_out/unit2/b1_${v}_$r.log 2>&1
done; done
grep -h cycle_us_mean gpurun_out/unit2/b1_*.log | cut -c1-140
