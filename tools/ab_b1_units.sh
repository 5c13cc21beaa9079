set -e
cd $GRAFT_REPO_ROOT
Q=quadrupedwholebodycontroller_amd
V=${VARIANTS:-cur,alldef,allit}; O=gpurun_out/${OUT:-unit2}
mkdir -p $O
timeout -k 10 500 python tools/variants.py 40 $V > $O/variants.log 2>&1
for r in 0 1; do for v in ${V//,/ }; do
  d=/tmp/b1v_$v; mkdir -p $d; cp $Q/wbc_control_loop $Q/libwbc_controller.so $d/; cp $Q/libwbc_hip_$v.so $d/libwbc_hip.so
  timeout -k 10 120 $d/wbc_control_loop stance 3000 0 default > $O/b1_${v}_$r.log 2>&1
done; done
grep -h cycle_us_mean $O/b1_*.log | cut -c1-140
