#!/bin/bash
# PMC passes (separate rocprofv3 runs; never combined with trace domains) of one bench workload:
# CONFIG=<bench config> [BATCH=<batch>] TAG=... bash tools/pmc.sh
# -> gpurun_out/pmc_$TAG/pmc_summary.json (tools/pmc_summary.py), read by bench.py for roofline.traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-pmc}
CONFIG=${CONFIG:-stance_cold_b4096}
BATCH=${BATCH:-4096}
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
CMD="python3 bench.py --config $CONFIG --steps 10 --warmup 2 --no-cpu-baseline"
# every bench config's step is one kernel: the default step's, or the mode loop's for hypotheses
STEPK=wbc_update_solve_kernel,wbc_modes_kernel
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" ${EXTRA_SETS:-}; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d $OUT -o pass$i -- $CMD > $OUT/pass$i.log 2>&1
  rc=$?
  echo "pass$i [$set] rc=$rc" >> $OUT/passes.txt
  if [ $rc -ne 0 ]; then echo "pmc pass $i failed rc=$rc"; tail -5 $OUT/pass$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $OUT $OUT/pmc_summary.json $CONFIG $BATCH $STEPK > /dev/null
