# Round-end evidence on one GPU box: GPU tests, smoke, the default bench line (with the CPU
# baseline), the --extra configs, a rocprofv3 kernel-trace summary of the same bench command, and
# the PMC passes (separate runs) whose summary bench.py reads for roofline.traffic.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-final}
O=gpurun_out/$TAG
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; if [ $rc -ne 0 ]; then tail -30 $O/$name.log; exit $rc; fi; }
step pytest 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
step smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
step pmc 600 env TAG=$TAG bash tools/pmc.sh
cp gpurun_out/pmc_$TAG/pmc_summary.json $O/pmc_stance_cold_b4096.json
cp $O/pmc_stance_cold_b4096.json profiles/r01/pmc_stance_cold_b4096.json  # read by bench.py below
step bench 300 python bench.py --steps 50 --warmup 5
step bench_extra 300 python bench.py --steps 20 --warmup 3 --extra --breakdown --no-cpu-baseline
step prof 300 rocprofv3 --kernel-trace --stats -d $O/prof -o prof --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline
tail -1 $O/bench.log
echo final done
