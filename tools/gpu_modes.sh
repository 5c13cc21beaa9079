set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/m1.pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/m1.pytest.log; exit 1; }
tail -3 gpurun_out/m1.pytest.log
timeout -k 10 200 python bench.py --config modes16_b16384 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/m1.bench_modes.log 2>&1 || { echo bench_modes rc=$?; tail gpurun_out/m1.bench_modes.log; exit 1; }
tail -1 gpurun_out/m1.bench_modes.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --extra --no-cpu-baseline > gpurun_out/m1.bench_extra.log 2>&1 || { echo bench_extra rc=$?; tail gpurun_out/m1.bench_extra.log; exit 1; }
tail -1 gpurun_out/m1.bench_extra.log
