cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/r03b.pytest.log 2>&1
echo "pytest rc=$?"
grep -E "PASSED|FAILED|ERROR" gpurun_out/r03b.pytest.log | grep -v PASSED | head -40
tail -3 gpurun_out/r03b.pytest.log
