# GPU tests on the default build, then an A/B timing of variant libraries (VARIANTS=a,b,...)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG.pytest.log 2>&1 || { echo "pytest rc=$?"; tail -40 gpurun_out/$TAG.pytest.log; exit 1; }
tail -2 gpurun_out/$TAG.pytest.log
fi
timeout -k 10 600 python tools/variants.py ${STEPS:-30} $VARIANTS > gpurun_out/$TAG.variants.log 2>&1 || { echo "variants rc=$?"; tail gpurun_out/$TAG.variants.log; exit 1; }
cat gpurun_out/$TAG.variants.log
