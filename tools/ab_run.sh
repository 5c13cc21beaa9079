#!/bin/bash
# A/B session on one GPU box: the GPU tests on the product library and on each variant library
# (WBC_LIB), then tools/variants.py timing the variants side by side.
# VARIANTS="old,new,nsz" TAG=ab bash tools/ab_run.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in ${TEST_VARIANTS:-}; do
  WBC_LIB=quadrupedwholebodycontroller_amd/libwbc_hip_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
timeout -k 10 400 python tools/variants.py ${STEPS:-50} ${VARIANTS:-old,new} > $O/variants.log 2>&1 || { tail -20 $O/variants.log; exit 1; }
python3 - $O/variants.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if '#' not in l.split(' ')[0]: continue
    n, d = l.split(' ', 1)
    d = json.loads(d)
    print(n, {k: round(v['solves_per_s'] / 1e6, 2) for k, v in d.items() if isinstance(v, dict) and 'solves_per_s' in v})
PY
