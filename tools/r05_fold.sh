#!/bin/bash
# partitioned-fold check: dot-set GPU tests, then the C3 line's fold figures and kernel times
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ "$TESTS" = none ] || timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  ${TESTS:-tests/test_gpu_dotset.py} > gpurun_out/fold_tests.log 2>&1 || { tail -40 gpurun_out/fold_tests.log; exit 1; }
[ "$TESTS" = none ] || tail -2 gpurun_out/fold_tests.log
CE_C3_NO_NAMES=1 timeout -k 10 300 python -u bench_configs.py --config c3 --steps 40 --no-cpu > gpurun_out/fold_c3.json 2> gpurun_out/fold_c3.err || { tail -30 gpurun_out/fold_c3.err; exit 1; }
python - <<'PY'
import json
l = json.loads(open("gpurun_out/fold_c3.json").read().strip().splitlines()[-1])
print(json.dumps({k: l.get(k) for k in ("ms_per_step", "fold", "checks")}))
print(json.dumps(l.get("kernels_ms_per_step")))
PY
