#!/bin/bash
# column-exchange GPU check: dot-set + multi-process tests, then a full-size 2-rank C3 rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ "$TESTS" = none ] || timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  ${TESTS:-tests/test_gpu_dotset.py tests/test_gpu_multi.py} > gpurun_out/cols_tests.log 2>&1 || { tail -40 gpurun_out/cols_tests.log; exit 1; }
[ "$TESTS" = none ] || tail -3 gpurun_out/cols_tests.log
CE_BENCH_SHARE_GPU=1 CE_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --versions 2 --steps 5 \
  --warmup 2 --no-cpu --no-variant-b --no-strong --configs c3 > gpurun_out/cols_c3.json 2> gpurun_out/cols_c3.err || { tail -30 gpurun_out/cols_c3.err; exit 1; }
python - <<'PY'
import json
l = json.loads(open("gpurun_out/cols_c3.json").read().strip().splitlines()[-1])
c = l["configs"]["c3"]
print(json.dumps({k: c[k] for k in ("ms_per_step", "exchange", "checks", "phases_ms_per_step_rank0", "kernels_ms_per_step_rank0")}))
PY
