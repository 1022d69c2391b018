#!/bin/bash
# round 6: C3 with read-context removals -- the small-size GPU test, then the full bench_configs line
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_configs.py -k read_context > gpurun_out/c3r_test.log 2>&1 || { tail -30 gpurun_out/c3r_test.log; exit 1; }
tail -2 gpurun_out/c3r_test.log
timeout -k 10 500 python -u bench_configs.py --config c3r ${C3R_ARGS:-} > gpurun_out/c3r.json 2> gpurun_out/c3r.err || { tail -30 gpurun_out/c3r.err; exit 1; }
python3 - <<'PY'
import json
l = json.loads(open("gpurun_out/c3r.json").read().strip().splitlines()[-1])
print(json.dumps({k: l.get(k) for k in ("ms_per_step", "value", "checks", "config", "fold", "kernels_ms_per_step", "phases_ms_per_step", "pipelined")}, indent=0)[:4000])
print("cpu", json.dumps(l.get("cpu_baseline"))[:600])
PY
for rc in own read; do
  timeout -k 10 400 python -u tools/cols_bench.py --parts 7 --rm-ctx $rc --steps 10 > gpurun_out/cols_k7_$rc.json 2> gpurun_out/cols_k7_$rc.err || { tail -20 gpurun_out/cols_k7_$rc.err; exit 1; }
  tail -1 gpurun_out/cols_k7_$rc.json
done
