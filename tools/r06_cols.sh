#!/bin/bash
# round 6: the column exchange with deferred sections -- its GPU tests, then the k=7 merge timings
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_dotset.py -k "column" > gpurun_out/cols_test.log 2>&1 || { tail -40 gpurun_out/cols_test.log; exit 1; }
grep -E "passed|failed" gpurun_out/cols_test.log | tail -3
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_multi.py > gpurun_out/cols_multi.log 2>&1 || { tail -40 gpurun_out/cols_multi.log; exit 1; }
grep -E "passed|failed" gpurun_out/cols_multi.log | tail -3
for rc in own read; do
  CE_HOST_PROF=1 timeout -k 10 400 python -u tools/cols_bench.py --parts 7 --rm-ctx $rc --steps 10 > gpurun_out/cols_k7_$rc.json 2> gpurun_out/cols_k7_$rc.err || { tail -20 gpurun_out/cols_k7_$rc.err; exit 1; }
  tail -1 gpurun_out/cols_k7_$rc.json
  grep -E "cols:" gpurun_out/cols_k7_$rc.err | tail -12
done
