#!/bin/bash
# Round 3: sharded-gate GPU tests, the whole GPU suite, a 2-rank bench rehearsal on one GPU
# (gloo), the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_multi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_shard.log 2>&1
rc=$?; echo "shard tests rc=$rc"; tail -5 gpurun_out/gpu_shard.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
CE_BENCH_SHARE_GPU=1 CE_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --configs '' --gpus 2 --steps 5 --warmup 1 --no-cpu --no-variant-b > gpurun_out/bench2.json 2> gpurun_out/bench2.err || { echo "bench2 failed"; tail gpurun_out/bench2.err; exit 1; }
cat gpurun_out/bench2.json
timeout -k 10 550 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
./tools/step_trace.sh > gpurun_out/steptrace.txt 2>&1 || { echo "step trace failed"; tail gpurun_out/steptrace.txt; exit 1; }
tail -60 gpurun_out/steptrace.txt
