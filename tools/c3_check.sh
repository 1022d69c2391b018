#!/bin/bash
# Every GPU test, then the C3 line without the names and one traced C3 step (op count, idle).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
CE_C3_NO_NAMES=1 timeout -k 10 300 python -u bench_configs.py --config c3 --no-cpu > gpurun_out/c3_nn.json 2> gpurun_out/c3_nn.err || exit 1
python3 -c "
import json;d=json.load(open('gpurun_out/c3_nn.json'));print(d['ms_per_step'], d['phases_ms_per_step'])"
CE_C3_NO_NAMES=1 bash tools/c3_step.sh > /dev/null && grep "step span" gpurun_out/c3s/c3_step.txt
