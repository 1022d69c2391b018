#!/bin/bash
# The state reader's single host wait: dot-set + multi-rank GPU tests, the C3 host phases
# (CE_HOST_PROF) and the C3 line / step trace without the names.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rd
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dotset.py tests/test_gpu_multi.py > gpurun_out/rd/tests.log 2>&1 || { tail -30 gpurun_out/rd/tests.log; exit 1; }
tail -2 gpurun_out/rd/tests.log
CE_HOST_PROF=1 CE_C3_NO_NAMES=1 timeout -k 10 300 python -u bench_configs.py --config c3 --no-cpu > gpurun_out/rd/c3hp.json 2> gpurun_out/rd/c3hp.err || { echo "c3 host prof failed"; exit 1; }
python3 tools/host_prof_summary.py gpurun_out/rd/c3hp.err 40 > gpurun_out/rd/hostprof.txt
CE_C3_NO_NAMES=1 timeout -k 10 300 python -u bench_configs.py --config c3 --no-cpu > gpurun_out/rd/c3nn.json 2> gpurun_out/rd/c3nn.err || { echo "c3 failed"; exit 1; }
tail -1 gpurun_out/rd/c3nn.json | head -c 200; echo
CE_C3_NO_NAMES=1 bash tools/c3_step.sh > /dev/null && grep "step span" gpurun_out/c3s/c3_step.txt
