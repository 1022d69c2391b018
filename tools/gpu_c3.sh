#!/bin/bash
# C3 host-phase profile + the box's CPU share
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))"
timeout -k 10 300 python -u -m pytest tests/test_gpu_dotset.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "compact" > gpurun_out/gpu_compact.log 2>&1
rc=$?; echo "compact tests rc=$rc"; tail -3 gpurun_out/gpu_compact.log; [ $rc -eq 0 ] || exit $rc
CE_HOST_PROF=1 timeout -k 10 300 python bench_configs.py --config c3 > gpurun_out/c3.json 2> gpurun_out/c3.err || { echo c3 failed; tail gpurun_out/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c3.json'));print('c3', d['ms_per_step'], d['phases_ms_per_step'], d['checks'])"
grep -v "states: \|ops: " gpurun_out/c3.err | tail -16
