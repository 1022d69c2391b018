#!/bin/bash
# Dot-set parity tests, then the C3 bench with host phases (CE_HOST_PROF) and its kernel times.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dotset or orswot or mvreg or c3 or template or parity" > gpurun_out/gpu_ds.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_ds.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/gpu_ds.log | head -60; exit $rc; }
CE_HOST_PROF=1 timeout -k 10 300 python bench_configs.py --config c3 --steps ${C3_STEPS:-20} --no-cpu > gpurun_out/c3.json 2> gpurun_out/c3_hostprof.err || { echo c3 failed; tail gpurun_out/c3_hostprof.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c3.json'));print('c3', d['ms_per_step'], d['phases_ms_per_step'], d['checks']); print(d['kernels_ms_per_step']); print(d['single_compact_latency'])"
grep "CE_HOST_PROF" gpurun_out/c3_hostprof.err | tail -26
