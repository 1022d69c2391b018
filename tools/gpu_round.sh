#!/bin/bash
# One GPU call: parity tests, the default bench (with the CPU baseline leg), rocprofv3 evidence
# (tools/rocprof.sh: kernel-trace stats + FETCH_SIZE/WRITE_SIZE passes), C3 with host phases.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
[ -n "$NO_ROCPROF" ] || ./tools/rocprof.sh || exit 1
cd $GRAFT_REPO_ROOT
CE_HOST_PROF=1 timeout -k 10 300 python bench_configs.py --config c3 > gpurun_out/c3.json 2> gpurun_out/c3.err || { echo c3 failed; tail gpurun_out/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c3.json'));print('c3', d['ms_per_step'], d['phases_ms_per_step'], d['checks'])"
