#!/bin/bash
# Round 3: the GPU suite, the C2 bench line + one-step timeline, C3 with host phases + timeline.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/gpu_all.log | head -80; exit $rc; }
timeout -k 10 300 python bench.py --configs '' --no-cpu --no-variant-b --no-host-buffers > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err || { echo "bench failed"; tail gpurun_out/bench_c2.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/bench_c2.json'))
print('C2', d.get('value'), d['ms_per_step'], d['roofline']['avg_launch_ms'], d.get('state_check'), d['kernels_ms_per_step'])"
./tools/step_trace.sh > gpurun_out/steptrace.txt 2>&1 || { echo "step trace failed"; tail gpurun_out/steptrace.txt; exit 1; }
tail -24 gpurun_out/steptrace.txt
CE_HOST_PROF=1 timeout -k 10 300 python bench_configs.py --config c3 --steps 10 --no-cpu > gpurun_out/c3.json 2> gpurun_out/c3_hostprof.err || { echo c3 failed; tail gpurun_out/c3_hostprof.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c3.json'));print('c3', d['ms_per_step'], d['phases_ms_per_step'], d['checks'])"
./tools/c3_trace.sh > gpurun_out/c3trace.txt 2>&1 || { echo "c3 trace failed"; tail gpurun_out/c3trace.txt; exit 1; }
python3 tools/c3_step_breakdown.py gpurun_out/c3trace/t 10 > gpurun_out/c3_step.txt && grep -A 30 "step span" gpurun_out/c3_step.txt
