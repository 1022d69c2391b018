#!/bin/bash
# GPU tests, C2 bench A/B (old vs v2) with host-phase timing, C3 bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/gpu_all.log
for V in "1 4 0" "2 4 2" "1 4 0" "2 4 2"; do
  set -- $V
  CE_FUSED=$1 CE_FILES_PER_WAVE=$2 CE_V2_WAVES=$3 timeout -k 10 150 python bench.py --configs '' --no-cpu \
    > gpurun_out/b_$1_$2_$3.json 2> gpurun_out/b_$1_$2_$3.err || { echo "bench $V failed"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b_$1_$2_$3.json'));print('$V', d['ms_per_step'], d['kernels_ms_per_step']['open_fold_small'], d['state_check'])"
done
CE_HOST_PROF=1 CE_FUSED=2 timeout -k 10 150 python bench.py --configs '' --no-cpu --steps 3 --warmup 1 > gpurun_out/b_hostprof.json 2> gpurun_out/b_hostprof.err || exit 1
tail -12 gpurun_out/b_hostprof.err
CE_HOST_PROF=1 timeout -k 10 300 python bench_configs.py --config c3 > gpurun_out/c3.json 2> gpurun_out/c3.err || { echo c3 failed; tail gpurun_out/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c3.json'));print('c3', d['ms_per_step'], d['phases_ms_per_step'], d['checks'])"
