#!/bin/bash
# GPU parity tests, then an A/B of the fused-kernel variants on the C2 bench (no CPU leg).
#   CE_FUSED (1 k_open_fold_small, 2 k_open_fold_v2), CE_FILES_PER_WAVE, CE_V2_WAVES
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/gpu_all.log
for V in ${VARIANTS:-"1 4 0" "2 4 2" "2 4 3" "2 2 3" "2 2 4"}; do
  set -- $V
  CE_FUSED=$1 CE_FILES_PER_WAVE=$2 CE_V2_WAVES=$3 timeout -k 10 150 python bench.py --no-cpu \
    > gpurun_out/b_$1_$2_$3.json 2> gpurun_out/b_$1_$2_$3.err || { echo "bench $V failed"; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/b_$1_$2_$3.json'));print('$V', d['ms_per_step'], d['kernels_ms_per_step']['open_fold_small'], d['state_check'])"
done
