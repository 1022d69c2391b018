#!/bin/bash
# round 6: the 8-lane DS open (k_open_ds8) -- dot-set tests, then C3 same-box A/B against the
# 16-lane DS form (CE_DS8=0), no names, no CPU leg
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 600 $T tests/test_gpu_dotset.py tests/test_gpu_configs.py 2>&1 | tee gpurun_out/t_ds8.log | tail -3
for r in 1 2; do for v in 1 0; do
  CE_DS8=$v CE_C3_NO_NAMES=1 timeout -k 10 300 python -u bench_configs.py --config c3 --no-cpu --steps 60 > gpurun_out/ds8_$v.json 2> gpurun_out/ds8_$v.err || { tail -20 gpurun_out/ds8_$v.err; exit 1; }
  python3 -c "
import json;l=json.loads(open('gpurun_out/ds8_$v.json').read().strip().splitlines()[-1]);k=l['kernels_ms_per_step']
print('CE_DS8=$v', l['ms_per_step'], {x:k.get(x) for x in ('open_setup','open_small','segments_open')}, l['checks'])"
done; done
