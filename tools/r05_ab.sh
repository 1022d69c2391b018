#!/bin/bash
# same-box A/B of an env knob on the C3 line without names: tools/r05_ab.sh VAR=value [...]
# (alternating runs: base, knob, base, knob) -> ms/step and the fold's ms
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab
for i in 1 2; do
  for mode in base knob; do
    if [ $mode = knob ]; then E="$*"; else E=""; fi
    env $E CE_C3_NO_NAMES=1 timeout -k 10 300 python -u bench_configs.py --config c3 --steps 60 --no-cpu > gpurun_out/ab/$mode$i.json 2> gpurun_out/ab/$mode$i.err || { echo "$mode rc=$?"; tail -5 gpurun_out/ab/$mode$i.err; exit 1; }
    python3 -c "
import json,sys
l=json.loads(open('gpurun_out/ab/$mode$i.json').read().strip().splitlines()[-1])
print('$mode$i', l['ms_per_step'], l['fold']['ms'], l['checks'])"
  done
done
