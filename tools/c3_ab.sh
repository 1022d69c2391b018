#!/bin/bash
# Same-box A/B of C3 env knobs without the names, alternating, twice: ms/step and phases.
#   AB="CE_HIPCUB_SCAN=1 X=0" tools/c3_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for v in ${AB:-CE_HIPCUB_SCAN=1 X=0}; do
    echo -n "$v "
    env CE_C3_NO_NAMES=1 ${v//,/ } timeout -k 10 300 python bench_configs.py --config c3 --no-cpu > gpurun_out/c3ab.json 2> gpurun_out/c3ab.err || { echo failed; tail -3 gpurun_out/c3ab.err; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/c3ab.json'));print(d['ms_per_step'], d['phases_ms_per_step'])"
  done
done
