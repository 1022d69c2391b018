#!/bin/bash
# C3 with the content names: A/B of the naming scheme (CE_NAME_BATCH=k multi-buffer batches,
# CE_NAME_THREADS), one run each: ms/step (with the drain), pipelined, drain.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in ${AB:-X=0 CE_NAME_BATCH=2 CE_NAME_BATCH=4 CE_NAME_BATCH=8}; do
  echo -n "$v "
  env ${v//,/ } timeout -k 10 300 python bench_configs.py --config c3 --no-cpu > gpurun_out/c3n.json 2> gpurun_out/c3n.err || { echo failed; tail -3 gpurun_out/c3n.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/c3n.json'));p=d['pipelined'];print(d['ms_per_step'], p['ms_per_step'], p['name_drain_ms'])"
done
