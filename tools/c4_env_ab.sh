#!/bin/bash
# Same-box A/B of env settings on C4, twice each:  AB="CE_SEG2=0 CE_SEG2=1" tools/c4_env_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for v in ${AB}; do
    echo -n "$v "
    env ${v//,/ } timeout -k 10 200 python bench_configs.py --config ${CFG:-c4} --no-cpu 2> gpurun_out/c4ab.err | python3 -c "
import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print(d['ms_per_step'], d['kernels_ms_per_step'], d.get('decode_paths'), d['checks'])" || { tail -3 gpurun_out/c4ab.err; exit 1; }
  done
done
