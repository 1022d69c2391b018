#!/bin/bash
# Same-box A/B of C2 env knobs, alternating, 40 steps each: ms/step, fused avg launch, step - fused.
#   AB="CE_GATE_DMA=1 X=0" tools/c2_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for v in ${AB:-"CE_GATE_DMA=1 X=0"}; do
    echo -n "$v "
    env ${v//,/ } timeout -k 10 200 python bench.py --configs '' --no-cpu --no-variant-b --no-host-buffers --no-clock --steps 40 > gpurun_out/c2ab.json 2> gpurun_out/c2ab.err || { echo "bench failed"; tail -3 gpurun_out/c2ab.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/c2ab.json').read().strip().splitlines()[-1]);a=d['roofline']['avg_launch_ms']
print(d['ms_per_step'], a, round(d['ms_per_step']-a,4), d['kernels_ms_per_step'])"
  done
done
