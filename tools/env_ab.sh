#!/bin/bash
# Same-box A/B of one env knob on the default C2 bench line (no CPU leg), twice each:
#   KNOB=CE_V3 VALS="0 1 2 3" tools/env_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for V in ${VALS}; do
    echo -n "$KNOB=$V "
    env $KNOB=$V timeout -k 10 200 python bench.py --configs '' --no-cpu --no-host-buffers ${BENCH_ARGS:-} 2> gpurun_out/envab.err | python3 -c "
import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);b=d.get('variant_b') or {}
print(d['ms_per_step'],d['roofline']['avg_launch_ms'],'B',b.get('ms_per_step'),b.get('avg_launch_ms'))" || { tail -3 gpurun_out/envab.err; exit 1; }
  done
done
