#!/bin/bash
# Same-box A/B of env knobs on the default bench (no CPU leg): one line per run.
#   AB="CE_V2_OPT=1 CE_V2_OPT=3" BENCH_ARGS="--no-variant-b" tools/gpu_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { echo -n "$1 "; env ${1//,/ } timeout -k 10 200 python bench.py --no-cpu ${BENCH_ARGS:-} 2> gpurun_out/ab.err | python3 -c "
import json,sys;d=json.loads(sys.stdin.read());b=d.get('variant_b') or {}
print(d['ms_per_step'],d['roofline']['avg_launch_ms'],d['kernels_ms_per_step'].get('open_setup'),'B',b.get('avg_launch_ms'))" || { tail -3 gpurun_out/ab.err; exit 1; }; }
for v in ${AB:-"X=0" "CE_SPIN=1"}; do run $v || exit 1; done
