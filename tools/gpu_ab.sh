#!/bin/bash
# Same-box A/B of env knobs on the default bench (no CPU leg): one line per run.  A run whose
# result check fails (diagnostic variants) still prints its times, marked CHECK-FAILED.
#   AB="CE_V2_OPT=1 CE_V2_OPT=3" BENCH_ARGS="--no-variant-b" tools/gpu_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {
  echo -n "$1 "
  env ${1//,/ } timeout -k 10 200 python bench.py --configs '' --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab.json 2> gpurun_out/ab.err
  local rc=$?
  [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ] && { echo "bench died rc=$rc"; tail -3 gpurun_out/ab.err; return 1; }
  python3 -c "
import json,sys;d=json.loads(open('gpurun_out/ab.json').read());b=d.get('variant_b') or {}
print(d['ms_per_step'],d['roofline']['avg_launch_ms'],d['kernels_ms_per_step'].get('open_setup'),'B',b.get('avg_launch_ms'),'' if $rc == 0 else 'CHECK-FAILED')" || { tail -3 gpurun_out/ab.err; return 1; }
}
for v in ${AB:-"X=0" "CE_SPIN=1"}; do run $v || exit 1; done
