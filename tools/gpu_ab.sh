#!/bin/bash
# A/B of host-side knobs on the default bench (no CPU leg): one line per run
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { echo -n "$1 "; env ${1//,/ } timeout -k 10 200 python bench.py --no-cpu 2> gpurun_out/ab.err | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'],d['roofline']['avg_launch_ms'],d['kernels_ms_per_step'].get('open_setup'))" || { tail -3 gpurun_out/ab.err; exit 1; }; }
for v in ${AB:-"X=0" "CE_SPIN=1" "X=0" "CE_SPIN=1" "CE_HOST_COMPACT=1"}; do run $v || exit 1; done
