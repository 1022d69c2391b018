#!/bin/bash
# Round-3 evidence in one call, everything under gpurun_out/r03 (copied into profiles/ here):
# the GPU suite, the default bench line (C2 + variant B + host buffers + CPU baseline + C3/C4/C5),
# rocprofv3 kernel-trace stats of the C2 bench and its FETCH/WRITE traffic passes, the VALU PMC
# passes.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r03
mkdir -p $O
export PROFILE_DIR=$O PROFILE_TAG=r03
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" $O/gpu_tests.log | head -60; exit $rc; }
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
print('C2', d.get('value'), d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('state_check'))
for k,v in (d.get('configs') or {}).items(): print(k, v.get('ms_per_step'), v.get('value'), v.get('checks'))"
if [ -z "$NO_ROCPROF" ]; then
  ./tools/rocprof.sh > $O/rocprof.log 2>&1 || { echo "rocprof failed"; tail -5 $O/rocprof.log; exit 1; }
  grep -E "k_open_fold|k_open_setup|fetch_bytes" $O/rocprof.log | head -5
  bash tools/pmc_valu.sh > $O/pmc_valu.log 2>&1 || { echo "pmc_valu failed"; tail -5 $O/pmc_valu.log; exit 1; }
  echo "pmc ok"
  rm -rf gpurun_out/rocprof/trace gpurun_out/rocprof/FETCH_SIZE gpurun_out/rocprof/WRITE_SIZE gpurun_out/pmc_valu/pass*
fi
