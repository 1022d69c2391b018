#!/bin/bash
# Round evidence in one GPU call: GPU tests, the default bench (CPU leg included), rocprofv3
# kernel-trace stats + FETCH_SIZE/WRITE_SIZE passes (tools/rocprof.sh), the VALU PMC passes
# (tools/pmc_valu.sh), then C3/C4/C5.  Summaries are made afterwards, off the box:
#   PROFILE_TAG=r02 python tools/summarize_profiles.py gpurun_out/rocprof
#   PROFILE_TAG=r02 python tools/summarize_valu.py gpurun_out/pmc_valu
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail gpurun_out/bench.err; exit 1; }
echo "bench ok"
bash tools/rocprof.sh > gpurun_out/rocprof.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/rocprof.log; exit 1; }
echo "rocprof ok"
cd $GRAFT_REPO_ROOT
bash tools/pmc_valu.sh > gpurun_out/pmc_valu.log 2>&1 || { echo "pmc_valu failed"; tail -5 gpurun_out/pmc_valu.log; exit 1; }
echo "pmc_valu ok"
cd $GRAFT_REPO_ROOT
for c in c3 c4 c5; do
  timeout -k 10 300 python bench_configs.py --config $c > gpurun_out/$c.json 2> gpurun_out/$c.err || { echo "$c failed"; tail -3 gpurun_out/$c.err; exit 1; }
  echo "$c ok"
done
