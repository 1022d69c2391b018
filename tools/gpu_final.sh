#!/bin/bash
# Round-end evidence in one call: tools/gpu_round.sh (tests, bench with the CPU leg, rocprof
# stats + PMC traffic, C3), then the VALU PMC passes and the C4/C5 benches.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_round.sh || exit 1
cd $GRAFT_REPO_ROOT
bash tools/pmc_valu.sh > gpurun_out/pmc_valu.log 2>&1 || { echo "pmc_valu failed"; tail -5 gpurun_out/pmc_valu.log; exit 1; }
echo "pmc_valu ok"
timeout -k 10 200 python bench_configs.py --config c3 > gpurun_out/c3_clean.json 2> gpurun_out/c3_clean.err || { echo c3 failed; exit 1; }
timeout -k 10 200 python bench_configs.py --config c4 > gpurun_out/c4.json 2> gpurun_out/c4.err || { echo c4 failed; exit 1; }
timeout -k 10 200 python bench_configs.py --config c5 > gpurun_out/c5.json 2> gpurun_out/c5.err || { echo c5 failed; exit 1; }
cat gpurun_out/c3_clean.json gpurun_out/c4.json gpurun_out/c5.json
