#!/bin/bash
# The C3 half of tools/evidence.sh: the C3 line with its CPU baseline, the line without the names,
# and the step traces (GPU timeline, host calls, traffic).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ev
timeout -k 10 300 python -u bench_configs.py --config c3 > gpurun_out/ev/c3.json 2> gpurun_out/ev/c3.err || { echo "c3 failed"; exit 1; }
CE_C3_NO_NAMES=1 timeout -k 10 300 python -u bench_configs.py --config c3 --no-cpu > gpurun_out/ev/c3_no_names.json 2> gpurun_out/ev/c3nn.err || { echo "c3nn failed"; exit 1; }
CE_C3_NO_NAMES=1 bash tools/c3_step.sh > /dev/null && CE_C3_NO_NAMES=1 bash tools/c3_host.sh > /dev/null && CE_C3_NO_NAMES=1 bash tools/c3_traffic.sh > /dev/null && echo evidence done
