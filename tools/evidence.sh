#!/bin/bash
# Round evidence on one box: the default bench line, rocprofv3 kernel stats of the C2 step, the C3
# line with its CPU baseline, and the C3 step traces (GPU timeline, host calls, traffic).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ev
timeout -k 10 900 python -u bench.py > gpurun_out/ev/bench.json 2> gpurun_out/ev/bench.err || { echo "bench rc=$?"; tail -5 gpurun_out/ev/bench.err; exit 1; }
tail -1 gpurun_out/ev/bench.json | head -c 300; echo
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ev/prof -o b -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --no-cpu --configs '' --no-variant-b --no-host-buffers > $GRAFT_REPO_ROOT/gpurun_out/ev/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/ev/bench_prof.err) || { echo "prof failed"; exit 1; }
timeout -k 10 300 python -u bench_configs.py --config c3 > gpurun_out/ev/c3.json 2> gpurun_out/ev/c3.err || { echo "c3 failed"; exit 1; }
CE_C3_NO_NAMES=1 timeout -k 10 300 python -u bench_configs.py --config c3 --no-cpu > gpurun_out/ev/c3_no_names.json 2> gpurun_out/ev/c3nn.err || { echo "c3nn failed"; exit 1; }
CE_C3_NO_NAMES=1 bash tools/c3_step.sh > /dev/null && CE_C3_NO_NAMES=1 bash tools/c3_host.sh > /dev/null && CE_C3_NO_NAMES=1 bash tools/c3_traffic.sh > /dev/null && echo evidence done
