#!/bin/bash
# One C3 step's host timeline: rocprofv3 HIP API + kernel trace of a short C3 run, then
# tools/c3_host_trace.py (HIP calls of the launching thread, host time between them).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c3h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CE_ROCTX=1 timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --marker-trace --output-format csv -d $O/t -o s -- \
  python3 $R/bench_configs.py --config c3 --steps 10 --no-cpu > $O/c3t.json 2> $O/c3t.err || { echo "trace rc=$?"; tail -5 $O/c3t.err; exit 1; }
python3 $R/tools/c3_host_trace.py $O/t > $O/c3_host.txt || { echo "host breakdown failed"; exit 1; }
tail -30 $O/c3_host.txt
rm -rf $O/t
