#!/bin/bash
# C2 host-side view of one step: HIP API calls (rocprofv3 --hip-runtime-trace) beside the
# kernel + copy trace, merged by tools/c2_api_breakdown.py into one timeline (host call spans
# and GPU operations on one clock).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $O/c2a -o s -- \
  python3 $R/bench.py --steps 6 --warmup 2 --configs '' --no-cpu --no-host-buffers --no-variant-b --no-clock \
  > $O/c2a.json 2> $O/c2a.err || { echo "trace rc=$?"; tail -5 $O/c2a.err; exit 1; }
python3 $R/tools/c2_api_breakdown.py $O/c2a > $O/c2_api.txt || { echo "breakdown failed"; exit 1; }
tail -60 $O/c2_api.txt
rm -rf $O/c2a
