#!/bin/bash
# Kernel + copy trace of a short default bench run (one step's timeline: tools/timeline.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/steptrace
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/t -o s -- \
  python3 $R/bench.py --configs '' --steps 4 --warmup 1 --no-cpu --no-variant-b --no-host-buffers --no-clock > $OUT/out.json 2> $OUT/err.txt || { echo "trace rc=$?"; tail -5 $OUT/err.txt; exit 1; }
python3 $R/tools/timeline.py $OUT/t
