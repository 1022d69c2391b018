#!/bin/bash
# kernel + copy trace of a short C3 run; one step's timeline (tools/timeline_c3.py)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/c3trace
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $OUT/t -o s -- \
  python3 $R/bench_configs.py --config c3 --steps 4 --no-cpu > $OUT/out.json 2> $OUT/err.txt || { echo "trace rc=$?"; tail -5 $OUT/err.txt; exit 1; }
python3 $R/tools/timeline_c3.py $OUT/t > $OUT/timeline.txt
tail -3 $OUT/timeline.txt
