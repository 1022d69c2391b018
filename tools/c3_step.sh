#!/bin/bash
# One C3 step's GPU timeline: rocprofv3 kernel + copy trace of a short bench_configs.py --config c3
# run, then tools/c3_step_breakdown.py (every GPU op of one timed step, idle gaps, totals).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c3s
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CE_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --marker-trace --output-format csv -d $O/t -o s -- \
  python3 $R/bench_configs.py --config c3 --steps 10 --no-cpu > $O/c3t.json 2> $O/c3t.err || { echo "trace rc=$?"; tail -5 $O/c3t.err; exit 1; }
python3 $R/tools/c3_step_breakdown.py $O/t > $O/c3_step.txt || { echo "breakdown failed"; exit 1; }
grep -A 30 "step span" $O/c3_step.txt
rm -rf $O/t
