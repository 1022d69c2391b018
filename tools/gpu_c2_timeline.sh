#!/bin/bash
# C2 one-step timeline under gpurun_out/c2t: a kernel + copy trace of a short variant-A bench run
# and tools/c2_step_breakdown.py over one timed step (GPU busy, idle gaps, step - fused).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c2t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/c2t -o s -- \
  python3 $R/bench.py --steps 6 --warmup 2 --configs '' --no-cpu --no-host-buffers --no-variant-b --no-clock \
  > $O/c2t.json 2> $O/c2t.err || { echo "trace rc=$?"; tail -5 $O/c2t.err; exit 1; }
python3 $R/tools/c2_step_breakdown.py $O/c2t > $O/c2_step.txt || { echo "breakdown failed"; exit 1; }
cat $O/c2_step.txt
