#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of the default bench command, then the
# HBM traffic passes (FETCH_SIZE, WRITE_SIZE in separate runs) on the same 1M-file workload.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/rocprof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- \
  python3 $R/bench.py --configs '' --steps 5 --warmup 1 --no-cpu --no-variant-b --no-host-buffers --no-clock > $OUT/trace.out 2> $OUT/trace.err || { echo "trace rc=$?"; tail -5 $OUT/trace.err; exit 1; }
echo "trace ok"; cat $OUT/trace.out
for P in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $OUT/$P -o p -- \
    python3 $R/bench.py --configs '' --steps 2 --warmup 1 --no-cpu --no-variant-b --no-host-buffers --no-clock > $OUT/$P.out 2> $OUT/$P.err || { echo "pmc $P rc=$?"; tail -5 $OUT/$P.err; exit 1; }
  echo "pmc $P ok"
done
python3 $R/tools/summarize_profiles.py $OUT
