#!/bin/bash
# Quick GPU check: parity tests, the default bench, a kernel-trace of a short bench run.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --configs '' ${BENCH_ARGS:---no-cpu} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/qtrace -o q -- \
  python3 $GRAFT_REPO_ROOT/bench.py --configs '' --steps 3 --warmup 1 --no-cpu > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/qtrace.err || { echo "trace failed"; exit 1; }
echo trace ok
