#!/bin/bash
# Same-box A/B of env knobs (tools/gpu_ab.sh), then the GPU parity tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AB="${AB}" BENCH_ARGS="${BENCH_ARGS:---no-variant-b --no-host-buffers}" ./tools/gpu_ab.sh || exit 1
[ -n "$NO_TESTS" ] && exit 0
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_all.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_all.log; exit $rc
