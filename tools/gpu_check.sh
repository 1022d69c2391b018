#!/bin/bash
# GPU parity tests, then the fused-kernel phase profile and the files-per-wave sweep
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
./tools/prof.sh && ./tools/sweep_fpw.sh
