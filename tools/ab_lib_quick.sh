#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "parity or template" > gpurun_out/gpu_sub.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/gpu_sub.log; [ $rc -eq 0 ] || exit $rc
LIBS="crdt-enc_amd/libcrdtenc_base.so crdt-enc_amd/libcrdtenc.so" BENCH_ARGS="--no-clock" ./tools/lib_ab.sh
