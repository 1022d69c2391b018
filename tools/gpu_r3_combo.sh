#!/bin/bash
# parity subset, same-box A/B of the product library against libcrdtenc_base.so (C2 + variant B),
# then the C3 evidence (trace + fold traffic)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "parity or segdec or configs or template" > gpurun_out/gpu_sub.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 gpurun_out/gpu_sub.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/gpu_sub.log | head -60; exit $rc; }
LIBS="crdt-enc_amd/libcrdtenc_base.so crdt-enc_amd/libcrdtenc.so" BENCH_ARGS="--no-clock" ./tools/lib_ab.sh || exit 1
./tools/gpu_c3_evidence.sh
