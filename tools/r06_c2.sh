#!/bin/bash
# Round 6: the C2 fused kernel -- parity tests, then a same-box A/B of library builds (LIBS) on
# the default C2 bench line (no CPU leg), twice each.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py ${EXTRA_TESTS:-} > gpurun_out/r06_c2_tests.log 2>&1 || { tail -30 gpurun_out/r06_c2_tests.log; exit 1; }
tail -2 gpurun_out/r06_c2_tests.log
LIBS="${LIBS:-crdt-enc_amd/libcrdtenc_base.so crdt-enc_amd/libcrdtenc.so}" bash tools/lib_ab.sh
