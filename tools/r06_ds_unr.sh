#!/bin/bash
# round 6: the DS open form with a rolled ChaCha20 loop -- DS tests, then C3 kernel stats A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
CRDTENC_LIB=$PWD/crdt-enc_amd/libcrdtenc_${TLIB:-ds1}.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_dotset.py -k "fused_decode or fast_path or full_size or tiled" > gpurun_out/ds_tests.log 2>&1 || { tail -30 gpurun_out/ds_tests.log; exit 1; }
tail -1 gpurun_out/ds_tests.log
for r in 1 2; do for v in ${VARS:-ds9 ds1}; do
  bash tools/c3_kstats.sh ${v}_$r CRDTENC_LIB=$PWD/crdt-enc_amd/libcrdtenc_$v.so | grep -E "total|k_open_fold|open_setup" || exit 1
done; done
