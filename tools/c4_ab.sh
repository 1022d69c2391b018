#!/bin/bash
# Same-box A/B of two library builds on C4: prints ms/step and the kernel split per run.
#   LIBS="crdt-enc_amd/libcrdtenc_ab.so crdt-enc_amd/libcrdtenc.so" tools/c4_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for L in ${LIBS}; do
    echo -n "$L "
    CRDTENC_LIB=$PWD/$L timeout -k 10 200 python bench_configs.py --config ${CFG:-c4} 2> gpurun_out/c4ab.err | python3 -c "
import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print(d['ms_per_step'], d['kernels_ms_per_step'])" || { tail -3 gpurun_out/c4ab.err; exit 1; }
  done
done
