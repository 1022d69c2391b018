#!/bin/bash
# Same-box A/B of library builds on the C3 bench (no CPU leg), alternating:
#   LIBS="crdt-enc_amd/libcrdtenc_base.so crdt-enc_amd/libcrdtenc.so" tools/c3_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for L in ${LIBS}; do
  echo -n "$L "
  CRDTENC_LIB=$PWD/$L timeout -k 10 300 python bench_configs.py --config c3 --steps ${C3_STEPS:-20} --no-cpu 2> gpurun_out/c3ab.err | python3 -c "
import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print(d['ms_per_step'], d.get('pipelined',{}).get('ms_per_step'), d['phases_ms_per_step'], d['checks'])" || { tail -3 gpurun_out/c3ab.err; exit 1; }
done
