#!/bin/bash
# Same-box A/B of library builds on the default bench (no CPU leg), twice each:
#   LIBS="crdt-enc_amd/libcrdtenc_ab.so crdt-enc_amd/libcrdtenc.so" tools/lib_ab.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  for L in ${LIBS}; do
    echo -n "$L "
    CRDTENC_LIB=$PWD/$L timeout -k 10 200 python bench.py --configs '' --no-cpu --no-host-buffers ${BENCH_ARGS:-} 2> gpurun_out/libab.err | python3 -c "
import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);b=d.get('variant_b') or {}
print(d['ms_per_step'],d['roofline']['avg_launch_ms'],'B',b.get('ms_per_step'),b.get('avg_launch_ms'))" || { tail -3 gpurun_out/libab.err; exit 1; }
  done
done
