#!/bin/bash
# per-phase cycles of the fused kernel (CE_PROF), 256K files, fpw 4/2/1
for f in 4 2 1; do
  CRDTENC_LIB=$GRAFT_REPO_ROOT/crdt-enc_amd/libcrdtenc_prof.so CE_PROF=1 CE_FILES_PER_WAVE=$f timeout -k 10 120 python -u bench.py --configs '' --versions 64 --steps 1 --warmup 0 --no-cpu > /dev/null 2> gpurun_out/prof_$f.err || { echo "prof $f failed"; tail -5 gpurun_out/prof_$f.err; exit 1; }
  echo "fpw $f"; grep CE_PROF gpurun_out/prof_$f.err | tail -1
done
