#!/bin/bash
# per-phase cycles of k_open_fold_v2 (CE_PROF, diagnostics build), 1M files; OPTS = CE_V2_OPT values
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for o in ${OPTS:-1}; do
  CRDTENC_LIB=$GRAFT_REPO_ROOT/crdt-enc_amd/libcrdtenc_prof.so CE_PROF=1 CE_V2_OPT=$o timeout -k 10 120 python -u bench.py --configs '' --steps 1 --warmup 1 --no-cpu --no-variant-b --no-host-buffers > gpurun_out/profv2_$o.json 2> gpurun_out/profv2_$o.err || { echo "prof $o failed"; tail -5 gpurun_out/profv2_$o.err; exit 1; }
  echo "opt $o"; grep CE_PROF gpurun_out/profv2_$o.err | tail -1
done
