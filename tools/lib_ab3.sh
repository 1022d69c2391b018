#!/bin/bash
# Same-box A/B of two library builds on the C2 bench, 3 rounds of 40 steps each, alternating:
#   A=crdt-enc_amd/libcrdtenc_base.so B=crdt-enc_amd/libcrdtenc.so tools/lib_ab3.sh
cd $GRAFT_REPO_ROOT
for r in 1 2 3; do
  for L in $A $B; do
    echo -n "$L "
    CRDTENC_LIB=$PWD/$L timeout -k 10 200 python bench.py --configs '' --no-cpu --no-host-buffers --no-variant-b --no-clock --steps 40 2>/dev/null | python3 -c "
import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);print(d['ms_per_step'],d['roofline']['avg_launch_ms'],d['state_check'])" || exit 1
  done
done
