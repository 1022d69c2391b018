#!/bin/bash
for b in ${ABL_BITS:-0 1 2 4 8 3 7 15}; do
  CRDTENC_LIB=$GRAFT_REPO_ROOT/crdt-enc_amd/libcrdtenc_prof.so CE_ABLATE=$b timeout -k 10 120 python -u tools/ablate.py > gpurun_out/abl_$b.json 2>gpurun_out/abl_$b.err || { echo "ablate $b failed"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/abl_$b.json')); print('ablate', $b, 'fold_small ms', d['kernels_ms_per_step'].get('open_fold_small'))"
done
