#!/bin/bash
# Shader clock beside the C2 fused kernel with parts of it switched off (diagnostics build,
# CE_ABLATE bits: 1 no decode, 2 no Poly1305 products, 4 no ChaCha20, 8 no ciphertext loads;
# results invalid, the bench's check fails and is ignored here): which part draws the power?
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for ab in ${ABL:-0 1 2 4 8}; do
  CRDTENC_LIB=$GRAFT_REPO_ROOT/crdt-enc_amd/libcrdtenc_prof.so CE_ABLATE=$ab timeout -k 10 200 \
    python tools/clock_ablate.py > gpurun_out/clk_$ab.json 2> gpurun_out/clk_$ab.err
  rc=$?
  [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -ge 128 ] && { echo "bench died rc=$rc"; tail -3 gpurun_out/clk_$ab.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/clk_$ab.json').read());r=d['roofline']
print('ablate $ab', r['avg_launch_ms'], r['clock']['under_step'], r['clock']['idle']['median_ghz'])" || { tail -3 gpurun_out/clk_$ab.err; exit 1; }
done
