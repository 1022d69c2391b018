#!/bin/bash
# bench the fused kernel geometry: 4, 2, 1 files per wavefront
mkdir -p gpurun_out
for f in 4 2 1; do
  CE_FILES_PER_WAVE=$f timeout -k 10 300 python -u bench.py --configs '' --no-cpu --steps 10 > gpurun_out/fpw_$f.json 2> gpurun_out/fpw_$f.err || exit 1
  python - "$f" <<'PY'
import json, sys
d = json.load(open("gpurun_out/fpw_%s.json" % sys.argv[1]))
print("fpw", sys.argv[1], "ms", d["ms_per_step"], "files/s %.3g" % d["value"], "hbm", d["roofline"]["achieved"],
      "valu_frac", d["roofline"]["valu"]["frac"], d["state_check"])
print("   ", d["kernels_ms_per_step"])
PY
done
