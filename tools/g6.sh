set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
c3() { CE_C3_NO_NAMES=1 timeout -k 10 300 python -u bench_configs.py --config c3 --no-cpu > gpurun_out/c3_$1.json 2> gpurun_out/c3_$1.err; }
c3 auto && CE_DMA_ENGINE=0 c3 e0 && CE_DMA_ENGINE=1 c3 e1 && CE_DMA_OFF=1 c3 off && python3 - <<'PY'
import json
for v in ("auto", "e0", "e1", "off"):
    d = json.load(open("gpurun_out/c3_%s.json" % v))
    print(v, d["ms_per_step"], d["pipelined"]["download_engine"], d["phases_ms_per_step"], d["kernels_ms_per_step"].get("ds_add_pairs"))
PY
