set -o pipefail
# C3 iteration on the GPU box: dot-set tests, the C3 line with and without the content names, one traced step
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_dotset.py > gpurun_out/g5.log 2>&1 && \
CE_C3_NO_NAMES=1 timeout -k 10 300 python -u bench_configs.py --config c3 --no-cpu > gpurun_out/c3_nn.json 2> gpurun_out/c3_nn.err && \
timeout -k 10 300 python -u bench_configs.py --config c3 --no-cpu > gpurun_out/c3_names.json 2> gpurun_out/c3_names.err && \
CE_C3_NO_NAMES=1 bash tools/c3_step.sh > /dev/null && python3 - <<'PY'
import json
for v in ("nn", "names"):
    d = json.load(open("gpurun_out/c3_%s.json" % v))
    print(v, d["ms_per_step"], d["pipelined"]["ms_per_step"], d["pipelined"]["name_drain_ms"], d["phases_ms_per_step"])
PY
