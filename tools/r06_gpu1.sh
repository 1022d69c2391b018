set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu"
timeout -k 10 300 $T tests/test_gpu_dotset.py -k "columns" > gpurun_out/t_cols.log 2>&1; tail -3 gpurun_out/t_cols.log
timeout -k 10 600 $T tests/test_gpu_multi.py tests/test_gpu_nccl.py > gpurun_out/t_multi.log 2>&1; tail -3 gpurun_out/t_multi.log
for v in 1 3; do CE_V3=$v timeout -k 10 300 $T tests/test_gpu_parity.py > gpurun_out/t$v.log 2>&1 || { tail -20 gpurun_out/t$v.log; exit 1; }; tail -1 gpurun_out/t$v.log; done
KNOB=CE_V3 VALS="0 1 2 3" bash tools/env_ab.sh
