set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu"
timeout -k 10 900 $T tests/test_gpu_dotset.py tests/test_gpu_parity.py tests/test_gpu_segdec.py 2>&1 | tee gpurun_out/t_ds.log | tail -15
