set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_multi.py "tests/test_gpu_dotset.py::test_state_bytes_and_merge_device" > gpurun_out/g1.log 2>&1
