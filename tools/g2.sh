set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -v --timeout 450 --timeout-method thread "tests/test_gpu_multi.py::test_bench_two_ranks_share_gpu" > gpurun_out/g2.log 2>&1
