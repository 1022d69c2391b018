cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_dotset.py -k "table_growth" tests/test_gpu_configs.py 2>&1 | tee gpurun_out/t_growth.log | tail -5
timeout -k 10 170 python -u tools/c3r_debug.py > gpurun_out/c3r_debug.log 2>&1; echo rc=$?; tail -2 gpurun_out/c3r_debug.log
