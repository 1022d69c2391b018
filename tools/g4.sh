set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread "tests/test_gpu_dotset.py::test_ingest_states_device_matches_host" "tests/test_gpu_dotset.py::test_c3_shaped_medium" > gpurun_out/g4.log 2>&1 && \
timeout -k 10 300 python -u bench_configs.py --config c3 --no-cpu > gpurun_out/c3.json 2> gpurun_out/c3.err
