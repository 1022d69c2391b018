#!/bin/bash
# round 6: the whole -m gpu suite in one process (as the driver runs it), then smoke()
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/full_gpu.log 2>&1 || { grep -E "FAILED|Error|error" gpurun_out/full_gpu.log | head -20; tail -30 gpurun_out/full_gpu.log; exit 1; }
tail -2 gpurun_out/full_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
