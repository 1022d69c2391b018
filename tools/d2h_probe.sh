set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "PROBE_TAG=default" "HSA_ENABLE_SDMA=1,PROBE_TAG=sdma1" "GPU_BLIT_ENGINE_TYPE=1,PROBE_TAG=blit1" "DEBUG_CLR_LIMIT_BLIT_WG=16,PROBE_TAG=limwg16" "HSA_ENABLE_SDMA_GANG=0,PROBE_TAG=nogang"; do
  env ${v//,/ } timeout -k 10 120 python -u tools/d2h_torch_probe.py >> gpurun_out/d2h_probe.txt 2>&1 || { echo "probe $v failed"; exit 1; }
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/dp -o s -- python3 $GRAFT_REPO_ROOT/tools/d2h_torch_probe.py > /dev/null 2>&1
grep -c copyBuffer /tmp/dp/*kernel_trace.csv >> $GRAFT_REPO_ROOT/gpurun_out/d2h_probe.txt; wc -l /tmp/dp/*memory_copy_trace.csv >> $GRAFT_REPO_ROOT/gpurun_out/d2h_probe.txt || true
