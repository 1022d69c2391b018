cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 170 python -u tools/c3r_debug.py > gpurun_out/c3r_debug.log 2>&1; echo rc=$?; cat gpurun_out/c3r_debug.log
