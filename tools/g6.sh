set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
c3() { timeout -k 10 300 python -u bench_configs.py --config c3 --no-cpu > gpurun_out/c3_$1.json 2> gpurun_out/c3_$1.err; }
AB="CE_GATE_AFTER_SETUP=1 X=0 CE_GATE_AFTER_SETUP=1 X=0" BENCH_ARGS="--no-variant-b --no-host-buffers --steps 40 --no-clock" bash tools/gpu_ab.sh > gpurun_out/ab_gate.txt 2>&1 && \
CE_C3_NO_NAMES=1 c3 nn && CE_C3_NO_NAMES=1 CE_ASYNC_BLIT=1 c3 nnblit && CE_C3_NO_NAMES=1 CE_C3_SYNC_COMPACT=1 c3 nnsync && c3 names && \
CE_C3_NO_NAMES=1 bash tools/c3_step.sh
