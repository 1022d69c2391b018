set -o pipefail
cd $GRAFT_REPO_ROOT
CE_C3_NO_NAMES=1 bash tools/c3_step.sh > /dev/null && CE_C3_NO_NAMES=1 bash tools/c3_host.sh > /dev/null && CE_C3_NO_NAMES=1 bash tools/c3_traffic.sh > /dev/null && \
timeout -k 10 300 python -u bench_configs.py --config c3 > gpurun_out/c3_full.json 2> gpurun_out/c3_full.err && echo done
