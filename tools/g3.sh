set -o pipefail
cd $GRAFT_REPO_ROOT
CE_BENCH_SHARE_GPU=1 CE_DIST_BACKEND=gloo timeout -k 10 500 python -u bench.py --gpus 2 --steps 5 --warmup 1 --no-cpu --no-variant-b > gpurun_out/b2.json 2> gpurun_out/b2.err
