set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 900 python -u bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { echo "bench rc=$?"; tail -5 gpurun_out/bench_full.err; exit 1; }
tail -1 gpurun_out/bench_full.json | head -c 600; echo
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof -o b -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --no-cpu --configs '' --no-variant-b --no-host-buffers > $GRAFT_REPO_ROOT/gpurun_out/prof/bench_prof.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof/bench_prof.err || { echo "prof rc=$?"; exit 1; }
ls $GRAFT_REPO_ROOT/gpurun_out/prof
