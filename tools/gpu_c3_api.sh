#!/bin/bash
# C3 host + GPU view of one step: HIP API calls beside the kernel + copy trace
# (tools/c2_api_breakdown.py with the step marked by every other k_open_setup: states, ops).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r03
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d $O/c3a -o s -- \
  python3 $R/bench_configs.py --config c3 --steps 4 --warmup 1 --no-cpu > $O/c3a.json 2> $O/c3a.err || { echo "trace rc=$?"; tail -5 $O/c3a.err; exit 1; }
python3 $R/tools/c2_api_breakdown.py $O/c3a 2 ce::k_rdm_count > $O/c3_api.txt || { echo "breakdown failed"; exit 1; }
tail -25 $O/c3_api.txt
rm -rf $O/c3a
