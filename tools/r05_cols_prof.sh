#!/bin/bash
# the C3 column exchange (tools/cols_bench.py) timed, then under rocprofv3 --kernel-trace --stats
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
CE_HOST_PROF=1 timeout -k 10 300 python3 -u tools/cols_bench.py > gpurun_out/cols_bench.log 2>&1 || { tail -30 gpurun_out/cols_bench.log; exit 1; }
tail -1 gpurun_out/cols_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/colsprof -o run -- python3 -u tools/cols_bench.py > gpurun_out/colsprof.log 2>&1 || { tail -30 gpurun_out/colsprof.log; exit 1; }
f=$(find gpurun_out/colsprof -name "run_kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:45]:
    print("%-60s %6s %10.1f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
