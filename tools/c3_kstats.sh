#!/bin/bash
# Per-kernel averages of a short C3 run (rocprofv3 --kernel-trace --stats), for same-box A/Bs of
# env knobs: tools/c3_kstats.sh <tag> [VAR=value ...]  -> gpurun_out/c3k_<tag>.csv (+ a summary)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; shift
O=$R/gpurun_out/c3k_$T
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
env "$@" CE_C3_NO_NAMES=1 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o k -- \
  python3 $R/bench_configs.py --config c3 --steps 20 --warmup 2 --no-cpu --no-clock > $O/out.json 2> $O/err.txt || { echo "rc=$?"; tail -5 $O/err.txt; exit 1; }
f=$(find $O -name "*kernel_stats.csv" | head -1)
cp $f $R/gpurun_out/c3k_$T.csv
python3 - $f $T <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(sys.argv[2], "total kernel ms per call-set: %.1f" % (tot / 1e6))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:14]:
    print("  %8.1f us x%4s  %s" % (float(r["AverageNs"]) / 1e3, r["Calls"], r["Name"][:90]))
PY
