#!/bin/bash
# One rocprofv3 --pmc pass (at most 8 SQ counters) over a short C3 run; per-kernel medians of
# every counter for the kernels matching $KERN (default: the partitioned fold) ->
# gpurun_out/c3pmc/pmc.json.   PMC="SQ_WAVES SQ_BUSY_CYCLES" KERN="k_ds_part" tools/c3_pmc.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/c3pmc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc ${PMC:-SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS} \
  --output-format csv -d $O/p -o p -- python3 $R/bench_configs.py --config c3 --steps 2 --warmup 1 --no-cpu \
  > $O/p.out 2> $O/p.err || { echo "pmc rc=$?"; tail -5 $O/p.err; exit 1; }
python3 - $O "${KERN:-k_ds_part}" <<'PY'
import csv, glob, json, re, sys
o, pat = sys.argv[1], sys.argv[2]
per = {}
for fn in glob.glob(o + "/p/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        m = re.search(r"(k_\w+)", row["Kernel_Name"])
        if not m or pat not in m.group(1):
            continue
        d = per.setdefault(m.group(1), {}).setdefault(row["Counter_Name"], {})
        d[row["Dispatch_Id"]] = d.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
res = {k: {c: sorted(v.values())[len(v) // 2] for c, v in cs.items()} for k, cs in per.items()}
json.dump(res, open(o + "/pmc.json", "w"), indent=1)
for k, cs in res.items():
    print(k, {c: round(v) for c, v in cs.items()})
PY
rm -rf $O/p
