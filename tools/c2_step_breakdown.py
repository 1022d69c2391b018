#!/usr/bin/env python3
"""One C2 step (bench.py variant A: ingest 1M op files + compact) from a rocprofv3 kernel + copy
trace: every GPU operation from the step's k_fill (the ingest's first launch) up to the next
step's, the idle gaps between them, and totals per category.  The step ends where the next one
begins, so the host time between two steps (bench loop, Python binding) is the last gap.

  tools/c2_step_breakdown.py <rocprofv3 output dir> [step index among the k_fill launches]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
rows = []
for fn in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
              r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-44:])
             for r in csv.DictReader(open(fn))]
for fn in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "DMA " + r.get("Direction", "")[-14:])
             for r in csv.DictReader(open(fn))]
rows.sort()
fills = [i for i, r in enumerate(rows) if "ce::k_fill" in r[2]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(fills) - 2
s0, s1 = fills[k], fills[k + 1]
t0 = rows[s0][0]
agg = collections.defaultdict(lambda: [0, 0.0])
idle = 0.0
prev = None
for s, e, n in rows[s0:s1 + 1]:
    gap = (s - prev) / 1e3 if prev is not None and s > prev else 0.0
    idle += gap
    print("%9.1f us gap %7.1f dur %8.1f %s" % ((s - t0) / 1e3, gap, (e - s) / 1e3, n))
    if s == rows[s1][0]:
        break
    cat = "blit " + n if n.startswith("__amd") else n
    agg[cat][0] += 1
    agg[cat][1] += (e - s) / 1e3
    prev = max(prev or 0, e)
span = (rows[s1][0] - t0) / 1e3
fused = sum(t for n, (c, t) in agg.items() if "k_open_fold_v2" in n)
print("\nstep span %.1f us (fill to next fill), GPU busy %.1f us, idle gaps %.1f us, ops %d, "
      "fused kernel %.1f us, step - fused %.1f us" % (span, span - idle, idle, s1 - s0, fused, span - fused))
for n, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%5d %9.1f us  %s" % (cnt, t, n))
