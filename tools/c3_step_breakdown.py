#!/usr/bin/env python3
"""One C3 step (bench_configs.py --config c3) from a rocprofv3 kernel + copy trace: the GPU
operations between one compaction's last serializer kernel (k_ser_tail) and the next step's, the
idle gaps between them, and totals per category (kernels by name, blit copies / fills, DMA
copies).  The step shown is the median-span one among the windows that hold exactly one op
decode (k_ds_count) and span under 20 ms (the timed steps, not the setup's compactions).
  python3 tools/c3_step_breakdown.py <trace dir>"""
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
tails = [i for i, r in enumerate(rows) if "k_ser_tail" in r[2]]
wins = []
for a, b in zip(tails, tails[1:]):
    n_count = sum("k_ds_count" in r[2] for r in rows[a + 1:b + 1])
    span = rows[b][1] - rows[a][1]
    if n_count == 1 and span < 20_000_000:
        wins.append((span, a, b))
if not wins:
    sys.exit("no step window found")
wins.sort()
span, a, b = wins[len(wins) // 2]
t0 = rows[a][1]
prev = t0
idle = 0.0
agg = collections.defaultdict(lambda: [0, 0.0])
for s, e, n in rows[a + 1:b + 1]:
    gap = max(0.0, (s - prev) / 1e3)
    idle += gap
    print("%9.1f us gap %7.1f dur %7.1f %s" % ((s - t0) / 1e3, gap, (e - s) / 1e3, n))
    cat = "blit " + n if n.startswith("__amd") else n
    agg[cat][0] += 1
    agg[cat][1] += (e - s) / 1e3
    prev = max(prev, e)
print("\nstep span %.1f us (ser_tail to ser_tail), GPU busy %.1f us, idle gaps %.1f us, ops %d, windows %d"
      % (span / 1e3, span / 1e3 - idle, idle, b - a, len(wins)))
for n, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%5d %9.1f us  %s" % (cnt, t, n))
