#!/usr/bin/env python3
"""One C3 step (bench_configs.py --config c3) from a rocprofv3 kernel + copy (+ marker) trace:
the GPU operations of one timed step, the idle gaps between them, and totals per category
(kernels by name, blit copies / fills, DMA copies).
With a marker trace (CE_ROCTX=1, rocprofv3 --marker-trace) the steps are the "c3_step" ranges:
step i's window runs from range i's start to range i+1's (every step ends in a host wait for its
compaction's length, so nothing of step i starts after range i+1 begins but the async download
of its sealed file); the median-span window among the timed steps is shown.  Without markers:
between one compaction's last serializer kernel (k_ser_tail) and the next step's.
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
marks = []
for fn in glob.glob(d + "/**/*marker_api_trace.csv", recursive=True):
    marks += sorted(int(r["Start_Timestamp"]) for r in csv.DictReader(open(fn))
                    if any("c3_step" in str(v) for v in r.values()))
wins = []
if len(marks) >= 3:
    for t0, t1 in zip(marks, marks[1:]):
        wins.append((t1 - t0, t0, t1))
    how = "ROCTx c3_step ranges"
else:
    tails = [r for r in rows if "k_ser_tail" in r[2]]
    for a, b in zip(tails, tails[1:]):
        n_count = sum(1 for r in rows if a[0] < r[0] <= b[0] and "k_ds_count" in r[2])
        if n_count == 1 and b[1] - a[1] < 20_000_000:
            wins.append((b[1] - a[1], a[1], b[1]))
    how = "k_ser_tail to k_ser_tail"
if not wins:
    sys.exit("no step window found")
wins.sort()
span, t0, t1 = wins[len(wins) // 2]
prev = t0
idle = 0.0
agg = collections.defaultdict(lambda: [0, 0.0])
sel = [r for r in rows if t0 <= r[0] < t1]
for s, e, n in sel:
    gap = max(0.0, (s - prev) / 1e3)
    idle += gap
    print("%9.1f us gap %7.1f dur %7.1f %s" % ((s - t0) / 1e3, gap, (e - s) / 1e3, n))
    cat = "blit " + n if n.startswith("__amd") else n
    agg[cat][0] += 1
    agg[cat][1] += (e - s) / 1e3
    prev = max(prev, e)
tail = max(0.0, (t1 - prev) / 1e3)
idle += tail
print("\nstep span %.1f us (%s), GPU busy %.1f us, idle gaps %.1f us (%.1f of it after the last op), ops %d, windows %d"
      % (span / 1e3, how, span / 1e3 - idle, idle, tail, len(sel), len(wins)))
for n, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%5d %9.1f us  %s" % (cnt, t, n))
