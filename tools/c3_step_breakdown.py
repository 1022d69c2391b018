#!/usr/bin/env python3
"""One C3 step (bench_configs.py --config c3) from a rocprofv3 kernel + copy trace: every GPU
operation between the step's first state-reader kernel and its compaction's last kernel, the
idle gaps between them, and totals per category (kernels by name, blit copies / fills, DMA
copies, idle)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
rows = []
for fn in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:])
             for r in csv.DictReader(open(fn))]
for fn in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "DMA " + r.get("Direction", "")[-14:])
             for r in csv.DictReader(open(fn))]
rows.sort()
count = [i for i, r in enumerate(rows) if "k_ds_count" in r[2]]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3     # which ingest_ops (a timed step)
c = count[k]
start = max(i for i in range(c) if ("k_rd_find" in rows[i][2] or "k_rdm_count" in rows[i][2]))
while start > 0 and ("k_rd_find" in rows[start - 1][2] or "k_rdm_count" in rows[start - 1][2]):
    start -= 1
# back to the step's reset (the fills before the states' upload)
s0 = start
while s0 > 0 and rows[s0 - 1][0] > rows[start][0] - 3000_000 and "k_ser_tail" not in rows[s0 - 1][2] \
        and "k_finalize_multi<true>" not in rows[s0 - 1][2]:
    s0 -= 1
end = min(i for i in range(c, len(rows)) if "k_ser_tail" in rows[i][2])
end = min(i for i in range(end, len(rows)) if "k_finalize_multi<true>" in rows[i][2] or i == len(rows) - 1)
while end + 1 < len(rows) and rows[end + 1][0] - rows[end][1] < 200_000 and "k_rd_find" not in rows[end + 1][2] \
        and "fillBuffer" not in rows[end + 1][2]:
    end += 1
t0 = rows[s0][0]
agg = collections.defaultdict(lambda: [0, 0.0])
idle = 0.0
prev = None
for s, e, n in rows[s0:end + 1]:
    gap = (s - prev) / 1e3 if prev is not None and s > prev else 0.0
    idle += gap
    print("%9.1f us gap %7.1f dur %7.1f %s" % ((s - t0) / 1e3, gap, (e - s) / 1e3, n))
    cat = "blit " + n if n.startswith("__amd") else n
    agg[cat][0] += 1
    agg[cat][1] += (e - s) / 1e3
    prev = max(prev or 0, e)
span = (rows[end][1] - t0) / 1e3
print("\nstep span %.1f us, GPU busy %.1f us, idle gaps %.1f us, ops %d" % (span, span - idle, idle, end + 1 - s0))
for n, (cnt, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print("%5d %9.1f us  %s" % (cnt, t, n))
