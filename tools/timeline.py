"""Print one bench step's GPU timeline (kernels and copies: start, gap, duration) from a
rocprofv3 kernel (+ memory-copy) trace directory."""
import csv, glob, sys
rows = []
for fn in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]) for r in csv.DictReader(open(fn))]
for fn in glob.glob(sys.argv[1] + "/**/*memory_copy_trace.csv", recursive=True):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY " + r.get("Direction", "") + " " + r.get("Size", ""))
             for r in csv.DictReader(open(fn))]
rows.sort()
idx = [i for i, r in enumerate(rows) if "k_open_fold" in r[2]]
a, b = idx[-3], idx[-2]
lo = max(i for i in range(a) if "k_open_fold" not in rows[i][2] and (i == 0 or i <= a - 1)) if a else 0
# from the kernel after the previous step's fused kernel to this step's fused kernel and its tail
start = idx[-4] + 1 if len(idx) >= 4 else 0
t0, prev = rows[start][0], None
for s, e, name in rows[start:b]:
    print("%9.1f us gap %7.1f dur %8.1f %s" % ((s - t0) / 1e3, (s - prev) / 1e3 if prev else 0, (e - s) / 1e3, name))
    prev = e
print("step span %.1f us" % ((rows[b][0] - rows[idx[-3] - (a - start - (idx[-3] - start))][0]) / 1e3 if False else (rows[b][0] - rows[start][0]) / 1e3))
