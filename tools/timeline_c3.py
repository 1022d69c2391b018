"""One C3 step's GPU timeline (kernels + copies: start, gap, duration) from a rocprofv3 trace of
bench_configs.py --config c3: everything between two consecutive k_ds_count launches."""
import csv, glob, sys
rows = []
for fn in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70]) for r in csv.DictReader(open(fn))]
for fn in glob.glob(sys.argv[1] + "/**/*memory_copy_trace.csv", recursive=True):
    rows += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "COPY %s %s" % (r.get("Direction", ""), r.get("Size", "")))
             for r in csv.DictReader(open(fn))]
rows.sort()
idx = [i for i, r in enumerate(rows) if "k_ds_count" in r[2]]
a, b = idx[-3], idx[-2]
t0, prev = rows[a][0], None
busy = 0
for s, e, name in rows[a:b]:
    print("%9.1f us gap %7.1f dur %8.1f %s" % ((s - t0) / 1e3, (s - prev) / 1e3 if prev else 0, (e - s) / 1e3, name))
    prev = e
    busy += e - s
print("step span %.1f us, busy %.1f us" % ((rows[b][0] - t0) / 1e3, busy / 1e3))
