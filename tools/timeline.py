"""Print one bench step's kernel timeline (start, gap, duration) from a rocprofv3 kernel trace."""
import csv, glob, sys
fn = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(fn)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "k_open_fold" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
t0, prev = int(rows[a - 6]["Start_Timestamp"]), None
for r in rows[a - 6:b - 5]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%9.1f us gap %7.1f dur %8.1f %s" % ((s - t0) / 1e3, (s - prev) / 1e3 if prev else 0,
                                                (e - s) / 1e3, r["Kernel_Name"][:60]))
    prev = e
