#!/usr/bin/env python3
"""One C3 step's HOST side from a rocprofv3 --hip-trace --kernel-trace --marker-trace run
(CE_ROCTX=1): the HIP calls the launching thread makes inside one timed "c3_step" range (the
median-length one), each call's duration and the host time before it (the library's own host
work and Python), and totals per HIP function.
  python3 tools/c3_host_trace.py <trace dir>"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
kern = {}
for fn in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        kern[int(r.get("Correlation_Id", 0) or 0)] = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:]
api = []
for fn in glob.glob(d + "/**/*hip_api_trace.csv", recursive=True):
    api += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"], int(r["Thread_Id"]),
             int(r.get("Correlation_Id", 0) or 0)) for r in csv.DictReader(open(fn))]
api.sort()
marks = []
for fn in glob.glob(d + "/**/*marker_api_trace.csv", recursive=True):
    marks += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(fn))
              if any("c3_step" in str(v) for v in r.values())]
if not marks:
    sys.exit("no c3_step ranges (run with CE_ROCTX=1 and --marker-trace)")
marks.sort(key=lambda m: m[1] - m[0])
h0, h1 = marks[len(marks) // 2]
main = collections.Counter(x[3] for x in api if h0 <= x[0] <= h1).most_common(1)[0][0]
calls = [x for x in api if h0 <= x[0] <= h1 and x[3] == main]
agg = collections.defaultdict(lambda: [0, 0.0])
prev = h0
host_gap = 0.0
print("host step %.1f us (median of %d timed steps), launching thread %d, %d calls"
      % ((h1 - h0) / 1e3, len(marks), main, len(calls)))
for s, e, f, _, corr in calls:
    gap = (s - prev) / 1e3
    host_gap += max(gap, 0.0)
    dur = (e - s) / 1e3
    agg[f][0] += 1
    agg[f][1] += dur
    k = kern.get(corr)
    if gap > 10 or dur > 10:
        print("%9.1f us  host %7.1f  call %7.1f  %s%s" % ((s - h0) / 1e3, gap, dur, f, ("  -> " + k) if k else ""))
    prev = e
host_gap += max(0.0, (h1 - prev) / 1e3)
print("\nhost time outside HIP calls %.1f us; in HIP calls %.1f us" % (host_gap, sum(v[1] for v in agg.values())))
for f, (n, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:25]:
    print("%5d %9.1f us  %s" % (n, t, f))
