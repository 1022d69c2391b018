#!/usr/bin/env python3
"""One C2 step's host HIP API calls and GPU operations on one clock (rocprofv3 --hip-runtime-trace
+ --kernel-trace + --memory-copy-trace): from the step's k_fill launch call to the next one.
Rows: 'API' = a host call (start, duration), 'GPU' = a kernel / copy (start, duration).

  tools/c2_api_breakdown.py <rocprofv3 output dir> [step index] [step marker kernel]
(the marker defaults to ce::k_fill, C2's first launch; C3: ce::k_open_setup of the states)"""
import csv
import glob
import sys

d = sys.argv[1]
ev = []
for fn in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "GPU",
                   r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-44:]))
for fn in glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "GPU", "DMA " + r.get("Direction", "")[-14:]))
api = []
for fn in glob.glob(d + "/**/*hip_api_trace.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        api.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "API", r["Function"][:44]))
ev += api
ev.sort()
marker = sys.argv[3] if len(sys.argv) > 3 else "ce::k_fill"
fills = [e for e in ev if e[2] == "GPU" and marker in e[3]]
k = int(sys.argv[2]) if len(sys.argv) > 2 and int(sys.argv[2]) >= 0 else len(fills) - 2
g0, g1 = fills[k][0], fills[k + 1][0]
# the host window: from the launch call of this step's fill to that of the next
launches = [e for e in api if "LaunchKernel" in e[3] or "ModuleLaunch" in e[3]]
def launch_before(t):
    c = [e for e in launches if e[0] <= t]
    return c[-1][0] if c else t
# the step's first host call: the earliest API call after the previous step's last GPU op ended
prev_end = max(e[1] for e in ev if e[2] == "GPU" and e[1] <= g0) if any(e[2] == "GPU" and e[1] <= g0 for e in ev) else g0
h0 = min(launch_before(g0), g0)
t0 = min(h0, g0)
tot = {}
for s, e, kind, name in ev:
    if s < t0 - 200_000 or s > g1:
        continue
    print("%9.1f us %s dur %8.1f %s" % ((s - t0) / 1e3, kind, (e - s) / 1e3, name))
    if kind == "API" and s >= t0:
        tot[name] = tot.get(name, [0, 0.0])
        tot[name][0] += 1
        tot[name][1] += (e - s) / 1e3
print("\nhost API time in the step window (calls, us):")
for n, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
    print("%5d %9.1f  %s" % (c, t, n))
