#!/usr/bin/env python3
"""Summarise CE_HOST_PROF=1 stderr (one line per host phase): count, median and total ms per
phase name over the last K occurrences of the most frequent phase's count (the timed steps).
  python3 tools/host_prof_summary.py <stderr file> [steps]"""
import collections
import statistics
import sys

rows = collections.defaultdict(list)
for line in open(sys.argv[1]):
    if line.startswith("CE_HOST_PROF"):
        parts = line.split()
        name, ms = " ".join(parts[1:-2]), float(parts[-2])
        rows[name].append(ms)
k = int(sys.argv[2]) if len(sys.argv) > 2 else 40
print("%-34s %6s %9s %9s" % ("phase", "n", "median", "mean"))
for name, v in sorted(rows.items(), key=lambda kv: -statistics.mean(kv[1][-k:])):
    v = v[-k:]
    print("%-34s %6d %9.3f %9.3f" % (name, len(v), statistics.median(v), statistics.mean(v)))
