"""Condense rocprofv3 output (tools/rocprof.sh) into profiles/: kernel stats CSV, the bench line
it was taken with, and per-launch HBM traffic of the fused kernel (FETCH_SIZE x 2 per
MI355X_MICROARCH.md's gfx950 correction for 16-B/lane streaming reads, + WRITE_SIZE; KB -> B)."""
import csv, glob, json, os, shutil, sys

out = sys.argv[1]
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
prof = os.environ.get("PROFILE_DIR") or os.path.join(repo, "profiles")  # on a gpurun box: under gpurun_out/
os.makedirs(prof, exist_ok=True)
tag = os.environ.get("PROFILE_TAG", "r01")

stats = glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(prof, "%s_kernel_stats.csv" % tag))
    fused = [r["Name"].split("(")[0].replace("void ", "") for r in csv.DictReader(open(stats[0]))
             if "k_open_fold" in r["Name"]]
    # what bench.py's roofline.rocprof checks before using these averages
    with open(os.path.join(prof, "%s_kernel_stats.meta.json" % tag), "w") as f:
        json.dump({"files_per_launch": 1 << 20, "fused_kernel": fused[0] if fused else None,
                   "command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --configs '' --steps 5 "
                              "--warmup 1 --no-cpu --no-variant-b --no-host-buffers --no-clock"}, f, indent=1)
    for row in csv.DictReader(open(stats[0])):
        print("%-60.60s calls %6s avg_us %10.2f pct %6.2f" % (row["Name"], row["Calls"],
              float(row["AverageNs"]) / 1e3, float(row["Percentage"])))
bl = open(os.path.join(out, "trace.out")).read().strip().splitlines()
if bl:
    with open(os.path.join(prof, "%s_bench_under_rocprof.json" % tag), "w") as f:
        f.write(bl[-1] + "\n")

def per_launch(counter):
    vals = {}
    for fn in glob.glob(os.path.join(out, counter, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            if "k_open_fold" in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.setdefault(row["Dispatch_Id"], []).append((float(row["Counter_Value"]), row["Grid_Size"]))
                kernel[0] = row["Kernel_Name"]
    return [sum(v for v, _ in x) for x in vals.values()]

kernel = [""]

fs, ws = per_launch("FETCH_SIZE"), per_launch("WRITE_SIZE")
if fs and ws:
    fetch = sum(fs) / len(fs) * 1024 * 2
    write = sum(ws) / len(ws) * 1024
    files = 1 << 20
    rec = {"kernel": kernel[0], "launches_measured": [len(fs), len(ws)],
           "files_per_launch": files,
           "fetch_bytes_per_launch": round(fetch), "write_bytes_per_launch": round(write),
           "bytes_per_launch": round(fetch + write),
           "algorithmic_bytes_per_launch": files * 4101,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
                     "bench.py --steps 2 --warmup 1 --no-cpu --no-variant-b --no-host-buffers (1M files, past the 256 MiB L3); "
                     "FETCH_SIZE (KB) x 1024 x 2 (gfx950: FETCH_SIZE reports half of 16-B/lane "
                     "streaming reads) + WRITE_SIZE (KB) x 1024"}
    with open(os.path.join(prof, "traffic_open_fold_small.json"), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))
