"""Per-dispatch PMC summary of the fused kernel and the setup kernel (tools/pmc_valu.sh output):
counter means over the dispatches of each kernel, durations from the same runs' kernel traces,
and derived rates: VALU lane-instructions/s (SQ_INSTS_VALU x 64 / duration) against the measured
int32 VALU rate (tools/ubench_int, 38.9 T lane-ops/s) and the 78.6 T lane-slot peak."""
import csv, glob, json, os, sys

out = sys.argv[1]
repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"k_open_fold_v": "fused", "k_open_setup": "setup"}
names = {}
acc = {}    # short -> counter -> [per-dispatch sums]
durs = {}   # short -> [ns]
for p in sorted(glob.glob(os.path.join(out, "pass*"))):
    if not os.path.isdir(p):
        continue
    per = {}
    for fn in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            short = next((v for k, v in KERNELS.items() if k in row["Kernel_Name"]), None)
            if short:
                names[short] = row["Kernel_Name"].split("(")[0]
                key = (short, row["Dispatch_Id"], row["Counter_Name"])
                per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
    for (short, _, cn), v in per.items():
        acc.setdefault(short, {}).setdefault(cn, []).append(v)
    for fn in glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(fn)):
            short = next((v for k, v in KERNELS.items() if k in row["Kernel_Name"]), None)
            if short:
                durs.setdefault(short, []).append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
res = {"method": "rocprofv3 --pmc <pass> --kernel-trace, bench.py --steps 2 --warmup 1 --no-cpu --no-variant-b --no-host-buffers "
                 "(1,048,576 files per launch); counters summed over the device per dispatch, "
                 "averaged over dispatches; durations from the same runs' kernel traces"}
for short, cs in acc.items():
    d = {cn: sum(v) / len(v) for cn, v in cs.items()}
    ns = sum(durs.get(short, [0])) / max(len(durs.get(short, [])), 1)
    r = {"dispatches": max(len(v) for v in cs.values()), "avg_duration_ms": round(ns / 1e6, 4),
         "counters": {k: round(v) for k, v in sorted(d.items())}}
    if ns and "SQ_INSTS_VALU" in d:
        lane_ops = d["SQ_INSTS_VALU"] * 64 / (ns * 1e-9) / 1e12
        r["valu_lane_instr_Tps"] = round(lane_ops, 2)
        r["valu_frac_of_measured_int32_rate"] = round(lane_ops / 38.9, 4)
        r["valu_frac_of_lane_slot_peak"] = round(lane_ops / 78.6, 4)
        r["valu_instr_per_file_per_lane"] = round(d["SQ_INSTS_VALU"] * 64 / (1 << 20), 1)
    if "SQ_WAVE_CYCLES" in d and "SQ_WAIT_ANY" in d:
        wc = d["SQ_WAVE_CYCLES"]
        r["wave_cycle_split"] = {k: round(d[k] / wc, 4) for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY",
                                                                   "SQ_WAIT_ANY") if k in d}
    res[short] = r
if "fused" in res:
    res["fused"]["kernel"] = names.get("fused", "k_open_fold_v3")
print(json.dumps(res, indent=1))
with open(os.path.join(out, "summary.json"), "w") as f:
    json.dump(res, f, indent=1)
# profiles/valu_pmc.json is what bench.py reads (roofline.pmc_valu); the tagged copy is the record
tag = os.environ.get("PROFILE_TAG", "r02")
for name in ("valu_pmc.json", "%s_valu_pmc.json" % tag):
    pdir = os.environ.get("PROFILE_DIR") or os.path.join(repo, "profiles")  # gpurun box: under gpurun_out/
    os.makedirs(pdir, exist_ok=True)
    with open(os.path.join(pdir, name), "w") as f:
        json.dump(res, f, indent=1)
