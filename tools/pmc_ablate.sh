#!/bin/bash
# SQ_INSTS_VALU / LDS of the fused kernel with phases switched off (diagnostics build, CE_ABLATE
# bits: 1 no decode, 2 no Poly1305 products, 4 no ChaCha20, 8 no ciphertext loads): where the
# VALU instructions go.  256K files per launch (tools/ablate.py), one rocprofv3 run per setting.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_ablate
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for b in ${ABL_BITS:-0 1 2 4 7}; do
  CRDTENC_LIB=$R/crdt-enc_amd/libcrdtenc_prof.so CE_ABLATE=$b timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/b$b -o p -- \
    python3 $R/tools/ablate.py > $OUT/b$b.out 2> $OUT/b$b.err
  rc=$?   # the bench's own checks fail by construction (ablated results); a crash or kill does not pass
  [ $rc -le 1 ] || [ $rc -eq 3 ] || { echo "ablate $b rc=$rc"; tail -5 $OUT/b$b.err; exit 1; }
  python3 - $OUT/b$b <<'PY'
import csv, glob, sys
p = sys.argv[1]; per = {}; durs = []
for fn in glob.glob(p + "/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        if "k_open_fold_v2" in row["Kernel_Name"]:
            k = (row["Dispatch_Id"], row["Counter_Name"]); per[k] = per.get(k, 0) + float(row["Counter_Value"])
for fn in glob.glob(p + "/**/*kernel_trace.csv", recursive=True):
    for row in csv.DictReader(open(fn)):
        if "k_open_fold_v2" in row["Kernel_Name"]:
            durs.append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
c = {}
for (d, n), v in per.items(): c.setdefault(n, []).append(v)
c = {n: sum(v) / len(v) for n, v in c.items()}
files = 262144
print(p.split("/")[-1], "ms %.4f" % (sum(durs) / len(durs) / 1e6), "valu/file %.0f" % (c["SQ_INSTS_VALU"] * 64 / files),
      "salu/wave-it %.0f" % (c["SQ_INSTS_SALU"] / (files / 4)), "lds/wave-it %.1f" % (c["SQ_INSTS_LDS"] / (files / 4)),
      "conf/wave-it %.0f" % (c["SQ_LDS_BANK_CONFLICT"] / (files / 4)))
PY
  rm -rf $OUT/b$b   # the per-dispatch CSVs are large; the line above is the record
done
