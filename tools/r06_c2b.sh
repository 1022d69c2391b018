#!/bin/bash
# round 6: parity + same-box A/B (prev vs current lib) + one VALU PMC pass of the current lib
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="${LIBS:-crdt-enc_amd/libcrdtenc_prev.so crdt-enc_amd/libcrdtenc.so}" bash tools/r06_c2.sh || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_c2b; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $OUT/pass1 -o p -- \
  python3 $GRAFT_REPO_ROOT/bench.py --configs '' --steps 2 --warmup 1 --no-cpu --no-variant-b --no-host-buffers --no-clock > $OUT/pass1.out 2> $OUT/pass1.err || { echo "pmc failed"; tail -5 $OUT/pass1.err; exit 1; }
python3 - <<'PY'
import csv,glob,collections,os
out=os.environ["GRAFT_REPO_ROOT"]+"/gpurun_out/pmc_c2b/pass1"
v=collections.defaultdict(lambda: collections.defaultdict(float))
for fn in glob.glob(out+"/**/*counter_collection.csv",recursive=True):
    for r in csv.DictReader(open(fn)):
        if "k_open_fold" in r["Kernel_Name"]:
            v[r["Dispatch_Id"]][r["Counter_Name"]]+=float(r["Counter_Value"])
vals=[d["SQ_INSTS_VALU"]*64/(1<<20) for d in v.values()]
print("fused VALU lane-instr/file", [round(x) for x in vals])
PY
