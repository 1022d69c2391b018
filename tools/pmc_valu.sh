#!/bin/bash
# VALU / LDS / wait-state PMC passes of the default bench workload (1M files, 2 steps), one
# rocprofv3 run per pass with kernel-trace for per-dispatch durations; summary -> gpurun_out/pmc_valu
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_valu
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/pass$i -o p -- \
    python3 $R/bench.py --configs '' --steps 2 --warmup 1 --no-cpu --no-variant-b --no-host-buffers --no-clock > $OUT/pass$i.out 2> $OUT/pass$i.err || { echo "pass $i failed rc=$?"; tail -5 $OUT/pass$i.err; exit 1; }
  echo "pass $i ok"
done
python3 $R/tools/summarize_valu.py $OUT
