#!/bin/bash
# PMC passes over a short bench run (256K files, 2 steps); one rocprofv3 run per pass.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
         "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $OUT/pass$i -o p -- python3 $R/bench.py --configs '' --versions 64 --steps 2 --warmup 1 --no-cpu --no-clock > $OUT/pass$i.out 2> $OUT/pass$i.err
  echo "pass $i rc=$?"
done
