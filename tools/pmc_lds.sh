#!/bin/bash
# One PMC pass over the fused kernel (256K files): LDS traffic / bank conflicts beside VALU.
set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_lds
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/p -o p -- python3 $R/bench.py --configs '' --versions 64 --steps 2 --warmup 1 --no-cpu --no-clock > $OUT/p.out 2> $OUT/p.err
echo "pmc rc=$?"
