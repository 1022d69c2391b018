#!/bin/bash
# VALU / LDS PMC passes (tools/pmc_valu.sh's two passes) for each library in $LIBS, same box:
#   LIBS="crdt-enc_amd/libcrdtenc_base.so crdt-enc_amd/libcrdtenc.so" tools/pmc_ab.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for L in ${LIBS}; do
  OUT=$R/gpurun_out/pmc_ab/$(basename $L .so)
  mkdir -p $OUT
  i=0
  for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    CRDTENC_LIB=$R/$L timeout -s KILL 180 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/pass$i -o p -- \
      python3 $R/bench.py --configs '' --steps 2 --warmup 1 --no-cpu --no-variant-b --no-host-buffers --no-clock > $OUT/pass$i.out 2> $OUT/pass$i.err || { echo "pass $i failed rc=$?"; tail -5 $OUT/pass$i.err; exit 1; }
  done
  echo "== $L"
  python3 $R/tools/summarize_valu.py $OUT | python3 -c "
import json,sys; d=json.load(sys.stdin); f=d['fused']; c=f['counters']
print('ms', f['avg_duration_ms'], 'valu/file', f.get('valu_instr_per_file_per_lane'), 'lds_conf', c['SQ_LDS_BANK_CONFLICT'], 'lds_inst', c['SQ_INSTS_LDS'], 'salu', c['SQ_INSTS_SALU'], 'split', f.get('wave_cycle_split'))"
done
