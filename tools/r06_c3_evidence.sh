#!/bin/bash
# round 6 C3 evidence: one step's GPU timeline, the fold / merge HBM traffic, the op open's VALU PMC
set -o pipefail
R=$GRAFT_REPO_ROOT
bash $R/tools/c3_step.sh > $R/gpurun_out/c3_step_summary.txt || exit 1
tail -25 $R/gpurun_out/c3_step_summary.txt
bash $R/tools/c3_traffic.sh > $R/gpurun_out/c3_traffic_out.txt || exit 1
PMC="SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS" KERN="k_open_ds8" bash $R/tools/c3_pmc.sh || exit 1
