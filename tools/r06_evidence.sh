#!/bin/bash
# round 6 evidence for profiles/: kernel-trace stats + HBM traffic passes of the C2 bench command,
# then the VALU PMC passes (written under gpurun_out/profiles, copied into profiles/ by hand)
set -o pipefail
export PROFILE_DIR=$GRAFT_REPO_ROOT/gpurun_out/profiles PROFILE_TAG=r06
mkdir -p $PROFILE_DIR
bash $GRAFT_REPO_ROOT/tools/rocprof.sh || exit 1
bash $GRAFT_REPO_ROOT/tools/pmc_valu.sh || exit 1
