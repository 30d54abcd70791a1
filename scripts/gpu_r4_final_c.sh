#!/bin/bash
# Round-4 evidence C: SQ/TA/TCC counter passes of configs 2, 5 and the halo
# line, then the driver's N>1 launch rehearsed on one GPU.
cd $GRAFT_REPO_ROOT
bash scripts/gpu_pmc_cfg2.sh || exit $?
bash scripts/gpu_pmc_cfg5.sh || exit $?
bash scripts/gpu_pmc_halo.sh || exit $?
bash scripts/gpu_scale_rehearsal.sh
