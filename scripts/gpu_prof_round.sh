#!/bin/bash
# Round profile: bench kernel trace + PMC traffic passes (scripts/profile.sh),
# then SQ counter passes on two YOLOv3 conv layers (scripts/pmc_run.sh).
set -u
TAG=${TAG:-r01} bash scripts/profile.sh || exit $?
cd $GRAFT_REPO_ROOT
for L in ${LAYERS:-11 45}; do
  NAME=l$L bash scripts/pmc_run.sh scripts/conv_only.py --layer $L --reps 20 > gpurun_out/pmc_l$L.txt 2>&1
  rc=$?; echo "pmc l$L rc=$rc"; tail -30 gpurun_out/pmc_l$L.txt; [ $rc -eq 0 ] || exit $rc
done
