#!/bin/bash
# scripts/profile.sh over the bench command, summarised on the box (the raw
# traces exceed what gpurun copies back): kernel stats csv, the SGEMM
# traffic json, per-kernel PMC summary; raw csv removed
set -u
TAG=${TAG:-r06}
R=$GRAFT_REPO_ROOT
bash $R/scripts/profile.sh || exit $?
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $R/gpurun_out/sum_$TAG
python3 $R/scripts/summarize_profile.py $OUT $TAG --steps ${STEPS:-20} > $R/gpurun_out/sum_$TAG/summary.log 2>&1
cp $R/profiles/${TAG}_* $R/gpurun_out/sum_$TAG/ 2>/dev/null
python3 $R/scripts/pmc_by_kernel.py $OUT $R/gpurun_out/sum_$TAG/${TAG}_pmc_by_kernel.json
rm -rf $OUT
