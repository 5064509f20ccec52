#!/bin/bash
# PMC counters of one YOLOv3 conv layer's forward under forced variants
set -u
L=${L:-11}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcv_$L
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for V in ${VARS:-100 300 400}; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/v$V -o v$V --output-format csv -- python3 $R/scripts/conv_one.py --layer $L --variants=$V --rounds 1 --reps 5 > $OUT/v$V.log 2>&1
  rc=$?; echo "pmc $V rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
