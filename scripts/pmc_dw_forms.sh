#!/bin/bash
# PMC counters of one YOLOv3 layer's dW (conv backward, no state.delta)
# under forced sdot forms
set -u
L=${L:-28}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmcdw_$L
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for F in ${FORMS:--1 64}; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d $OUT/f$F -o f$F --output-format csv -- python3 $R/scripts/dw_forms.py --layers $L --forms=$F --reps 2 > $OUT/f$F.log 2>&1
  rc=$?; echo "pmc $F rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
