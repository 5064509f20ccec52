#!/bin/bash
# PMC counters of one YOLOv3 conv layer's forward (scripts/conv_fwd_layers.py
# --layers L): MFMA busy, LDS instructions / bank conflicts, wave waits
set -u
L=${L:-11}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_conv_$L
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY GRBM_GUI_ACTIVE -d $OUT/p1 -o p1 --output-format csv -- python3 $R/scripts/conv_fwd_layers.py --layers $L --reps 5 > $OUT/p1.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
