#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run per set) over a python script:
#   NAME=tag bash scripts/pmc_run.sh scripts/conv_only.py --layer 45 ...
# Output: gpurun_out/pmc_$NAME/p<i>/...; summary via scripts/pmc_summary.py
set -u
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/pmc_${NAME:-run}; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
SCRIPT=$R/$1; shift
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_INSTS_SMEM SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d $OUT/p$i -o p$i --output-format csv -- python3 $SCRIPT "$@" > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $R/scripts/pmc_summary.py $OUT
