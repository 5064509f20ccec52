#!/bin/bash
# SQ counter passes on the 4096^3 SGEMM alone.
set -u
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/pmc_sgemm; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
V=${VARIANT:--1}
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $set -d $OUT/p$i -o p$i --output-format csv -- python3 $R/scripts/sgemm_only.py --variant $V --reps 5 > $OUT/p$i.log 2>&1
  echo "pass $i rc=$?"
done
