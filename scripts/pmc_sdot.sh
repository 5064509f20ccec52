#!/bin/bash
# counter passes over scripts/sdot_one.py (args passed through)
set -u
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/pmc_${NAME:-sdot}; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
i=0
for set in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM_RD"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/p$i -o p$i --output-format csv -- python3 $R/scripts/sdot_one.py "$@" > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 $R/scripts/pmc_summary.py $OUT
