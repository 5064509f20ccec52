#!/bin/bash
# Round-5 counter evidence:
#  * elementwise traffic on the shipped BN kernels (profile_elementwise.sh)
#  * conv_tile4 forward, layers 11 (52^2), 28 (26^2), 45 (13^2), 10 (1x1):
#    SQ pass (MFMA busy, LDS, waits, VALU) and FETCH / WRITE passes
#  * conv backward dominant kernels on the same layers: MFMA busy, FETCH, WRITE
# Output under gpurun_out/pmc_r5/ (summarised by scripts/summarize_pmc_r5.py).
set -u
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/pmc_r5
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
SQ="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
pass() {  # name, counters, command...
  local name=$1 ctr=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $ctr -d $OUT/$name -o $name --output-format csv -- "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
for L in ${LAYERS:-11 28 45 10}; do
  F="python3 $R/scripts/conv_one.py --layer $L --variants=-1 --rounds 1 --reps 5"
  pass fwd${L}_sq "$SQ" $F || exit $?
  pass fwd${L}_fetch "FETCH_SIZE" $F || exit $?
  pass fwd${L}_write "WRITE_SIZE" $F || exit $?
  B="python3 $R/scripts/conv_bwd_one.py --layer $L --reps 3"
  pass bwd${L}_sq "$SQ" $B || exit $?
  pass bwd${L}_fetch "FETCH_SIZE" $B || exit $?
  pass bwd${L}_write "WRITE_SIZE" $B || exit $?
done
pass sgemm_sq "$SQ" python3 $R/scripts/sgemm_one.py --reps 5 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- python3 $R/scripts/conv_one.py --layer 11 --variants=-1 --rounds 1 --reps 5 > $OUT/trace.log 2>&1
echo "trace rc=$?"
if [ "${EW:-1}" = "1" ]; then TAG=r05 bash $R/scripts/profile_elementwise.sh || exit $?; fi
exit 0
