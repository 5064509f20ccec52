#!/bin/bash
# rocprofv3 passes for the bench command: kernel trace + stats, then PMC
# passes (FETCH_SIZE and WRITE_SIZE separately, per the gfx950 guide), then
# MFMA busy + GPU clock.  Output under gpurun_out/prof_<tag>/.
set -u
TAG=${TAG:-r01}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
ARGS="${PROF_ARGS:---no-cpu}"
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $R/bench.py $ARGS > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run trace --kernel-trace --stats || exit $?
[ "${PMC:-1}" = "1" ] || exit 0
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
run mfma --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES || exit $?
exit 0
