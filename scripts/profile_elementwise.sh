#!/bin/bash
# rocprofv3 passes over scripts/elementwise_traffic.py: kernel trace + stats,
# then FETCH_SIZE and WRITE_SIZE in separate passes (MI355X_MICROARCH.md §HBM).
# Output under gpurun_out/prof_ew_<tag>/.
set -u
TAG=${TAG:-r02}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/prof_ew_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
run() { local name=$1; shift; timeout -k 10 300 rocprofv3 "$@" -d $OUT/$name -o $name --output-format csv -- python3 $R/scripts/elementwise_traffic.py > $OUT/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; return $rc; }
run trace --kernel-trace --stats || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
exit 0
