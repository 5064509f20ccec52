#!/bin/bash
# kernel-trace of the elementwise sweep (pure kernel durations, no host gaps)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ewprof -o ew --output-format csv -- python3 $R/scripts/elementwise_perf.py > $R/gpurun_out/ewprof.log 2>&1
rc=$?; tail -2 $R/gpurun_out/ewprof.log; exit $rc
