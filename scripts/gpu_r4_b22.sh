#!/bin/bash
# Round-4 batch 22: 16-byte stores in the short-row rearrangement (13^2):
# conv tests, layer 45 dW forms under a kernel trace, the bench.
set -u
mkdir -p gpurun_out/dwres10
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b22_tests.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -2 gpurun_out/b22_tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for L in 45; do
  (cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dwres10/l$L -o l$L --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/dw_res_prof.py --layer $L > $GRAFT_REPO_ROOT/gpurun_out/dwres10/l$L.json 2> $GRAFT_REPO_ROOT/gpurun_out/dwres10/l$L.err) || exit $?
  echo "layer $L ok"; cat gpurun_out/dwres10/l$L.json | cut -c1-400
done
NOTESTS=1 timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; exit $rc
