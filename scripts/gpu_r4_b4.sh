#!/bin/bash
# Round-4 batch 4: dw_res tests, then per-layer dW forms with a kernel trace
# each (the per-kernel split of the rearrangement passes and the product).
set -u
mkdir -p gpurun_out/dwres
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -k "dw_res or yolov3_batch8 or overlap or caller_workspace" > gpurun_out/b4_tests.log 2>&1
rc=$?; echo "targeted tests rc=$rc"; tail -3 gpurun_out/b4_tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for L in 11 28 45 9 26 43 6; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dwres/l$L -o l$L --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/dw_res_prof.py --layer $L > $GRAFT_REPO_ROOT/gpurun_out/dwres/l$L.json 2> $GRAFT_REPO_ROOT/gpurun_out/dwres/l$L.err) || exit $?
  echo "layer $L ok"; cat gpurun_out/dwres/l$L.json
done
