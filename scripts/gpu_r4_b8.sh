#!/bin/bash
# Round-4 batch 8: dw_res with 16-byte fragment reads + the one-residue-first
# picks: tests, per-layer forms, then the whole GPU suite and the bench.
set -u
mkdir -p gpurun_out/dwres4
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -k "dw_res or yolov3_batch8 or overlap or caller_workspace or dx_conv" > gpurun_out/b8_tests.log 2>&1
rc=$?; echo "dw tests rc=$rc"; tail -3 gpurun_out/b8_tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for L in 11 28 45 4 3; do
  (cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dwres4/l$L -o l$L --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/dw_res_prof.py --layer $L > $GRAFT_REPO_ROOT/gpurun_out/dwres4/l$L.json 2> $GRAFT_REPO_ROOT/gpurun_out/dwres4/l$L.err) || exit $?
  echo "layer $L ok"; cat gpurun_out/dwres4/l$L.json
done
bash scripts/gpu_r4_check.sh
