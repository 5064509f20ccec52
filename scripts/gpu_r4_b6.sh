#!/bin/bash
# Round-4 batch 6: dw_res (faster rearrangement, measured picks) tests and
# per-layer forms, BN staging tests + perf, the whole GPU suite, the bench.
set -u
mkdir -p gpurun_out/dwres2
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -k "dw_res or yolov3_batch8 or overlap or caller_workspace or matches_oracle" > gpurun_out/b6_tests.log 2>&1
rc=$?; echo "dw tests rc=$rc"; tail -3 gpurun_out/b6_tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for L in 11 28 45 9 3 4 6; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dwres2/l$L -o l$L --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/dw_res_prof.py --layer $L > $GRAFT_REPO_ROOT/gpurun_out/dwres2/l$L.json 2> $GRAFT_REPO_ROOT/gpurun_out/dwres2/l$L.err) || exit $?
  echo "layer $L ok"; cat gpurun_out/dwres2/l$L.json
done
bash scripts/gpu_r4_b5.sh || exit $?
bash scripts/gpu_r4_check.sh
