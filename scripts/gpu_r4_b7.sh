#!/bin/bash
# Round-4 batch 7: dw_res tests and per-layer forms (incl. the one-residue
# forms on the long-k layers), then the counter evidence (conv forward /
# backward PMC passes, elementwise traffic).
set -u
mkdir -p gpurun_out/dwres3
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -k "dw_res or yolov3_batch8 or overlap or caller_workspace" > gpurun_out/b7_tests.log 2>&1
rc=$?; echo "dw tests rc=$rc"; tail -3 gpurun_out/b7_tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for L in 11 28 45 9 3 1 4 6; do
  (cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dwres3/l$L -o l$L --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/dw_res_prof.py --layer $L > $GRAFT_REPO_ROOT/gpurun_out/dwres3/l$L.json 2> $GRAFT_REPO_ROOT/gpurun_out/dwres3/l$L.err) || exit $?
  echo "layer $L ok"; cat gpurun_out/dwres3/l$L.json
done
bash scripts/gpu_r4_b5.sh || exit $?
timeout -k 10 300 python scripts/bwd_sweep.py --what dx --layers 28,45,11,6,43 > gpurun_out/bwd_dx2.json 2> gpurun_out/bwd_dx2.err || exit $?
echo "bwd dx sweep ok"
bash scripts/gpu_r4_evidence.sh
