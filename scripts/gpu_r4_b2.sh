#!/bin/bash
# Round-4 batch 2: the changed paths' tests first (fail fast), the state.delta
# forms per layer, then smoke + the whole GPU suite + the bench line.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_sgemm.py -x -q --timeout 120 --timeout-method thread -k "dx_conv or dx_yolov3 or nn_big or overlap or matches_oracle or dx_tiles" > gpurun_out/b2_tests.log 2>&1
rc=$?; echo "targeted tests rc=$rc"; tail -3 gpurun_out/b2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bwd_sweep.py --what dx --layers 6,11,28,45,10,27,44 > gpurun_out/bwd_dx.json 2> gpurun_out/bwd_dx.err || exit $?
echo "bwd dx sweep ok"
bash scripts/gpu_r4_check.sh
