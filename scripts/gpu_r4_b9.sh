#!/bin/bash
# Round-4 batch 9: per-layer backward split with the final dW / dX picks,
# the conv tests, the bench line.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b9_tests.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -2 gpurun_out/b9_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_r4_b5.sh || exit $?
timeout -k 10 300 python scripts/conv_bwd_layers.py > gpurun_out/bwd_layers_r4.json 2> gpurun_out/bwd_layers_r4.err || exit $?
echo "bwd layers ok"
NOTESTS=1 timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; exit $rc
