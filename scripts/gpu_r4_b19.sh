#!/bin/bash
# Round-4 batch 19: the derivative fused into the bias sums: every GPU test,
# the bench.
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/conv_bwd_layers.py > gpurun_out/bwd_layers_b19.json 2> gpurun_out/bwd_layers_b19.err || exit $?
echo "bwd layers ok"
NOTESTS=1 timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; exit $rc
