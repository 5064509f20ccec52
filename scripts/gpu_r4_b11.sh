#!/bin/bash
# Round-4 batch 11: conv tests, per-layer backward split, the dX sweep on
# the 1x1 / 13^2 layers, the bench.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b11_tests.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -2 gpurun_out/b11_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bwd_sweep.py --what dx --layers 10,27,44,45,4 > gpurun_out/bwd_dx4.json 2> gpurun_out/bwd_dx4.err || exit $?
echo "dx sweep ok"
timeout -k 10 300 python scripts/conv_bwd_layers.py > gpurun_out/bwd_layers_r4b.json 2> gpurun_out/bwd_layers_r4b.err || exit $?
echo "bwd layers ok"
NOTESTS=1 timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; exit $rc
