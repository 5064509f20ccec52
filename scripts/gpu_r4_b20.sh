#!/bin/bash
# Round-4 batch 20: state.delta of the stride-2 layers as parity-class
# transposed convolutions: conv tests, the dX forms on layers 1/4/9/26/43,
# the bench.
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b20_tests.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -2 gpurun_out/b20_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bwd_sweep.py --what dx --layers 1,4,9,26,43 > gpurun_out/bwd_dx_s2.json 2> gpurun_out/bwd_dx_s2.err || exit $?
echo "dx s2 sweep ok"; cat gpurun_out/bwd_dx_s2.json | cut -c1-1500
timeout -k 10 300 python scripts/bwd_graph.py --steps 5 --rounds 2 > gpurun_out/bwd_graph3.json 2> gpurun_out/bwd_graph3.err || exit $?
echo "bwd_graph ok"; cat gpurun_out/bwd_graph3.json
NOTESTS=1 timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; exit $rc
