#!/bin/bash
# Round-4 batch 10: the 32-row dX conv form (layer 3), dw_res on the 1x1
# layers: tests, per-layer forms, the dX sweep on layer 3, the bench.
set -u
mkdir -p gpurun_out/dwres5
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b10_tests.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -2 gpurun_out/b10_tests.log; [ $rc -eq 0 ] || exit $rc
for L in 10 27 44 5; do
  timeout -k 10 120 python scripts/dw_res_prof.py --layer $L > gpurun_out/dwres5/l$L.json 2> gpurun_out/dwres5/l$L.err || exit $?
  echo "layer $L ok"; cat gpurun_out/dwres5/l$L.json
done
timeout -k 10 200 python scripts/bwd_sweep.py --what dx --layers 3 > gpurun_out/bwd_dx3.json 2> gpurun_out/bwd_dx3.err || exit $?
echo "dx l3 ok"; cat gpurun_out/bwd_dx3.json | cut -c1-600
NOTESTS=1 timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; exit $rc
