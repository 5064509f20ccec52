#!/bin/bash
# Round-4 batch 12: image-folded dw_res on the 13^2 planes, the 208^2->104^2
# dX tile: conv tests, forms on layers 45 / 43, the bench.
set -u
mkdir -p gpurun_out/dwres6
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b12_tests.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -2 gpurun_out/b12_tests.log; [ $rc -eq 0 ] || exit $rc
for L in 45 43; do
  timeout -k 10 120 python scripts/dw_res_prof.py --layer $L > gpurun_out/dwres6/l$L.json 2> gpurun_out/dwres6/l$L.err || exit $?
  echo "layer $L ok"; cat gpurun_out/dwres6/l$L.json
done
NOTESTS=1 timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; exit $rc
