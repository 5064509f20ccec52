#!/bin/bash
# dW form sweep on the 13^2 / 26^2 layers (whole backward calls without
# state.delta, HIP events) + the dW form tests
out=${1:-gpurun_out/r6dw}
mkdir -p "$out"
for L in 45 28; do
  timeout -k 10 120 python -u scripts/dw_res_prof.py --layer $L --reps 20 > "$out/l$L.json" || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_conv.py -k "dw_res" > "$out/test.log" 2>&1 || { tail -20 "$out/test.log"; exit 1; }
tail -2 "$out/test.log"
