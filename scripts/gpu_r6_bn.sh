#!/bin/bash
# BN backward check: the train / conv / whole-net train tests, then a bench
# line without the CPU legs
out=${1:-gpurun_out/r6bn}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_train.py tests/test_gpu_train_net.py tests/test_gpu_conv.py \
  tests/test_gpu_elementwise.py > "$out/test.log" 2>&1 || { tail -30 "$out/test.log"; exit 1; }
tail -3 "$out/test.log"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 20 --no-cpu > "$out/bench.json" 2> "$out/bench.err"
