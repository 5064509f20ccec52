#!/bin/bash
# conv forward product check after a pick change: the 75-layer and network
# tests, the conv test file, then a bench line without the CPU legs
out=${1:-gpurun_out/r6conv}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_configs.py tests/test_darknet.py tests/test_gpu_conv.py > "$out/test.log" 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 20 --no-cpu > "$out/bench.json" 2> "$out/bench.err"
