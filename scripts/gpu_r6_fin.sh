#!/bin/bash
# fused-finish BN backward + W^T-reading 1x1 dX: tests, train backward A/B, bench line
out=${1:-gpurun_out/r6fin}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_train.py tests/test_gpu_train_net.py tests/test_gpu_conv.py tests/test_gpu_configs.py tests/test_darknet.py > "$out/test.log" 2>&1 || { tail -30 "$out/test.log"; exit 1; }
tail -1 "$out/test.log"
for r in 1 2; do
  timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/fused$r.txt" || exit 1
  TNS_BN_FUSED=0 timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/three$r.txt" || exit 1
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 20 --no-cpu > "$out/bench.json" 2> "$out/bench.err"
