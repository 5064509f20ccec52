#!/bin/bash
# fused BN backward: tests, then train backward passes fused / three-pass (A/B)
out=${1:-gpurun_out/bnb}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_train.py tests/test_gpu_train_net.py tests/test_gpu_conv.py > "$out/test.log" 2>&1 || { tail -30 "$out/test.log"; exit 1; }
tail -2 "$out/test.log"
for r in 1 2; do
  timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/fused$r.txt" || exit 1
  TNS_BN_FUSED=0 timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/three$r.txt" || exit 1
done
