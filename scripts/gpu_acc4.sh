#!/bin/bash
# float4 dW accumulate: tests, train backward passes float4 / scalar (A/B), then bench both
out=${1:-gpurun_out/acc4}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_train.py tests/test_gpu_train_net.py tests/test_gpu_conv.py > "$out/test.log" 2>&1 || { tail -30 "$out/test.log"; exit 1; }
tail -2 "$out/test.log"
for r in 1 2; do
  timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/acc4_$r.txt" || exit 1
  TNS_ACC4=0 timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/scalar_$r.txt" || exit 1
done
timeout -k 10 600 python -u bench.py > "$out/bench_acc4.json" 2> "$out/bench_acc4.err" || exit 1
TNS_ACC4=0 timeout -k 10 600 python -u bench.py > "$out/bench_scalar.json" 2> "$out/bench_scalar.err" || exit 1
