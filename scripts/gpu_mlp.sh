#!/bin/bash
# MNIST fused-step loop: train tests, stage stamps (diagnostic build), bench line.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mlp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/mlp_tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TNS_LIB=ab/stamps/libtensorium_hip.so timeout -k 10 120 python scripts/mlp_stamps.py > gpurun_out/mlp_stamps.log 2>&1
rc=$?; echo "stamps rc=$rc"; cat gpurun_out/mlp_stamps.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-yolo --no-cpu --no-batched --steps 5 --warmup 3 > gpurun_out/bench_mlp.log 2>&1
rc=$?; echo "bench rc=$rc"; python3 -c "
import json; d=json.loads(open('gpurun_out/bench_mlp.log').read().strip().splitlines()[-1]); print(d['mnist_train'])"
