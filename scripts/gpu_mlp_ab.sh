#!/bin/bash
# MNIST train step: parity tests and bench line for side builds (LIBS)
set -u
mkdir -p gpurun_out
for L in ${LIBS:-base}; do
  if [ $L = base ]; then lib=tensorium_amd/libtensorium_hip.so; else lib=ab/$L/libtensorium_hip.so; fi
  TNS_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -x -q --timeout 120 --timeout-method thread > gpurun_out/mlp_tests_$L.log 2>&1
  rc=$?; echo "$L tests rc=$rc"; tail -1 gpurun_out/mlp_tests_$L.log; [ $rc -eq 0 ] || exit $rc
  TNS_LIB=$lib timeout -k 10 300 python bench.py --no-yolo --no-cpu --no-batched --steps 5 --warmup 3 > gpurun_out/bench_mlp_$L.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/bench_mlp_$L.log').read().strip().splitlines()[-1]); print('$L', d['mnist_train'])"
done
