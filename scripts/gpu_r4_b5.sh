#!/bin/bash
# Round-4 batch 5: BN chain kernels (two-tiles-ahead staging): tests + perf
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -k "batchnorm or bn or means or var or dots or sums or normalize" > gpurun_out/b5_tests.log 2>&1
rc=$?; echo "bn tests rc=$rc"; tail -3 gpurun_out/b5_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/bn_perf.py > gpurun_out/bn_perf_r4b.json 2> gpurun_out/bn_perf_r4b.err || exit $?
echo "bn perf ok"; cat gpurun_out/bn_perf_r4b.json
