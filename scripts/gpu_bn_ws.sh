#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/bn_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/bn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/bn_perf.py > gpurun_out/bn_perf.json 2>&1; rc=$?; echo "perf rc=$rc"; cut -c1-1500 gpurun_out/bn_perf.json; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_cd_quick.sh
