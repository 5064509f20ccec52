#!/bin/bash
# im2col parity tests, then the elementwise HBM-rate sweep (scripts/elementwise_perf.py)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_im2col.py tests/test_gpu_conv.py tests/test_gpu_large.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ew_tests.log 2>&1
rc=$?; tail -2 gpurun_out/ew_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/elementwise_perf.py > gpurun_out/ew.json 2> gpurun_out/ew.err
rc=$?; tail -2 gpurun_out/ew.err; exit $rc
