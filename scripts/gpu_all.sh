#!/bin/bash
# all GPU tests, then the elementwise sweep
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/elementwise_perf.py > gpurun_out/ew.json 2> gpurun_out/ew.err
rc=$?; tail -2 gpurun_out/ew.err; exit $rc
