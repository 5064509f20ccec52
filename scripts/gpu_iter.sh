#!/bin/bash
# Iteration check: gpu tests -> conv sweep (optional) -> bench (no CPU leg).
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
if [ "${SWEEP:-0}" = "1" ]; then
  timeout -k 10 600 python -u scripts/conv_sweep.py --rounds 2 > gpurun_out/conv_sweep.log 2>&1
  rc=$?; echo "sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/conv_sweep.log | tail -25; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 600 python -u bench.py --no-cpu ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
