#!/bin/bash
# gpu tests + sgemm sweep + bench (no profiling).  Stops on crash/timeout.
set -u
mkdir -p gpurun_out
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 600 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log; ok $rc || exit $rc
if [ -n "${SWEEP:-}" ]; then
  timeout -k 10 600 python scripts/sgemm_sweep.py $SWEEP > gpurun_out/sweep.log 2>&1
  rc=$?; echo "sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/sweep.log | tail -25; ok $rc || exit $rc
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
