#!/bin/bash
# sgemm + conv tests, conv sweep, 4096 sgemm sweep of the production shapes.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_sgemm.py tests/test_gpu_conv.py -q -x > gpurun_out/perf_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/perf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/conv_sweep.py ${SWEEP_ARGS:-} > gpurun_out/conv_sweep.log 2>&1
rc=$?; echo "conv sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/conv_sweep.log | tail -26; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/sgemm_sweep.py --sizes 4096 --variants ${VARIANTS:-0,1,2,5,6} > gpurun_out/sweep.log 2>&1
rc=$?; echo "sgemm sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/sweep.log | tail -3; exit $rc
