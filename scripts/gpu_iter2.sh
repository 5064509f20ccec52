#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/conv_sweep.py --rounds 2 > gpurun_out/conv_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/conv_sweep.log | tail -25; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u scripts/sgemm_sweep.py --sizes 4096 --variants ${SV:-5,17,16,0} --rounds 5 > gpurun_out/sgemm_sweep.log 2>&1
rc=$?; echo "ssweep rc=$rc"; grep -v amdgpu.ids gpurun_out/sgemm_sweep.log | tail -12
