#!/bin/bash
# conv GPU tests + conv schedule sweep.  Stops on crash/timeout.
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_conv.py -q -x > gpurun_out/gpu_conv_tests.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -5 gpurun_out/gpu_conv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python scripts/conv_sweep.py ${SWEEP_ARGS:-} > gpurun_out/conv_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; grep -v amdgpu.ids gpurun_out/conv_sweep.log | tail -40; exit $rc
