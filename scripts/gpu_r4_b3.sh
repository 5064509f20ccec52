#!/bin/bash
# Round-4 batch 3: residue-sequential dW (tests, per-layer forms), then the
# SGEMM bench profile (kernel trace + PMC passes) for profiles/r04_*.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread -k "dw_res or dx_conv or yolov3_batch8 or overlap or dw_auto or caller_workspace or matches_oracle or dw_tiles" > gpurun_out/b3_tests.log 2>&1
rc=$?; echo "targeted tests rc=$rc"; tail -3 gpurun_out/b3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/bwd_sweep.py --what dw --layers 6,9,11,26,28,43,45,4 > gpurun_out/bwd_dw.json 2> gpurun_out/bwd_dw.err || exit $?
echo "bwd dw sweep ok"
TAG=r04 bash scripts/profile.sh || exit $?
echo "profile ok"
