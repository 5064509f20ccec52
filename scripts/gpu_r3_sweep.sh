#!/bin/bash
# Round 3: plain-GEMM tile heuristic check (strided-batched NN at the YOLOv3
# conv-GEMM shapes + FC / generic shapes), then the SGEMM parity tests.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/sgemm_sweep.py --sizes 2048 --yolo --rounds 3 \
  --shapes "32,4096,4096;32,784,64;32,64,784;256,256,256;1000,1000,1000;512,512,512;128,4096,4096;64,4096,4096;1024,1024,1024;96,4096,1024" \
  > gpurun_out/sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -30 gpurun_out/sweep.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_sgemm.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_sgemm.log; exit $rc
