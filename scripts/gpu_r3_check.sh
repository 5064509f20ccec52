#!/bin/bash
# Round 3: heuristic sweep, the whole GPU suite, then the default bench line.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/sgemm_sweep.py --sizes 2048 --yolo --rounds 3 \
  --shapes "32,4096,4096;32,784,64;32,64,784;256,256,256;1000,1000,1000;512,512,512;128,4096,4096;64,4096,4096;1024,1024,1024;96,4096,1024" \
  > gpurun_out/sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log; exit $rc
