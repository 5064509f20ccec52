#!/bin/bash
# ping-pong NN SGEMM: parity tests, then A/B against the lock-step form
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_host_multi.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/nn_big_ab.py --n 4096 --rounds 7 --variants 0,5 > gpurun_out/pp_ab4096.json 2>&1
rc=$?; echo "ab rc=$rc"; grep -E '"2|ms_median|exact' gpurun_out/pp_ab4096.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/nn_big_ab.py --n 8192 --rounds 3 --reps 10 --variants 0,5 > gpurun_out/pp_ab8192.json 2>&1
rc=$?; echo "ab8192 rc=$rc"; grep -E '"2|ms_median|exact' gpurun_out/pp_ab8192.json; exit $rc
