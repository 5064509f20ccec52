#!/bin/bash
# tests -> A/B quick_perf over LIBS -> optional sgemm sweep (SV variants)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="${LIBS:-base cur}" ROUNDS=${ROUNDS:-2} bash scripts/gpu_ab.sh || exit $?
if [ -n "${SV:-}" ]; then
  timeout -k 10 600 python -u scripts/sgemm_sweep.py --sizes ${SIZES:-4096} --variants $SV --rounds 5 > gpurun_out/sgemm_sweep.log 2>&1
  rc=$?; echo "ssweep rc=$rc"; grep -v amdgpu.ids gpurun_out/sgemm_sweep.log | tail -12
fi
