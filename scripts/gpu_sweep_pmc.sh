#!/bin/bash
# tests -> conv sweep (CONV_VARIANTS) -> SQ PMC passes on LAYERS
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u scripts/conv_sweep.py --rounds 2 > gpurun_out/conv_sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -1 gpurun_out/conv_sweep.log; [ $rc -eq 0 ] || exit $rc
for L in ${LAYERS:-}; do
  NAME=l$L bash scripts/pmc_run.sh scripts/conv_only.py --layer $L --reps 20 > gpurun_out/pmc_l$L.txt 2>&1
  rc=$?; echo "pmc l$L rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
