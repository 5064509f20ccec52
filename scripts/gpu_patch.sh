#!/bin/bash
set -u
mkdir -p gpurun_out
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k "patch_variants" > gpurun_out/cpatch_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/cpatch_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for layer in ${LAYERS:-11 28 45 6 3}; do
  timeout -k 10 60 python scripts/conv_one.py --layer $layer --variants=${VARS:--1,100,400,401,402,403,404,405} 2>/dev/null || exit 1
done
