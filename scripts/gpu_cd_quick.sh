#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dma_variants" > gpurun_out/cdma_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/cdma_tests.log; [ $rc -eq 0 ] || exit $rc
for layer in ${LAYERS:-11 28 45 6}; do
  timeout -k 10 60 python scripts/conv_one.py --layer $layer --variants=${VARS:--1,100,300,301,302} 2>/dev/null || exit 1
done
