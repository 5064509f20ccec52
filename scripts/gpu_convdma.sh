#!/bin/bash
# LDS-DMA-ring conv tiles: parity, then the per-layer sweep against the others
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k "dma_variants" > gpurun_out/cdma_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 gpurun_out/cdma_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/conv_tile_sweep.py --rounds 2 --only 100,101,102,300,301,302,303,304 > gpurun_out/cdma_sweep.json 2> gpurun_out/cdma_sweep.err
rc=$?; echo "sweep rc=$rc"; cut -c1-330 gpurun_out/cdma_sweep.err; exit $rc
