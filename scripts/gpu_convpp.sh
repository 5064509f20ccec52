#!/bin/bash
# ping-pong conv tiles: parity, then the per-layer sweep against the others
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 120 --timeout-method thread -k "pp_variants or tile_variants" > gpurun_out/cpp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/cpp_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/conv_tile_sweep.py --rounds 2 > gpurun_out/cpp_sweep.json 2> gpurun_out/cpp_sweep.err
rc=$?; echo "sweep rc=$rc"; cat gpurun_out/cpp_sweep.err | cut -c1-400; exit $rc
