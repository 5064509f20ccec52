#!/bin/bash
# round-6 GPU iteration: SGEMM w4 A/B + bit-exactness, conv slab tests and
# kernel trace; everything under $1
out=${1:-gpurun_out/r6}
mkdir -p "$out"
timeout -k 10 60 ./scripts/w4_probe > "$out/w4probe.json" || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_sgemm.py tests/test_gpu_conv.py -k "nn_big or 4096 or slab or w4" > "$out/test.log" 2>&1 || exit 1
timeout -k 10 400 python -u scripts/sgemm_ab.py --rounds 4 tensorium_amd/libtensorium_hip.so ab/w4a32/libtensorium_hip.so > "$out/sgemm_ab.json" || exit 1
VARS="-1 503 504" timeout -k 10 400 ./scripts/slab_prof.sh "$out/slabprof"
