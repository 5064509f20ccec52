#!/bin/bash
# conv backward A/B: GPU tests on the main build, then per-layer backward
# tables (scripts/conv_bwd_layers.py) for the main build and ab/<name> side
# builds, alternating twice.  Stops on the first failure.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${TESTS:-tests/test_gpu_conv.py tests/test_gpu_sgemm.py} > gpurun_out/bwd_ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/bwd_ab_tests.log; [ $rc -eq 0 ] || exit $rc
for pass in 1 2; do
  for L in ${LIBS:-main base}; do
    if [ $L = main ]; then lib=tensorium_amd/libtensorium_hip.so; else lib=ab/$L/libtensorium_hip.so; fi
    TNS_LIB=$lib timeout -k 10 200 python -u scripts/conv_bwd_layers.py > gpurun_out/bwd_${L}_$pass.json 2> gpurun_out/bwd_${L}_$pass.err || exit 1
  done
  python scripts/cmp_bwd_layers.py gpurun_out/bwd_${REF:-base}_$pass.json gpurun_out/bwd_main_$pass.json
done
