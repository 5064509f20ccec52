#!/bin/bash
# ping-pong NN SGEMM diagnostics: form 5 with parts of the staging removed
# (side builds under ab/, timing only) beside form 0 and the real form 5
set -u
mkdir -p gpurun_out
for L in base pp_noa pp_nob pp_noab; do
  if [ $L = base ]; then lib=tensorium_amd/libtensorium_hip.so; else lib=ab/$L/libtensorium_hip.so; fi
  echo "== $L"
  TNS_LIB=$lib timeout -k 10 120 python scripts/nn_big_ab.py --variants 0,5 --rounds 5 > gpurun_out/ppd_$L.json 2>&1 || exit 1
  grep -E '"2|ms_median' gpurun_out/ppd_$L.json
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_sgemm.py tests/test_gpu_host_multi.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pp_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pp_tests.log; exit $rc
