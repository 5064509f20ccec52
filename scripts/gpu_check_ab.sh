#!/bin/bash
# smoke + GPU tests + default bench (optional), then nn_big A/B over side builds
set -u
mkdir -p gpurun_out
if [ "${CHECK:-1}" = "1" ]; then
  timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
fi
for L in ${LIBS:-}; do
  if [ $L = base ]; then lib=tensorium_amd/libtensorium_hip.so; else lib=ab/$L/libtensorium_hip.so; fi
  echo "== $L"; TNS_LIB=$lib timeout -k 10 120 python scripts/nn_big_ab.py --variants 0 --rounds 5 ${NB_ARGS:-} > gpurun_out/ab_$L.json 2>&1 || exit 1
  grep -A1 '"256x256x32_w2x4' gpurun_out/ab_$L.json | grep ms_median
done
