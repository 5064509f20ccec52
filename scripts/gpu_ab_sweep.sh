set -u
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
LIBS="${LIBS:-base nopre pre}" ROUNDS=2 bash scripts/gpu_ab.sh || exit $?
timeout -k 10 600 python -u scripts/conv_sweep.py --rounds 2 > gpurun_out/conv_sweep.log 2>&1; rc=$?; echo "sweep rc=$rc"; tail -1 gpurun_out/conv_sweep.log
