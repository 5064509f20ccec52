#!/bin/bash
# residue-register dW forms: parity tests, then per-shape timing
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_sgemm.py -k "sdot" tests/test_gpu_conv.py::test_conv_backward_dw_rc_forms > gpurun_out/dw_rc_tests.log 2>&1 || { tail -30 gpurun_out/dw_rc_tests.log; exit 1; }
tail -3 gpurun_out/dw_rc_tests.log
timeout -k 10 300 python scripts/dw_forms.py ${LAYERS:+--layers $LAYERS} > gpurun_out/dw_forms.json 2> gpurun_out/dw_forms.err || { tail -20 gpurun_out/dw_forms.err; exit 1; }
cat gpurun_out/dw_forms.err
