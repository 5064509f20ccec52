#!/bin/bash
# conv / sgemm GPU tests, then the per-layer YOLOv3 forward table
set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_sgemm.py ${EXTRA_TESTS:-} -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_conv_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/gpu_conv_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/conv_fwd_layers.py > gpurun_out/conv_fwd_layers.json 2> gpurun_out/conv_fwd_layers.err
rc=$?; echo "layers rc=$rc"; [ $rc -eq 0 ] || exit $rc
python - <<'PY'
import json
d=json.loads(open('gpurun_out/conv_fwd_layers.json').read().strip().splitlines()[-1])
print('sum_ms', d['sum_ms']); print([ (r['layer'], r['ms'], r['tflops']) for r in d['layers'][:4]])
PY
