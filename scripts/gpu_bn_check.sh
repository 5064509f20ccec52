#!/bin/bash
# BN / conv / elementwise parity tests, then the bench's elementwise rates
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_conv.py tests/test_gpu_elementwise.py tests/test_gpu_im2col.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu --no-batched --no-mnist > gpurun_out/bench_ew.log 2>&1 || exit 1
python3 - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_ew.log").read().strip().splitlines()[-1])
print({k: (v["achieved"], v["ms"]) for k, v in d["elementwise_roofline"].items() if isinstance(v, dict)})
PY
