#!/bin/bash
# dW tile parity, then per-layer backward calls by forced dW tile: VARS="v:layers ..."
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -k "dw_tiles" -x -q --timeout 240 --timeout-method thread > gpurun_out/dw_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/dw_tests.log; [ $rc -eq 0 ] || exit $rc
for VL in $VARS; do
  v=${VL%%:*}; l=${VL#*:}
  timeout -k 10 120 python -u scripts/conv_bwd_layers.py --layers $l --dw-tile $v > gpurun_out/dw_$v.json 2> gpurun_out/dw_$v.err || { tail -3 gpurun_out/dw_$v.err; exit 1; }
  python - "$v" <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/dw_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], [(r['layer'], r['dw_ms'], r['im2col_ms'], r['call_ms']) for r in d])
PY
done
