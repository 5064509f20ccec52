#!/bin/bash
# dX tile parity, then per-layer backward calls by forced dX tile: VARS="v:layers ..."
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -k "dx_tiles" -x -q --timeout 240 --timeout-method thread > gpurun_out/dx_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/dx_tests.log; [ $rc -eq 0 ] || exit $rc
for VL in $VARS; do
  v=${VL%%:*}; l=${VL#*:}
  timeout -k 10 120 python -u scripts/conv_bwd_layers.py --layers $l --dx-tile $v > gpurun_out/dx_$v.json 2> gpurun_out/dx_$v.err || { tail -3 gpurun_out/dx_$v.err; exit 1; }
  python - "$v" <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/dx_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], [(r['layer'], r['dx_ms'], r['call_ms']) for r in d])
PY
done
