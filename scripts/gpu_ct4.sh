#!/bin/bash
# conv_tile4 parity (every conv tile variant) then per-layer timing by forced variant
# VARS="v:layers ..." (variant -1 = the heuristic)
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -k "tile_variants" -x -q --timeout 240 --timeout-method thread > gpurun_out/ct4_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ct4_tests.log; [ $rc -eq 0 ] || exit $rc
for VL in $VARS; do
  v=${VL%%:*}; l=${VL#*:}
  timeout -k 10 120 python -u scripts/conv_fwd_layers.py --layers $l --reps 20 --warm-ms ${WARM:-0} --variant $v > gpurun_out/ct4_$v.json 2> gpurun_out/ct4_$v.err || { tail -3 gpurun_out/ct4_$v.err; exit 1; }
  python - "$v" <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/ct4_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], [(r['layer'], r['ms'], r['tflops']) for r in d['layers']])
PY
done
