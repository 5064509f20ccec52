#!/bin/bash
# per-layer YOLOv3 forward tables for several side builds (first 4 layers + sum)
set -u
mkdir -p gpurun_out
for L in ${LIBS:-base}; do
  if [ $L = base ]; then lib=tensorium_amd/libtensorium_hip.so; else lib=ab/$L/libtensorium_hip.so; fi
  TNS_LIB=$lib timeout -k 10 200 python -u scripts/conv_fwd_layers.py > gpurun_out/layers_$L.json 2> gpurun_out/layers_$L.err || exit 1
  python - "$L" <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/layers_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], 'sum_ms', d['sum_ms'], [(r['layer'], r['ms']) for r in d['layers'][:4]])
PY
done
