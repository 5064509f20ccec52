#!/bin/bash
# conv_tile diagnostic side builds on the 52^2 / 104^2 3x3 layers (timing only)
set -u
mkdir -p gpurun_out
for L in ${LIBS:-base}; do
  if [ $L = base ]; then lib=tensorium_amd/libtensorium_hip.so; else lib=ab/$L/libtensorium_hip.so; fi
  TNS_LIB=$lib timeout -k 10 120 python -u scripts/conv_fwd_layers.py --layers ${LAYERS:-6,11} --reps 20 > gpurun_out/diag_$L.json 2> gpurun_out/diag_$L.err || { tail -3 gpurun_out/diag_$L.err; exit 1; }
  python - "$L" <<'PY'
import json,sys
d=json.loads(open(f'gpurun_out/diag_{sys.argv[1]}.json').read().strip().splitlines()[-1])
print(sys.argv[1], [(r['layer'], r['ms'], r['tflops']) for r in d['layers']])
PY
done
