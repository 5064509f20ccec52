#!/bin/bash
# conv_tile4 diagnostic side builds (ab/ct4d<N>: -DTNS_CT4_STAMPS -DTNS_CT4_DIAG=<N>,
# timing only): warm layer time, per-phase cycles and the held clock
set -u
mkdir -p gpurun_out
for d in ${DIAGS:-0 1 2 3 12 15}; do
  TNS_LIB=ab/ct4d$d/libtensorium_hip.so timeout -k 10 150 python -u scripts/ct4_stamps.py --layer ${LAYERS:-11,28,45} --warm-ms ${WARM:-150} > gpurun_out/ct4d$d.json 2> gpurun_out/ct4d$d.err || { tail -3 gpurun_out/ct4d$d.err; exit 1; }
  python - "$d" <<'PY'
import json,sys
for l in open(f'gpurun_out/ct4d{sys.argv[1]}.json'):
    r=json.loads(l); c=r['cycles_per_tile_wave0']
    print('diag', sys.argv[1], 'L', r['layer'], 'ms', r['layer_ms'], 'GHz', r['clock_ghz_median'], 'cyc/tile', c['total'], 'bar', c['barrier_wait'])
PY
done
