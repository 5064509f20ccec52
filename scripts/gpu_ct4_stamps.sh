#!/bin/bash
# conv_tile4 phase stamps (ab/ct4s: -DTNS_CT4_STAMPS) per forced variant: VARS="v ..."
set -u
mkdir -p gpurun_out
for v in ${VARS:--1}; do
  TNS_LIB=ab/ct4s/libtensorium_hip.so timeout -k 10 150 python -u scripts/ct4_stamps.py --layer ${LAYERS:-11} --variant $v --warm-ms ${WARM:-100} > gpurun_out/ct4s_$v.json 2> gpurun_out/ct4s_$v.err || { tail -3 gpurun_out/ct4s_$v.err; exit 1; }
  python - "$v" <<'PY'
import json,sys
for l in open(f'gpurun_out/ct4s_{sys.argv[1]}.json'):
    r=json.loads(l)
    print('v', sys.argv[1], 'L', r['layer'], 'ms', r['layer_ms'], 'GHz', r['clock_ghz_median'], r['cycles_per_tile_wave0'])
PY
done
