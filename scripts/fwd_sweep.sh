#!/bin/bash
# conv forward variants on chosen YOLOv3 layers (scripts/conv_fwd_layers.py,
# warm clock): one JSON line per variant under $1; VARS / LAYERS from the env
out=${1:-gpurun_out/fwdsweep}
mkdir -p "$out"
for v in ${VARS:--1}; do
  timeout -k 10 120 python -u scripts/conv_fwd_layers.py --variant $v --layers ${LAYERS:-10,27} \
    --warm-ms 30 --reps 20 > "$out/v$v.json" || exit 1
done
