#!/bin/bash
# conv_slab forms against the default pick on the 13^2 / 26^2 YOLOv3 layers
# (scripts/conv_fwd_layers.py, warm clock); one JSON line per variant
out=${1:-gpurun_out/slab}
mkdir -p "$out"
for v in -1 500 501 502 503 504 505; do
  timeout -k 10 120 python -u scripts/conv_fwd_layers.py --variant $v --layers ${LAYERS:-26,28,43,45,47,44} \
    --warm-ms 50 --reps 20 > "$out/v$v.json" || exit 1
done
