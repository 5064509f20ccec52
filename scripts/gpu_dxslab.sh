#!/bin/bash
# dX on the slab GEMM: per-layer backward calls (joined, telemetry split) by
# forced form on the TN + col2im layers
out=${1:-gpurun_out/dxslab}
mkdir -p "$out"
for v in -2 0 1 2 3 4 5; do
  timeout -k 10 200 python -u scripts/conv_bwd_layers.py --dx-slab $v --layers 9,26,28,43,45,57,62 > "$out/v$v.json" || exit 1
done
