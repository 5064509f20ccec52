#!/bin/bash
# per-layer conv forward (warm clock, current picks) and per-layer conv
# backward (joined, telemetry split) for YOLOv3 batch 8
out=${1:-gpurun_out/r6layers}
mkdir -p "$out"
timeout -k 10 300 python -u scripts/conv_fwd_layers.py --warm-ms 30 --reps 20 > "$out/fwd.json" || exit 1
timeout -k 10 300 python -u scripts/conv_bwd_layers.py > "$out/bwd.json" || exit 1
