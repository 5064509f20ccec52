#!/bin/bash
# A/Bs (the specialised-wave fused BN; the 1x1 dX on conv1x1.hip), then the
# round-end set (tests, smoke, bench) and the profile passes of the bench
# command, summarised on the box
set -o pipefail
./scripts/gpu_bnb_ws.sh gpurun_out/bnbws || exit 1
mkdir -p gpurun_out/dx1
for r in 1 2; do
  timeout -k 10 200 python -u scripts/conv_bwd_layers.py --layers 2,5,7,10,68 > gpurun_out/dx1/c1_$r.json || exit 1
  TNS_DX_C1=0 timeout -k 10 200 python -u scripts/conv_bwd_layers.py --layers 2,5,7,10,68 > gpurun_out/dx1/base_$r.json || exit 1
done
./scripts/gpu_r6_full.sh gpurun_out/r6final || exit 1
TAG=r06b PROF_ARGS="--steps 20 --warmup 20 --no-cpu" ./scripts/profile_r6.sh
