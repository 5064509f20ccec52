#!/bin/bash
# train backward: fused BN everywhere / fused below 16384 pixels / three-pass (A/B, 3 rounds)
out=${1:-gpurun_out/bnbws}
mkdir -p "$out"
for r in 1 2 3; do
  timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/all$r.txt" || exit 1
  TNS_BN_WS=0 timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/small$r.txt" || exit 1
  TNS_BN_FUSED=0 timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/three$r.txt" || exit 1
done
