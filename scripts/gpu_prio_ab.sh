#!/bin/bash
# train backward passes: product / side stream at low priority / chain waves
# at issue priority / both (interleaved twice)
out=${1:-gpurun_out/prio}
mkdir -p "$out"
for r in 1 2; do
  timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/base$r.txt" || exit 1
  TNS_STREAM_PRIO=1 timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/sprio$r.txt" || exit 1
  TNS_LIB=ab/cprio/libtensorium_hip.so timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/cprio$r.txt" || exit 1
  TNS_STREAM_PRIO=1 TNS_LIB=ab/cprio/libtensorium_hip.so timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/both$r.txt" || exit 1
done
