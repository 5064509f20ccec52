#!/bin/bash
set -u
mkdir -p gpurun_out
for L in ${LIBS:-base cd_noa cd_nob}; do
  if [ $L = base ]; then lib=tensorium_amd/libtensorium_hip.so; else lib=ab/$L/libtensorium_hip.so; fi
  echo "== $L"
  for layer in ${LAYERS:-11 28 45}; do
    TNS_LIB=$lib timeout -k 10 60 python scripts/conv_one.py --layer $layer --variants=${VARS:-100,300,301,302} 2>/dev/null || exit 1
  done
done
