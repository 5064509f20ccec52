#!/bin/bash
# NN big-kernel A/B over side builds: LIBS="base name ..." VARS=0,5 N=4096
set -u
mkdir -p gpurun_out
for L in ${LIBS:-base}; do
  if [ $L = base ]; then lib=tensorium_amd/libtensorium_hip.so; else lib=ab/$L/libtensorium_hip.so; fi
  echo "== $L"
  TNS_LIB=$lib timeout -k 10 120 python scripts/nn_big_ab.py --n ${N:-4096} --variants ${VARS:-0,5} --rounds ${ROUNDS:-5} > gpurun_out/ab_$L.json 2>&1 || { tail -5 gpurun_out/ab_$L.json; exit 1; }
  grep -E '"2|ms_median' gpurun_out/ab_$L.json
done
