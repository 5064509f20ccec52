#!/bin/bash
# MNIST step A/B between builds: LIBS="base x" (base = the in-tree library)
set -u
mkdir -p gpurun_out
for r in 1 2; do for L in ${LIBS}; do
  if [ $L = base ]; then lib=tensorium_amd/libtensorium_hip.so; else lib=ab/$L/libtensorium_hip.so; fi
  TNS_LIB=$lib timeout -k 10 200 python bench.py --no-yolo --no-cpu --no-batched --steps 5 --warmup 3 > gpurun_out/bench_$L.log 2>&1 || exit 1
  echo "$L $(python3 -c "import json; d=json.loads(open('gpurun_out/bench_$L.log').read().strip().splitlines()[-1]); print(d['mnist_train']['us_per_step'])")"
done; done
