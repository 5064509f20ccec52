#!/bin/bash
# Round-4 batch 29: every dX form on one layer of each class (warm clock
# before the default timing).
set -u
mkdir -p gpurun_out
timeout -k 10 900 python scripts/bwd_sweep.py --what dx --layers 5,6,10,11,27,28,44,45 > gpurun_out/bwd_dx_sweep_r4.json 2> gpurun_out/bwd_dx_sweep_r4.err
rc=$?; echo "sweep rc=$rc"; cut -c1-2000 gpurun_out/bwd_dx_sweep_r4.json; exit $rc
