#!/bin/bash
# Round-4 batch 27: every dW form on the first layers and the 104^2 1x1 layer
# (warm clock before the default timing).
set -u
mkdir -p gpurun_out
timeout -k 10 600 python scripts/bwd_sweep.py --what dw --layers 0,1,2,3,5,9 > gpurun_out/bwd_dw_sweep_r4.json 2> gpurun_out/bwd_dw_sweep_r4.err
rc=$?; echo "sweep rc=$rc"; cut -c1-3000 gpurun_out/bwd_dw_sweep_r4.json; exit $rc
