#!/bin/bash
# Round-4 experiment batch: SGEMM one-wave-per-SIMD forms, conv addtid forms,
# backward form sweep, then the whole GPU suite.  Each step bounded; stop at
# the first failure.
set -u
mkdir -p gpurun_out
timeout -k 10 240 python scripts/nn_big_ab.py --variants 5,6 --rounds 5 > gpurun_out/ab_w4.json 2> gpurun_out/ab_w4.err || exit $?
echo "ab ok"; tail -2 gpurun_out/ab_w4.json
timeout -k 10 300 python scripts/conv_tile_sweep.py --rounds 2 --only 105,107,112,117,122,125,129,130,131,132,133,134,135 > gpurun_out/ct_sweep_at.json 2> gpurun_out/ct_sweep_at.err || exit $?
echo "conv sweep ok"
timeout -k 10 400 python scripts/bwd_sweep.py > gpurun_out/bwd_sweep.json 2> gpurun_out/bwd_sweep.err || exit $?
echo "bwd sweep ok"
timeout -k 10 120 python scripts/bn_perf.py > gpurun_out/bn_perf_r4.json 2> gpurun_out/bn_perf_r4.err || exit $?
echo "bn perf ok"
NOBENCH=1 bash scripts/gpu_r4_check.sh || exit $?
