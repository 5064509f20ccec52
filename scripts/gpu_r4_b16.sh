#!/bin/bash
# Round-4 batch 16: the 75-layer backward per call vs replayed from a HIP
# graph (overlap on / off), bit-identity of the replay; the bench.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bwd_graph.py --steps 5 --rounds 3 > gpurun_out/bwd_graph.json 2> gpurun_out/bwd_graph.err
rc=$?; echo "bwd_graph rc=$rc"; cat gpurun_out/bwd_graph.json; tail -3 gpurun_out/bwd_graph.err; exit $rc
