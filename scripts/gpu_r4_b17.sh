#!/bin/bash
# Round-4 batch 17: the pipelined backward schedule (TNS_OPT_BWD_OVERLAP = 2):
# conv tests (its chain test included), the 75-layer timing of every schedule.
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b17_tests.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -2 gpurun_out/b17_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/bwd_graph.py --steps 5 --rounds 3 > gpurun_out/bwd_graph2.json 2> gpurun_out/bwd_graph2.err
rc=$?; echo "bwd_graph rc=$rc"; cat gpurun_out/bwd_graph2.json; exit $rc
