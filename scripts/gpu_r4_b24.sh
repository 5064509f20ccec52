#!/bin/bash
# Round-4 batch 24: the pipelined schedule with the lazy-join hazard guard: every GPU test,
# short-row stores), layer-45 dW forms under a kernel trace, the schedules'
# timing and bit-identity, the bench.
set -u
mkdir -p gpurun_out/dwres11
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dwres11/l45 -o l45 --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/dw_res_prof.py --layer 45 > $GRAFT_REPO_ROOT/gpurun_out/dwres11/l45.json 2> $GRAFT_REPO_ROOT/gpurun_out/dwres11/l45.err) || exit $?
echo "layer 45 ok"; cut -c1-300 gpurun_out/dwres11/l45.json
timeout -k 10 300 python scripts/bwd_graph.py --steps 5 --rounds 2 > gpurun_out/bwd_graph5.json 2> gpurun_out/bwd_graph5.err || exit $?
echo "bwd_graph ok"; cat gpurun_out/bwd_graph5.json
NOTESTS=1 timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; exit $rc
