#!/bin/bash
# Round-4 batch 25: short-row rearrangement up to 1024 (26^2): every GPU test,
# short-row stores), layer-45 dW forms under a kernel trace, the schedules'
# timing and bit-identity, the bench.
set -u
mkdir -p gpurun_out/dwres12
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dwres12/l28 -o l28 --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/dw_res_prof.py --layer 28 > $GRAFT_REPO_ROOT/gpurun_out/dwres12/l28.json 2> $GRAFT_REPO_ROOT/gpurun_out/dwres12/l28.err) || exit $?
echo "layer 28 ok"; cut -c1-300 gpurun_out/dwres12/l28.json
timeout -k 10 300 python scripts/bwd_graph.py --steps 5 --rounds 2 > gpurun_out/bwd_graph6.json 2> gpurun_out/bwd_graph6.err || exit $?
echo "bwd_graph ok"; cat gpurun_out/bwd_graph6.json
NOTESTS=1 timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; exit $rc
