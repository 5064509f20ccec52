#!/bin/bash
# Round-4 batch 15: dw_res last k-tile by 8, XCD-contiguous tiles, 16-byte col' writes:
# kernels on layers 3 / 4 / 6 / 9 / 11 / 28 under a kernel trace, the bench.
set -u
mkdir -p gpurun_out/dwres9
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/b15_tests.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -2 gpurun_out/b15_tests.log; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
for L in 45 28 11 3; do
  (cd /tmp && timeout -k 10 150 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/dwres9/l$L -o l$L --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/dw_res_prof.py --layer $L > $GRAFT_REPO_ROOT/gpurun_out/dwres9/l$L.json 2> $GRAFT_REPO_ROOT/gpurun_out/dwres9/l$L.err) || exit $?
  echo "layer $L ok"; cat gpurun_out/dwres9/l$L.json | cut -c1-400
done
timeout -k 10 300 python scripts/conv_bwd_layers.py > gpurun_out/bwd_layers_b15.json 2> gpurun_out/bwd_layers_b15.err || exit $?
echo "bwd layers ok"
NOTESTS=1 timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c1-200; exit $rc
