#!/bin/bash
# slab fill: uniform-k form (product) vs the per-lane form (A/B), tests first
out=${1:-gpurun_out/fill}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py -k "slab" tests/test_gpu_configs.py > "$out/test.log" 2>&1 || { tail -20 "$out/test.log"; exit 1; }
tail -1 "$out/test.log"
cd /tmp && export TMPDIR=/tmp
for r in 1 2; do
  for v in u lane; do
    if [ $v = lane ]; then export TNS_LIB=$GRAFT_REPO_ROOT/ab/filllane/libtensorium_hip.so; else unset TNS_LIB; fi
    timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$out/t_${v}_$r -o run -- \
      python3 $GRAFT_REPO_ROOT/scripts/conv_fwd_layers.py --layers 28,45 --reps 20 --warm-ms 30 > $GRAFT_REPO_ROOT/$out/${v}_$r.json || exit 1
    python3 $GRAFT_REPO_ROOT/scripts/trace_summary.py $GRAFT_REPO_ROOT/$out/t_${v}_$r slab > $GRAFT_REPO_ROOT/$out/${v}_$r.txt
    rm -rf $GRAFT_REPO_ROOT/$out/t_${v}_$r
  done
done
