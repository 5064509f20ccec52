#!/bin/bash
# kernel trace of conv slab forms on one 13^2 and one 26^2 layer: fill vs
# GEMM per form (rocprofv3 --kernel-trace, csv), warm clock
out=${1:-gpurun_out/slabprof}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for v in ${VARS:-503 504}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$out/v$v" -o run -- \
    python3 "$GRAFT_REPO_ROOT/scripts/conv_fwd_layers.py" --variant $v --layers ${LAYERS:-45,28} \
    --reps 20 --warm-ms 30 > "$GRAFT_REPO_ROOT/$out/v$v.json" || exit 1
done
