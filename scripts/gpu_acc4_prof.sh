#!/bin/bash
# kernel stats of 3 training backward passes, float4 and scalar dW accumulate
out=${1:-gpurun_out/acc4p}
R=$GRAFT_REPO_ROOT
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/a -o run -- python3 $R/scripts/train_bwd_once.py --passes 3 > $R/$out/a.log 2>&1 || exit 1
TNS_ACC4=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/s -o run -- python3 $R/scripts/train_bwd_once.py --passes 3 > $R/$out/s.log 2>&1 || exit 1
cd $R
for m in a s; do f=$(ls $out/$m/*/run_kernel_stats.csv 2>/dev/null || ls $out/$m/run_kernel_stats.csv); grep -E "accumulate|Name" $f > $out/$m.stats; done
find $out/a $out/s -name '*kernel_trace.csv' -delete
