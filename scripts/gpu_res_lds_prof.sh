#!/bin/bash
# im2col_res_lds alone: kernel stats of the dW form sweep on layers 3 (208^2), 6 (104^2), 11 (52^2)
out=${1:-gpurun_out/reslds}
R=$GRAFT_REPO_ROOT
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for L in 3 6 11; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/l$L -o run -- python3 $R/scripts/dw_res_prof.py --layer $L --reps 5 > $R/$out/l$L.log 2>&1 || exit 1
  f=$(ls $R/$out/l$L/run_kernel_stats.csv $R/$out/l$L/*/run_kernel_stats.csv 2>/dev/null | head -1)
  cp $f $R/$out/l$L.stats.csv
  rm -rf $R/$out/l$L
done
