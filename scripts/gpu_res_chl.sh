#!/bin/bash
# im2col_res_lds chunk A/B (TNS_RES_CHL=1024 vs the default 2048 on rows >= 2048):
# the dW form tests with 1024, then kernel stats of the dW form sweep per layer
out=${1:-gpurun_out/reschl}
R=$GRAFT_REPO_ROOT
mkdir -p "$out"
TNS_RES_CHL=1024 timeout -k 10 400 python -u -m pytest -x -q --timeout 250 --timeout-method thread \
  tests/test_gpu_conv.py tests/test_gpu_train_net.py > "$out/test.log" 2>&1 || { tail -20 "$out/test.log"; exit 1; }
tail -1 "$out/test.log"
cd /tmp && export TMPDIR=/tmp
for L in 1 3 6 11; do
  for C in 1024 2048; do
    TNS_RES_CHL=$C timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$out/l${L}_$C -o run -- python3 $R/scripts/dw_res_prof.py --layer $L --reps 5 > $R/$out/l${L}_$C.log 2>&1 || exit 1
    f=$(ls $R/$out/l${L}_$C/run_kernel_stats.csv $R/$out/l${L}_$C/*/run_kernel_stats.csv 2>/dev/null | head -1)
    grep -E "Name|res_lds" $f > $R/$out/l${L}_$C.stats.csv
    rm -rf $R/$out/l${L}_$C
  done
done
