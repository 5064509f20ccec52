#!/bin/bash
# the rearrangement chunk rule: whole -m gpu suite, then training backward and
# bench with the rule / with 2048 everywhere (TNS_RES_CHL=2048), interleaved
out=${1:-gpurun_out/reschl2}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/test.log" 2>&1 || { tail -30 "$out/test.log"; exit 1; }
tail -1 "$out/test.log"
for r in 1 2; do
  timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/rule_$r.txt" || exit 1
  TNS_RES_CHL=2048 timeout -k 10 120 python -u scripts/train_bwd_once.py --passes 8 > "$out/c2048_$r.txt" || exit 1
done
timeout -k 10 600 python -u bench.py > "$out/bench_rule.json" 2> "$out/bench_rule.err" || exit 1
TNS_RES_CHL=2048 timeout -k 10 600 python -u bench.py > "$out/bench_2048.json" 2> "$out/bench_2048.err" || exit 1
