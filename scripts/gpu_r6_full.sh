#!/bin/bash
# the round-end set: the whole -m gpu suite, smoke(), then the default bench line
out=${1:-gpurun_out/r6full}
mkdir -p "$out"
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$out/test.log" 2>&1 || { tail -30 "$out/test.log"; exit 1; }
tail -2 "$out/test.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -1 "$out/smoke.log"
timeout -k 10 900 python -u bench.py > "$out/bench.json" 2> "$out/bench.err"
