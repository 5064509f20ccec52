#!/bin/bash
# A/B perf of alternative builds under ab/<name>/ (interleaved rounds, one
# process per build per round), plus optional probe binaries.
#   LIBS="base kp" ROUNDS=2 PROBE=1 bash scripts/gpu_ab.sh
set -u
mkdir -p gpurun_out
if [ "${PROBE:-0}" = "1" ]; then
  timeout -k 10 60 ./scripts/probe/mfma_order > gpurun_out/probe.log 2>&1; rc=$?; cat gpurun_out/probe.log; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for L in ${LIBS}; do
    TNS_LIB=ab/$L/libtensorium_hip.so timeout -k 10 300 python -u scripts/quick_perf.py --tag $L ${QP_ARGS:-} >> gpurun_out/ab.jsonl 2> gpurun_out/ab_$L.err
    rc=$?; [ $rc -eq 0 ] || { echo "$L rc=$rc"; tail -5 gpurun_out/ab_$L.err; exit $rc; }
  done
done
python3 - <<'PY'
import json
rows=[json.loads(l) for l in open("gpurun_out/ab.jsonl")]
for r in rows:
    print(r["tag"], {k: v for k, v in r.items() if k not in ("tag", "yolo_layers_ms")})
PY
