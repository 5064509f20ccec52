#!/bin/bash
# Round-5 GPU batch: STEPS selects the steps (space-separated names).
#   tests   — pytest -m gpu (whole suite, or TESTK=<pytest -k expression>)
#   diagtests — the variant sweeps against the ab/diag build (TNS_DIAG=1:
#             the measured, not picked forms included)
#   mlpst   — MNIST fused-step stage stamps (ab/mlpst: -DTNS_MLP_STAMPS)
#   bnab    — BN reduction rates (bn_perf.py) for LIBS
#   abfwd   — conv forward A/B: LIBS builds under ab/ (+ "main" = the tree)
#   bwdab   — conv backward schedules (bwd_graph.py) for LIBS
#   bench   — python bench.py (default flags) -> gpurun_out/bench.json
#   stamps  — conv_tile4 phase stamps (ab/stamps build) for LAYERS
#   trace   — rocprofv3 kernel trace of BENCH_ARGS -> gpurun_out/prof_trace
set -u
mkdir -p gpurun_out
lib_of() { [ "$1" = main ] && echo tensorium_amd/libtensorium_hip.so || echo ab/$1/libtensorium_hip.so; }
for S in ${STEPS}; do
  case $S in
    tests)
      if [ -n "${TESTK:-}" ]; then KARG=(-k "$TESTK"); else KARG=(); fi
      timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${KARG[@]}" > gpurun_out/gpu_tests.log 2>&1
      rc=$?; tail -5 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc ;;
    diagtests)
      TNS_LIB=ab/diag/libtensorium_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q --timeout 600 --timeout-method thread -k "variants" > gpurun_out/gpu_diag_tests.log 2>&1
      rc=$?; tail -5 gpurun_out/gpu_diag_tests.log; [ $rc -eq 0 ] || exit $rc ;;
    mlpst)
      TNS_LIB=ab/mlpst/libtensorium_hip.so timeout -k 10 120 python -u scripts/mlp_stamps.py > gpurun_out/mlp_stamps.log 2>&1
      rc=$?; grep -v amdgpu.ids gpurun_out/mlp_stamps.log; [ $rc -eq 0 ] || exit $rc ;;
    bnab)
      for r in $(seq 1 ${ROUNDS:-2}); do for L in ${LIBS}; do
        echo -n "{\"tag\": \"$L\", \"res\": " >> gpurun_out/bnab.jsonl
        TNS_LIB=$(lib_of $L) timeout -k 10 300 python -u scripts/bn_perf.py >> gpurun_out/bnab.jsonl 2> gpurun_out/bnab_$L.err
        rc=$?; echo "}" >> gpurun_out/bnab.jsonl; [ $rc -eq 0 ] || { echo "$L rc=$rc"; tail -5 gpurun_out/bnab_$L.err; exit $rc; }
      done; done
      python3 -c "
import json
for l in open('gpurun_out/bnab.jsonl'):
    r=json.loads(l); d=r['res']['8x32x173056']; print(r['tag'], d['means_vars_ms'], d['add_sums_ms'], d['add_dots_ms'], d['means_vars_delta_ms'])" ;;
    abfwd)
      for r in $(seq 1 ${ROUNDS:-2}); do for L in ${LIBS}; do
        TNS_LIB=$(lib_of $L) timeout -k 10 300 python -u scripts/quick_perf.py --tag $L --yolo-only >> gpurun_out/abfwd.jsonl 2> gpurun_out/abfwd_$L.err
        rc=$?; [ $rc -eq 0 ] || { echo "$L rc=$rc"; tail -5 gpurun_out/abfwd_$L.err; exit $rc; }
      done; done
      python3 -c "
import json
for l in open('gpurun_out/abfwd.jsonl'):
    r=json.loads(l); print(r['tag'], r['yolo_ms'], r['yolo_tflops'])" ;;
    abgemm)
      for r in $(seq 1 ${ROUNDS:-2}); do for L in ${LIBS}; do
        TNS_LIB=$(lib_of $L) timeout -k 10 300 python -u scripts/quick_perf.py --tag $L >> gpurun_out/abgemm.jsonl 2> gpurun_out/abgemm_$L.err
        rc=$?; [ $rc -eq 0 ] || { echo "$L rc=$rc"; tail -5 gpurun_out/abgemm_$L.err; exit $rc; }
      done; done
      python3 -c "
import json
for l in open('gpurun_out/abgemm.jsonl'):
    r=json.loads(l); print(r['tag'], r['sgemm4096_ms'], r['batched_tflops'], r['yolo_ms'])" ;;
    batched)
      for L in ${LIBS:-main}; do
        TNS_LIB=$(lib_of $L) timeout -k 10 300 python -u scripts/batched_probe.py > gpurun_out/batched_$L.json 2> gpurun_out/batched_$L.err
        rc=$?; echo "$L $(cat gpurun_out/batched_$L.json)"; [ $rc -eq 0 ] || { tail -5 gpurun_out/batched_$L.err; exit $rc; }
      done ;;
    bwdab)
      for r in $(seq 1 ${ROUNDS:-2}); do for L in ${LIBS}; do
        echo "{\"tag\": \"$L\"}" >> gpurun_out/bwdab.jsonl
        TNS_LIB=$(lib_of $L) timeout -k 10 400 python -u scripts/bwd_graph.py --rounds 1 >> gpurun_out/bwdab.jsonl 2> gpurun_out/bwdab_$L.err
        rc=$?; [ $rc -eq 0 ] || { echo "$L rc=$rc"; tail -5 gpurun_out/bwdab_$L.err; exit $rc; }
      done; done
      cat gpurun_out/bwdab.jsonl | cut -c1-400 ;;
    stamps)
      TNS_LIB=ab/stamps/libtensorium_hip.so timeout -k 10 300 python -u scripts/ct4_stamps.py --layer ${LAYERS:-11,28,45,10} --warm-ms 200 ${STAMP_ARGS:-} > gpurun_out/stamps.jsonl 2> gpurun_out/stamps.err
      rc=$?; cat gpurun_out/stamps.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/stamps.err; exit $rc; } ;;
    fwdsweep)
      # VARIANTS: "<layers>:<v1>,<v2>,..." groups separated by spaces (v as
      # TNS_OPT_CONV_VARIANT, -1 the pick); two passes, interleaved
      for r in 1 2; do for grp in ${VARIANTS}; do
        L=${grp%%:*}; VS=${grp#*:}
        for v in ${VS//,/ }; do
          echo -n "{\"round\": $r, \"variant\": $v, \"res\": " >> gpurun_out/fwdsweep.jsonl
          timeout -k 10 120 python -u scripts/conv_fwd_layers.py --layers $L --variant $v --warm-ms 100 --reps 20 >> gpurun_out/fwdsweep.jsonl 2> gpurun_out/fwdsweep.err
          rc=$?; echo "}" >> gpurun_out/fwdsweep.jsonl; [ $rc -eq 0 ] || { tail -5 gpurun_out/fwdsweep.err; exit $rc; }
        done
      done; done
      python3 scripts/parse_fwdsweep.py ;;
    bwdsweep)
      timeout -k 10 900 python -u scripts/bwd_sweep.py --layers ${BLAYERS:-1,3,4,6,11} --what ${BWHAT:-dx} > gpurun_out/bwdsweep.json 2> gpurun_out/bwdsweep.err
      rc=$?; tail -c 4000 gpurun_out/bwdsweep.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bwdsweep.err; exit $rc; } ;;
    bench)
      timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
      rc=$?; tail -c 3000 gpurun_out/bench.json; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench.err; exit $rc; } ;;
    trace)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_trace -o trace -- python3 bench.py ${BENCH_ARGS:---no-cpu} > gpurun_out/trace_bench.json 2> gpurun_out/trace.err
      rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/trace.err; exit $rc; } ;;
  esac
done
