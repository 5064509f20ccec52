#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/mfma_probe > gpurun_out/mfma_probe.log 2>&1; rc=$?; cat gpurun_out/mfma_probe.log; [ $rc -eq 0 ] || exit $rc
LIBS="base ct_nogather ct_nocheck ct_noa ct_nostore ct_nobar ct_bare ct_barest" ./scripts/gpu_ct_diag.sh
