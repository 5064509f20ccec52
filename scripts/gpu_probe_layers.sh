#!/bin/bash
# MFMA loop-rate probe, then the per-layer YOLOv3 forward table under a kernel trace
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 60 ./scripts/mfma_probe > gpurun_out/mfma_probe.log 2>&1; rc=$?; cat gpurun_out/mfma_probe.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fwd -o fwd -- python3 -u scripts/conv_fwd_layers.py > gpurun_out/conv_fwd_layers.json 2> gpurun_out/conv_fwd_layers.err
rc=$?; echo "layers rc=$rc"; [ $rc -eq 0 ] || exit $rc
tail -c 400 gpurun_out/conv_fwd_layers.json
