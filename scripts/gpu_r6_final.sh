#!/bin/bash
# A/B of the specialised-wave fused BN, then the round-end set (tests, smoke,
# bench) and the profile passes of the bench command, summarised on the box
./scripts/gpu_bnb_ws.sh gpurun_out/bnbws || exit 1
./scripts/gpu_r6_full.sh gpurun_out/r6final || exit 1
TAG=r06b PROF_ARGS="--steps 20 --warmup 20 --no-cpu" ./scripts/profile_r6.sh
