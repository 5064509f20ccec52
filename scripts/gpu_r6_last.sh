#!/bin/bash
# the committed build: the round-end set, then the bench command's profile
./scripts/gpu_r6_full.sh gpurun_out/r6last2 || exit 1
TAG=r06d PROF_ARGS="--steps 20 --warmup 20 --no-cpu" ./scripts/profile_r6.sh
