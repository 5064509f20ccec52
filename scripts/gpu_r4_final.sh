#!/bin/bash
# Round-4 evidence: the rocprofv3 passes of scripts/profile.sh on the bench
# command (kernel trace + stats; FETCH_SIZE; WRITE_SIZE; MFMA busy + clock).
set -u
mkdir -p gpurun_out
TAG=r04 bash scripts/profile.sh
