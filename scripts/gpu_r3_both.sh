#!/bin/bash
set -u
bash scripts/gpu_pp.sh && bash scripts/gpu_convpp.sh
