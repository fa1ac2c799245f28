#!/bin/bash
# helper used with gpurun: run the GPU test suite under a time limit
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 ${1:-900} python -m pytest tests -m gpu -x -q ${@:2} 2>&1 | tee gpurun_out/gpu_tests.log
