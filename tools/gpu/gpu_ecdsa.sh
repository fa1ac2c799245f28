#!/bin/bash
# GPU: ECDSA parity tests (then the RSA suite), under time limits
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ecdsa.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_ecdsa.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_ecdsa.log
exit $rc
