#!/bin/bash
# GPU (round 3, f2): the ECDSA parity tests (SIG 20, 21 through the generic-chunk EC path, then 24 and 25),
# then the rest of the -m gpu suite.
set -o pipefail
mkdir -p gpurun_out/r3_f2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ecdsa.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3_f2/ecdsa.log 2>&1 || { tail -60 gpurun_out/r3_f2/ecdsa.log; exit 1; }
tail -12 gpurun_out/r3_f2/ecdsa.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  --deselect tests/test_gpu_ecdsa.py > gpurun_out/r3_f2/pytest.log 2>&1 || { tail -40 gpurun_out/r3_f2/pytest.log; exit 1; }
tail -3 gpurun_out/r3_f2/pytest.log
