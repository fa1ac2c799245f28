#!/bin/bash
# Round 5: k_emit_mm<32> (O0) with 512-thread workgroups (PZK_MM_THREADS=512) vs 256, one box, alternated; register
# parity under the switch first
set -o pipefail
O=gpurun_out/r5z
mkdir -p $O
PZK_MM_THREADS=512 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "register and not symmap" > $O/pytest_512.log 2>&1 || { tail -30 $O/pytest_512.log; exit 1; }
tail -1 $O/pytest_512.log
tools/gpu/gpu_lines.sh r5z "c3:--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3w:PZK_MM_THREADS=512|--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3b:--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3wb:PZK_MM_THREADS=512|--steps 20 --warmup 5 --no-cpu --no-host"
