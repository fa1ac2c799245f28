#!/bin/bash
# Round 5: 512-thread k_emit_mm (default) vs 256 (PZK_MM_THREADS=256), second box, alternated
set -o pipefail
tools/gpu/gpu_lines.sh r5z2 "c3:--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3n:PZK_MM_THREADS=256|--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3b:--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3nb:PZK_MM_THREADS=256|--steps 20 --warmup 5 --no-cpu --no-host"
