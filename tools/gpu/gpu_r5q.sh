#!/bin/bash
# Round 5: mapped layouts default to two SHA emitter streams (per-section k_emit_mm again); O2 / O1-shaped lines with
# one and two streams, config 3
set -o pipefail
T0=$(date +%s)
TESTS="symmap or register" tools/gpu/gpu_lines.sh r5q \
  "o2:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2s1:PZK_SHA_STREAMS=1|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o1:--sym o1shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o1s1:PZK_SHA_STREAMS=1|--sym o1shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "c3:--steps 20 --warmup 5 --no-cpu --no-host" \
  "o2b:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
