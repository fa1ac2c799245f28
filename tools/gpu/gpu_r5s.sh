#!/bin/bash
# Round 5: A/B on one box — mapped Poseidon blocks filling only the image parts their kept signals read (default) vs
# the whole image (PZK_POS_FULL=1), the O2-shaped line, alternated
set -o pipefail
T0=$(date +%s)
tools/gpu/gpu_lines.sh r5s \
  "o2:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2full:PZK_POS_FULL=1|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2b:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2fullb:PZK_POS_FULL=1|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2s1:PZK_SHA_STREAMS=1|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "c3:--steps 20 --warmup 5 --no-cpu --no-host" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
