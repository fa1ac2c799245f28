#!/bin/bash
# Round 5: config 3 (+4) lines on the final tree, twice, and QueryIdentity (box check after r5x's slow box)
set -o pipefail
tools/gpu/gpu_lines.sh r5y "c3:--steps 20 --warmup 5 --no-cpu --no-host" \
  "query:--workload query --steps 20 --warmup 5 --no-cpu --no-host" \
  "c3b:--steps 20 --warmup 5 --no-cpu --no-host" \
  "o2:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu"
