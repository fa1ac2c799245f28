#!/bin/bash
# Round 5: mapped Poseidon blocks fill only the image parts their kept signals read; two SHA streams only for maps
# keeping at most half the signals. Parity, the O2 / O1-shaped lines, config 3 (+ 4), QueryIdentity, then the
# O2-shaped PMC passes
set -o pipefail
T0=$(date +%s)
TESTS="symmap or register or small or poseidon or query" tools/gpu/gpu_lines.sh r5r \
  "o2:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o1:--sym o1shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "c3:--steps 20 --warmup 5 --no-cpu --no-host" \
  "query:--workload query --steps 20 --warmup 5 --no-cpu --no-host" \
  "o2b:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5o2c 4096 "--sym o2shape" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
