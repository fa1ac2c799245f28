#!/bin/bash
# Round 5: Poseidon image fill copies the S-box inputs of layers 1-3, 5-7 and of the partial rounds from the mix rows
# (77 of t = 3's 81 conversions). Parity, config 3 (+4), then the config-4 PMC passes
set -o pipefail
T0=$(date +%s)
TESTS="register or symmap or small or poseidon or query or r1cs" tools/gpu/gpu_lines.sh r5x \
  "c3:--steps 20 --warmup 5 --no-cpu --no-host" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5c4d 2048 "--workload config4" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
