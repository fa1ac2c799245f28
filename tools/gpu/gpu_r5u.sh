#!/bin/bash
# Round 5: k_emit_mm with half-size store stages and 5-word Karatsuba node outputs (K = 32: 36.9 -> 31.0 KB of LDS,
# five workgroups per CU; K = 64: four instead of three). RSA parity (K = 32 / 48 / 64, mapped), config 3 (+4), SIG 2
# (RSA-4096), the O2-shaped line, then the config-3 PMC passes
set -o pipefail
T0=$(date +%s)
TESTS="register or symmap or mixed or pss or r1cs" tools/gpu/gpu_lines.sh r5u \
  "c3:--steps 20 --warmup 5 --no-cpu --no-host" \
  "sig2:--sig 2 --steps 10 --warmup 3 --no-cpu --no-host" \
  "o2:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "c3b:--steps 20 --warmup 5 --no-cpu --no-host" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5c3d 2048 "" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
