#!/bin/bash
# Round 5: mapped k_emit_mm with 896-signal kept-list segments (32.8 KB of LDS: five workgroups per CU), k_emit_bjj
# at <= 80 VGPRs (six per CU). Parity, config 3 (+4), the O2-shaped line twice, QueryIdentity
set -o pipefail
T0=$(date +%s)
TESTS="register or symmap or mixed or query or r1cs" tools/gpu/gpu_lines.sh r5v \
  "c3:--steps 20 --warmup 5 --no-cpu --no-host" \
  "o2:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "query:--workload query --steps 20 --warmup 5 --no-cpu --no-host" \
  "o2b:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "c3b:--steps 20 --warmup 5 --no-cpu --no-host" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
