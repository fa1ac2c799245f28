#!/bin/bash
# Round 5: BabyJubJub core A/B (PZK_BJJ=rc|scratch) and chain product (PZK_CHAIN_MUL) on configs 3 / 4 and the
# O2-shaped line
set -o pipefail
T0=$(date +%s)
tools/gpu/gpu_lines.sh r5e "c3rc:--steps 10 --warmup 2 --no-host --no-cpu --no-config4" \
  "c3sc:PZK_BJJ=scratch|--steps 10 --warmup 2 --no-host --no-cpu --no-config4" \
  "c4rc:--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "c4sc:PZK_BJJ=scratch|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "c4scfips:PZK_BJJ=scratch PZK_CHAIN_MUL=fips|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "o2rc:--sym o2shape --steps 10 --warmup 2 --no-host --no-cpu" \
  "o2sc:PZK_BJJ=scratch|--sym o2shape --steps 10 --warmup 2 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
