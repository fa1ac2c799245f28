#!/bin/bash
# Round 5: k_smt_chain without the 40 KB sibling stage in LDS (its workgroups sit beside the emitters on every CU)
set -o pipefail
T0=$(date +%s)
TESTS="register or smt or query or scalar" tools/gpu/gpu_lines.sh r5d "default:--steps 10 --warmup 2 --no-host --no-cpu" \
  "c4n4:PZK_NSETS=4|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "c4fips:PZK_CHAIN_MUL=fips|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "query:--workload query --steps 10 --warmup 2 --no-host --no-cpu" \
  "queryfips:PZK_CHAIN_MUL=fips|--workload query --steps 10 --warmup 2 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
