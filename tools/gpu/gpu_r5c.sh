#!/bin/bash
# Round 5: SMT chain streams on the high-priority queue pool (PZK_CHAIN_PRIO), with the post-chain split
set -o pipefail
T0=$(date +%s)
TESTS="register or smt or query or scalar" tools/gpu/gpu_lines.sh r5c "default:--steps 10 --warmup 2 --no-host --no-cpu" \
  "c4lo:PZK_CHAIN_PRIO=lo|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "c4post0:PZK_POST=0|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "c4q8:GPU_MAX_HW_QUEUES=8|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "query:--workload query --steps 10 --warmup 2 --no-host --no-cpu" \
  "querylo:PZK_CHAIN_PRIO=lo|--workload query --steps 10 --warmup 2 --no-host --no-cpu" \
  "o2:--sym o2shape --steps 10 --warmup 2 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
