#!/bin/bash
# Round 5: O2-shaped line with two SHA streams — pipeline depth 4, the signature emitters on their own stream with 8
# hardware queues (low / high priority); then the PMC passes of config 3 and QueryIdentity on the current kernels
set -o pipefail
T0=$(date +%s)
tools/gpu/gpu_lines.sh r5t \
  "o2:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2n4:PZK_NSETS=4|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2q8own:GPU_MAX_HW_QUEUES=8 PZK_SIGEMIT=own|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2q8ownhi:GPU_MAX_HW_QUEUES=8 PZK_SIGEMIT=own PZK_MM_PRIO=hi|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2b:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5c3c 2048 "" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5q2 4096 "--workload query" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
