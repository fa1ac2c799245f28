#!/bin/bash
# Round 5: the post-chain emission split (PZK_POST), pipeline depth and hardware-queue A/B on config 4, after the
# GPU parity suite.
set -o pipefail
T0=$(date +%s)
TESTS=all tools/gpu/gpu_lines.sh r5b "default:--steps 10 --warmup 2 --no-host --no-cpu" \
  "c4post0:PZK_POST=0|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "c4post1:--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "c4n4:PZK_NSETS=4|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "c4q8:GPU_MAX_HW_QUEUES=8|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "c4q8n4:GPU_MAX_HW_QUEUES=8 PZK_NSETS=4|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "c3q8:GPU_MAX_HW_QUEUES=8|--steps 10 --warmup 2 --no-host --no-cpu --no-config4" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
