#!/bin/bash
# Round 5: zero-input Poseidon blocks copied from precomputed O0 zero rows; SHA emitters alternating over two streams
# (PZK_SHA_STREAMS=2) with / without the signature emitters on their own stream, on config 3 and the O2-shaped line;
# the SHA emitter stream at high priority (8 hardware queues); then the config-4 PMC passes (k_emit_pos VALU with the zero rows)
set -o pipefail
T0=$(date +%s)
TESTS="register or symmap or small or query or poseidon" tools/gpu/gpu_lines.sh r5o \
  "c3:--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3sha2:PZK_SHA_STREAMS=2|--steps 20 --warmup 5 --no-cpu --no-host" \
  "o2:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2sha2:PZK_SHA_STREAMS=2|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2sha2own:PZK_SHA_STREAMS=2 PZK_SIGEMIT=own|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "c3sha2own:PZK_SHA_STREAMS=2 PZK_SIGEMIT=own|--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3q8:GPU_MAX_HW_QUEUES=8|--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3shahi:GPU_MAX_HW_QUEUES=8 PZK_SHA_PRIO=hi|--steps 20 --warmup 5 --no-cpu --no-host" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5c4c 2048 "--workload config4" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
