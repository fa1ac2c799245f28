#!/bin/bash
# Round 5: zero-input Poseidon blocks copied from O0 zero rows; occupancy (k_emit_pos t <= 3 and k_emit_gen at <= 96
# VGPRs, MAP_SEG 1,664 so four mapped k_emit_mm / eight mapped k_emit_sha workgroups fit per CU); mapped k_emit_mm
# with merged section runs (A/B: PZK_MM_SPLIT=1); SHA emitters over two streams (PZK_SHA_STREAMS=2) and the SHA
# stream at high priority (8 hardware queues); then the config-4 PMC passes
set -o pipefail
T0=$(date +%s)
TESTS="register or symmap or small or query or poseidon" tools/gpu/gpu_lines.sh r5p \
  "c3:--steps 20 --warmup 5 --no-cpu --no-host" \
  "o2:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2split:PZK_MM_SPLIT=1|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "c3sha2:PZK_SHA_STREAMS=2|--steps 20 --warmup 5 --no-cpu --no-host" \
  "o2sha2:PZK_SHA_STREAMS=2|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "c3q8:GPU_MAX_HW_QUEUES=8|--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3shahi:GPU_MAX_HW_QUEUES=8 PZK_SHA_PRIO=hi|--steps 20 --warmup 5 --no-cpu --no-host" \
  "o2b:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5c4c 2048 "--workload config4" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
