#!/bin/bash
# Round 5: config 5 with the per-process stream-set policy (the first register instance keeps the full set), the
# rounds 1-4 set forced, and config 2 serial vs overlapped on the same box
set -o pipefail
T0=$(date +%s)
tools/gpu/gpu_lines.sh r5l "mixed:--workload mixed --steps 6 --warmup 2 --no-host --no-cpu" \
  "mixedr4:PZK_CHAIN_PRIO=lo PZK_POST=0|--workload mixed --steps 6 --warmup 2 --no-host --no-cpu" \
  "sha256:--workload sha256 --steps 10 --warmup 2 --no-host --no-cpu" \
  "sha256ov:PZK_OVERLAP=1|--workload sha256 --steps 10 --warmup 2 --no-host --no-cpu" \
  "sha256b:--workload sha256 --steps 10 --warmup 2 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
