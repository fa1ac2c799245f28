#!/bin/bash
# Round 5: the mixed (config 5) regression — chain stream priority / post split A/B with three instances; config 2
# back on one stream
set -o pipefail
T0=$(date +%s)
tools/gpu/gpu_lines.sh r5k "sha256:--workload sha256 --steps 10 --warmup 2 --no-host --no-cpu" \
  "mixedlo:PZK_CHAIN_PRIO=lo|--workload mixed --steps 6 --warmup 2 --no-host --no-cpu" \
  "mixedlo0:PZK_CHAIN_PRIO=lo PZK_POST=0|--workload mixed --steps 6 --warmup 2 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
