#!/bin/bash
# Round 5: mapped SHA chunks merged to EMIT_CHUNK kept signals, QueryIdentity with six scratch sets: parity tests
# of both, the lines, and the O2-shaped PMC pass on the new chunks
set -o pipefail
T0=$(date +%s)
TESTS="symmap or query or capi" tools/gpu/gpu_lines.sh r5j "o2:--sym o2shape --steps 10 --warmup 2 --no-host --no-cpu" \
  "o1:--sym o1shape --steps 10 --warmup 2 --no-host --no-cpu" \
  "query:--workload query --steps 10 --warmup 2 --no-host --no-cpu" \
  "querytd1:--workload query-td1 --steps 10 --warmup 2 --no-host --no-cpu" \
  "sha256:--workload sha256 --steps 10 --warmup 2 --no-host --no-cpu" \
  "mixed:--workload mixed --steps 6 --warmup 2 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5o2b 2048 "--sym o2shape" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
