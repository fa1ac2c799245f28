#!/bin/bash
# Round 5: standalone-circuit emitters beside the next core (config 1 line), tail placement A/B (PZK_TAIL=emit) on
# the O2-shaped line and configs 3 / 4, QueryIdentity with four chain streams / four scratch sets
set -o pipefail
T0=$(date +%s)
TESTS="small or poseidon or sha or stream" tools/gpu/gpu_lines.sh r5h "poseidon:--workload poseidon --steps 20 --warmup 5" \
  "o2:--sym o2shape --steps 10 --warmup 2 --no-host --no-cpu" \
  "o2temit:PZK_TAIL=emit|--sym o2shape --steps 10 --warmup 2 --no-host --no-cpu" \
  "c3temit:PZK_TAIL=emit|--steps 10 --warmup 2 --no-host --no-cpu" \
  "c3:--steps 10 --warmup 2 --no-host --no-cpu" \
  "query:--workload query --steps 10 --warmup 2 --no-host --no-cpu" \
  "queryc4:PZK_QRY_CHAINS=4|--workload query --steps 10 --warmup 2 --no-host --no-cpu" \
  "queryc4n4:PZK_QRY_CHAINS=4 PZK_NSETS=4|--workload query --steps 10 --warmup 2 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
