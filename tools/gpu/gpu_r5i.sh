#!/bin/bash
# Round 5: QueryIdentity pipeline depth (defaults now 4 scratch sets, 4 chain streams), the O2-shaped line's depth and
# sub-batch, config 1 with a ~10 s CPU sample
set -o pipefail
T0=$(date +%s)
TESTS="query" tools/gpu/gpu_lines.sh r5i "query:--workload query --steps 10 --warmup 2 --no-host --no-cpu" \
  "queryn5:PZK_NSETS=5|--workload query --steps 10 --warmup 2 --no-host --no-cpu" \
  "queryn6:PZK_NSETS=6|--workload query --steps 10 --warmup 2 --no-host --no-cpu" \
  "querytd1:--workload query-td1 --steps 10 --warmup 2 --no-host --no-cpu" \
  "o2n4:PZK_NSETS=4|--sym o2shape --steps 10 --warmup 2 --no-host --no-cpu" \
  "o2s2k:--sym o2shape --sub 2048 --steps 10 --warmup 2 --no-host --no-cpu" \
  "o2s2kn4:PZK_NSETS=4|--sym o2shape --sub 2048 --steps 10 --warmup 2 --no-host --no-cpu" \
  "o2ch16k:PZK_CHUNK_1=16384|--sym o2shape --steps 10 --warmup 2 --no-host --no-cpu" \
  "o2ch64k:PZK_CHUNK_1=65536|--sym o2shape --steps 10 --warmup 2 --no-host --no-cpu" \
  "poseidon:--workload poseidon --steps 20 --warmup 5" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
