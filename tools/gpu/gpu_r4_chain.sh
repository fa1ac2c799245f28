#!/bin/bash
# GPU (round 4): full parity suite + smoke, the chain product-policy A/B, then kernel-trace timelines of SIG 20 and
# the mixed config-5 batch.
set -o pipefail
B="--steps 8 --warmup 2 --no-cpu --no-host"
TESTS=all SMOKE=1 tools/gpu/gpu_lines.sh r4_chain "d60:$B --smt-depth 40-79" "d60call:PZK_CHAIN_MUL=call|$B --smt-depth 40-79" \
  "d0:$B" "query:--workload query --steps 10 --no-cpu" "querycall:PZK_CHAIN_MUL=call|--workload query --steps 10 --no-cpu" || exit 1
tools/gpu/gpu_timeline.sh r4_tl "sig20:--sig 20 --steps 3 --warmup 1 --no-cpu --no-host" \
  "mixed:--workload mixed --steps 2 --warmup 1 --no-cpu"
