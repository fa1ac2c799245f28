#!/bin/bash
# Round 5: register chain streams created at the first call by the per-process policy; parity tests, config 5, the
# default line (config 3 + 4), QueryIdentity with FIPS chain products
set -o pipefail
T0=$(date +%s)
TESTS="register or mixed or symmap or stream or fullsize" tools/gpu/gpu_lines.sh r5m "mixed:--workload mixed --steps 6 --warmup 2 --no-host --no-cpu" \
  "default:--steps 10 --warmup 2 --no-host --no-cpu" \
  "query:--workload query --steps 10 --warmup 2 --no-host --no-cpu" \
  "queryfips:PZK_CHAIN_MUL=fips|--workload query --steps 10 --warmup 2 --no-host --no-cpu" &&
python3 -c "import json; d=json.load(open('gpurun_out/r5m/bench_default.json')); c=d['config4']; print('config4', c['value'], c['job_hbm']['frac'])" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
