#!/bin/bash
# Round 5: full GPU suite + smoke + the driver's default bench command, then PMC passes of configs 3 and 4 on the
# new defaults (scratch BabyJubJub core, FIPS register chain, post-chain split)
set -o pipefail
T0=$(date +%s)
TESTS=all SMOKE=1 tools/gpu/gpu_lines.sh r5f "driver:--gpus 1 --steps 20 --warmup 5" &&
python3 -c "import json; d=json.load(open('gpurun_out/r5f/bench_driver.json')); c=d['config4']; print('config4', c['value'], c['job_hbm']['frac'], 'cpu', d['cpu_baseline']['value'], d['cpu_baseline']['value_nproc_scaled'])" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5c3 2048 "" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5c4b 2048 "--workload config4" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
