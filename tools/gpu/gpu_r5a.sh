#!/bin/bash
# Round 5, first pass: config 3 + embedded config 4 (default line), config 4 pipeline-depth A/B, a kernel-trace
# timeline of config 4, then the config-4 PMC passes.
set -o pipefail
T0=$(date +%s)
tools/gpu/gpu_lines.sh r5a "default:--steps 10 --warmup 2 --no-host --no-cpu" \
  "c4n4:PZK_NSETS=4|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" \
  "c4n4c3:PZK_NSETS=4 PZK_SMT_CHAINS=3|--workload config4 --steps 10 --warmup 2 --no-host --no-cpu" &&
python3 -c "import json; d=json.load(open('gpurun_out/r5a/bench_default.json')); print('config4', d['config4']['value'], d['config4']['job_hbm'], {k: v['ms_per_launch'] for k, v in d['config4']['phases'].items()})" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_timeline.sh r5a "c4tl:--workload config4 --steps 4 --warmup 1 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5c4 2048 "--workload config4" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
