#!/bin/bash
# sub-batch size A/B of the default config-3 bench (4096 per step): 2048 (default), 1366, 1024
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-sub}
for S in ${SUBS:-2048 1366 1024 2048}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu --sub $S > gpurun_out/bench_${TAG}_$S.json 2> gpurun_out/bench_${TAG}_$S.err || { tail gpurun_out/bench_${TAG}_$S.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$S.json')); print('sub $S', d['value'], d['ms_per_step'], d['config']['sub_batch'])"
done
