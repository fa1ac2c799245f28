#!/bin/bash
# Round 5, last tree: the whole -m gpu suite, smoke(), the driver's default bench command
set -o pipefail
TESTS=all SMOKE=1 tools/gpu/gpu_lines.sh r5w "driver:--gpus 1 --steps 20 --warmup 5" &&
python3 -c "import json; d=json.load(open('gpurun_out/r5w/bench_driver.json')); c=d['config4']; print('config4', c['value'], c['job_hbm']['frac'], 'cpu', d['cpu_baseline']['value'], 'roof', d['roofline']['frac'], d['roofline']['avg_launch_ms'])"
