#!/bin/bash
# GPU: full parity suite, then config-3 bench with the cooperative RSA core vs the lane core,
# and a kernel-trace summary of the default bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { tail -40 gpurun_out/gpu_all.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_all.log | tail -2
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_coop.json 2> gpurun_out/bench_coop.err || { tail -20 gpurun_out/bench_coop.err; exit 1; }
cat gpurun_out/bench_coop.json
PZK_RSA_CORE=lane timeout -k 10 600 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_lane.json 2> gpurun_out/bench_lane.err || { tail -20 gpurun_out/bench_lane.err; exit 1; }
cat gpurun_out/bench_lane.json
rm -rf gpurun_out/prof_coop
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_coop -o run -- python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/prof_coop.log 2>&1 || { tail -20 gpurun_out/prof_coop.log; exit 1; }
find gpurun_out/prof_coop -name "*kernel_stats.csv" | head -1 | xargs head -14
