#!/bin/bash
# GPU: full parity suite (one process), then the config-3 bench line
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_all.log 2>&1 || { tail -40 gpurun_out/gpu_all.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_all.log | tail -2
timeout -k 10 600 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_all.json 2> gpurun_out/bench_all.err || { tail -20 gpurun_out/bench_all.err; exit 1; }
cat gpurun_out/bench_all.json
