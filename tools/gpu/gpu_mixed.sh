#!/bin/bash
# GPU: mixed-flow parity test + config-5 bench line (1 GPU)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mixed.py -x -v --timeout 500 --timeout-method thread > gpurun_out/gpu_mixed.log 2>&1 || { tail -30 gpurun_out/gpu_mixed.log; exit 1; }
grep -E "passed|failed" gpurun_out/gpu_mixed.log | tail -1
timeout -k 10 900 python -u bench.py --workload mixed --steps 2 --warmup 1 > gpurun_out/bench_mixed.json 2> gpurun_out/bench_mixed.err || { tail -20 gpurun_out/bench_mixed.err; exit 1; }
cat gpurun_out/bench_mixed.json
