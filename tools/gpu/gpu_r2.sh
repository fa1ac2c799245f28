#!/bin/bash
# round-2 check: GPU parity suite, then the default bench line and a rocprofv3 stats run of it
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json | head -c 600; echo
if [ -n "$PROF" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/prof_$TAG.log 2>&1 || exit 1
fi
