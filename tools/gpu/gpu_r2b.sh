#!/bin/bash
# round-2 closing check: the GPU parity suite, the default bench line, a rocprofv3 stats run of it, and the
# host throughput of the SOD preprocessor on the box's CPU share
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2b}
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
head -c 700 gpurun_out/bench_$TAG.json; echo
timeout -k 10 200 python tools/bench_passport.py --n 32768 > gpurun_out/bench_passport_$TAG.json 2>&1 || { tail gpurun_out/bench_passport_$TAG.json; exit 1; }
cat gpurun_out/bench_passport_$TAG.json
