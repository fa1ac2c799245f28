#!/bin/bash
# SIGNATURE_TYPE 13 (RSA-PSS over SHA-384): GPU suite, its bench line and a rocprofv3 stats run of it
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-sig13}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 400 python bench.py --sig 13 --steps 3 --warmup 1 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
head -c 400 gpurun_out/bench_$TAG.json; echo
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --sig 13 --steps 1 --warmup 1 --no-cpu > gpurun_out/prof_$TAG.log 2>&1
