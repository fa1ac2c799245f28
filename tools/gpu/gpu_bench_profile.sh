#!/bin/bash
# bench (config 3) + rocprofv3 kernel-trace stats of the same command; results under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r1}
timeout -k 10 600 python bench.py --steps ${STEPS:-3} --warmup 1 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_$TAG.log 2>&1
echo rc=$?
