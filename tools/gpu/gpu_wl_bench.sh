#!/bin/bash
# GPU: bench line of one workload + rocprofv3 kernel stats of the same workload (usage: TAG WORKLOAD)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-x}
WL=${2:-register}
timeout -k 10 600 python -u bench.py --workload $WL --steps ${STEPS:-2} --warmup 1 ${EXTRA} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --workload $WL --steps 1 --warmup 1 --no-cpu --batch ${PBATCH:-2048} > gpurun_out/prof_$TAG.log 2>&1
echo rc=$?
