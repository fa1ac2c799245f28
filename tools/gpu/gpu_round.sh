#!/bin/bash
# one GPU round-trip: parity tests, serialized per-kernel profile, concurrent bench + profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-x}
timeout -k 10 800 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/serial_$TAG -o run -- python bench.py --steps 1 --warmup 1 --batch 2048 --no-cpu > gpurun_out/serial_$TAG.log 2>&1 || exit $?
tools/gpu/gpu_bench_profile.sh $TAG
