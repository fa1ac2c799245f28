#!/bin/bash
# round-2 closing check after the core-kernel occupancy changes (k_bjj_core 32 lanes, k_smt_prep 8 lanes
# per witness): the full GPU parity suite, the default bench line, rocprofv3 stats of the bench command
# (concurrent) and of the serialized schedule (standalone kernel times)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2d}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
head -c 400 gpurun_out/bench_$TAG.json; echo
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 4 --warmup 1 --no-cpu > gpurun_out/prof_$TAG.log 2>&1 || { tail gpurun_out/prof_$TAG.log; exit 1; }
PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_serial -o run -- python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_${TAG}_serial.log 2>&1 || { tail gpurun_out/prof_${TAG}_serial.log; exit 1; }
echo profiles done
