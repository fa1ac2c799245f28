#!/bin/bash
# Poseidon emitter change: parity subset, default bench line, serialized kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pos}
timeout -k 10 500 python -u -m pytest tests/test_gpu_small_circuits.py tests/test_gpu_register.py tests/test_gpu_r1cs.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], d.get('job_hbm'))"
PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_$TAG.log 2>&1 || { tail gpurun_out/prof_$TAG.log; exit 1; }
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -d, -f1-4
