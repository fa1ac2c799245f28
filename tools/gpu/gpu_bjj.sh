#!/bin/bash
# k_bjj_core lanes-per-witness A/B (PZK_BJJ_SEGS 8 / 16 / 32): parity subset at the default, then per
# setting a default-config bench line and serialized kernel stats (standalone k_bjj_core time)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-bjj}
timeout -k 10 500 python -u -m pytest tests/test_gpu_register.py tests/test_gpu_r1cs.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || { tail -40 gpurun_out/gpu_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/gpu_tests_$TAG.log
for S in ${SEGS:-8 16 32}; do
  PZK_BJJ_SEGS=$S timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/bench_${TAG}_$S.json 2> gpurun_out/bench_${TAG}_$S.err || { tail gpurun_out/bench_${TAG}_$S.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$S.json')); print('segs $S', d['value'], d['ms_per_step'])"
  PZK_BJJ_SEGS=$S PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$S -o run -- python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_${TAG}_$S.log 2>&1 || { tail gpurun_out/prof_${TAG}_$S.log; exit 1; }
  f=$(find gpurun_out/prof_${TAG}_$S -name "*kernel_stats.csv" | head -1); grep -E "k_bjj_core|k_emit_sha" "$f" | cut -d, -f1-4
done
