#!/bin/bash
# emit_sha store-pattern probe (serialized phases): PZK_SHA_MODE 0 = 32 B/lane, 1 = 16 B/lane nt, 2 = 16 B/lane
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 0 1 2; do
  PZK_SERIAL=1 PZK_SHA_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/shamode_$m -o run -- python bench.py --steps 1 --warmup 1 --batch 2048 --no-cpu > gpurun_out/shamode_$m.log 2>&1 || exit $?
done
PZK_SHA_MODE=1 timeout -k 10 300 python -m pytest tests/test_gpu_small_circuits.py tests/test_gpu_register.py -q -x -m gpu -k "canonical or sha" > gpurun_out/shamode_test.log 2>&1 || exit $?
echo done
