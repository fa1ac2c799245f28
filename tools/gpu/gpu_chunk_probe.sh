#!/bin/bash
# emit_sha chunk-size probe: standalone kernel time via rocprofv3 stats for several chunk sizes
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 2048 4096 8192 16384 32768; do
  PZK_SERIAL=1 PZK_CHUNK_1=$c PZK_CHUNK_5=$c timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/chunk_$c -o run -- python bench.py --steps 1 --warmup 1 --batch 2048 --no-cpu > gpurun_out/chunk_$c.log 2>&1 || exit $?
done
echo done
