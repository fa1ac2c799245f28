#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 0 1 2 3; do
  PZK_SERIAL=1 PZK_POS_PROBE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/posp_$m -o run -- python bench.py --steps 1 --warmup 1 --batch 2048 --no-cpu > gpurun_out/posp_$m.log 2>&1 || exit $?
done
echo done
