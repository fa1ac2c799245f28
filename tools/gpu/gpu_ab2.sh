#!/bin/bash
# A/B (serialized kernels + concurrent bench) of an env switch: gpu_ab2.sh VAR VAL0 VAL1
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in $2 $3; do
  export $1=$v
  PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab2s_$v -o run -- python bench.py --steps 1 --warmup 1 --batch 2048 --no-cpu > gpurun_out/ab2s_$v.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu > gpurun_out/ab2b_$v.json 2> gpurun_out/ab2b_$v.err || exit $?
done
echo done
