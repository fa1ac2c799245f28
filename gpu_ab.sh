#!/bin/bash
# A/B of an environment switch on the concurrent bench timeline: gpu_ab.sh VAR
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
  if [ $v = 1 ]; then export $1=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab_$v -o run -- python bench.py --steps 2 --warmup 1 --no-cpu > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || exit $?
done
echo done
