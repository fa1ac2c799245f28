#!/bin/bash
# A/B of where the chain's tail emitters run (PZK_TAIL, runtime.cpp) on the default config-3 bench
set -o pipefail
mkdir -p gpurun_out
for m in split rsa sha emit; do
  export PZK_TAIL=$m
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/tail_$m.json 2> gpurun_out/tail_$m.err || { tail -5 gpurun_out/tail_$m.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/tail_$m.json')); print('$m', d['value'], d['ms_per_step'])"
done
