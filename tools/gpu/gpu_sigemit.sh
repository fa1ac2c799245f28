#!/bin/bash
# A/B: signature emitters on the RSA stream (default) or on the emit stream (PZK_SIGEMIT=emit); tail on the RSA stream too
set -o pipefail
mkdir -p gpurun_out
for m in default emit tailrsa default tailrsa; do
  unset PZK_SIGEMIT PZK_TAIL
  case $m in emit) export PZK_SIGEMIT=emit;; tailrsa) export PZK_TAIL=rsa;; esac
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/se_$m.json 2> gpurun_out/se_$m.err || { tail -5 gpurun_out/se_$m.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/se_$m.json')); print('$m', d['value'], d['ms_per_step'])"
done
