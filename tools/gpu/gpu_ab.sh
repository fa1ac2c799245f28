#!/bin/bash
# A/B bench runs: each argument is one variant "ENV=V ... -- bench args" (env assignments, then
# bench.py arguments); one JSON line per variant into gpurun_out/ab_<i>.json, summary printed
set -o pipefail
mkdir -p gpurun_out
i=0
for spec in "$@"; do
  envs="${spec%%--*}"; bargs="${spec#*--}"
  [ "$envs" = "$spec" ] && bargs=""
  env $envs timeout -k 10 240 python bench.py --steps ${STEPS:-8} --warmup 2 --no-cpu $bargs > gpurun_out/ab_$i.json 2> gpurun_out/ab_$i.err || { echo "variant $i failed"; tail -5 gpurun_out/ab_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$i.json')); print('$i [$spec]', d['value'], d['config']['sub_batch'], d['roofline']['frac'], d['job_hbm']['frac'])"
  i=$((i+1))
done
