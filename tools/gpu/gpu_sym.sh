#!/bin/bash
# GPU (round 4): mapped-layout parity tests, then the config-3 line O0 / --O2-shaped / --O1-shaped / synthetic map.
# usage: tools/gpu/gpu_sym.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-r4_sym}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
K=${2:-symmap or query or stream}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "$K" \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in o2shape o1shape synthetic:4 O0; do
  f=$O/bench_${m%%:*}.json
  extra="--sym $m"; [ "$m" = O0 ] && extra=""
  timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-host $extra > $f 2> ${f%.json}.err \
    || { tail -20 ${f%.json}.err; exit 1; }
  python3 -c "import json; d=json.load(open('$f')); print('$m', d['value'], d['config']['witness_elements'], d['job_hbm']['frac'], {k: v['ms_per_launch'] for k, v in d['phases'].items()})"
done
