#!/bin/bash
# GPU (round 3): QueryIdentity stream A/B: 3 chain streams with one emitter stream (4 streams = 4 HW queues).
set -o pipefail
O=gpurun_out/r3q5
mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload query --steps 10 --no-cpu > $O/bench_$tag.json 2> $O/bench_$tag.err \
    || { tail -20 $O/bench_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); print('$tag', d['value'], d['ms_per_step'], {k: v['ms_per_launch'] for k, v in d['phases'].items()})"
}
run c3e1 PZK_QRY_CHAINS=3 PZK_QRY_EMIT1=1 && run c3 PZK_QRY_CHAINS=3 && run c3e1q8 PZK_QRY_CHAINS=3 PZK_QRY_EMIT1=1 GPU_MAX_HW_QUEUES=8 && run c3e1b PZK_QRY_CHAINS=3 PZK_QRY_EMIT1=1
