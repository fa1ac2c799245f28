#!/bin/bash
# GPU (round 3): QueryIdentity chain-stream A/B: 2 vs 3 chain streams, and 3 with 8 hardware queues.
set -o pipefail
O=gpurun_out/r3q3
mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload query --steps 10 --no-cpu > $O/bench_$tag.json 2> $O/bench_$tag.err \
    || { tail -20 $O/bench_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); print('$tag', d['value'], d['ms_per_step'], {k: v['ms_per_launch'] for k, v in d['phases'].items()})"
}
run c3 PZK_QRY_CHAINS=3 && run c2 PZK_QRY_CHAINS=2 && run c3q8 PZK_QRY_CHAINS=3 GPU_MAX_HW_QUEUES=8 && run c2q8 PZK_QRY_CHAINS=2 GPU_MAX_HW_QUEUES=8
