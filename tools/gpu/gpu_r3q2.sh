#!/bin/bash
# GPU (round 3): QueryIdentity schedule A/B (PZK_QRY_CHAINS 1 vs 2 chain streams) and serialized kernel stats.
set -o pipefail
O=gpurun_out/r3q2
mkdir -p $O
export TMPDIR=/tmp
for c in 2 1; do
  PZK_QRY_CHAINS=$c timeout -k 10 300 python -u bench.py --workload query --steps 10 --no-cpu > $O/bench_query_c$c.json 2> $O/bench_query_c$c.err \
    || { tail -20 $O/bench_query_c$c.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_query_c$c.json')); print('chains $c', d['value'], d['ms_per_step'], {k: v['ms_per_launch'] for k, v in d['phases'].items()})"
done
PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- \
  python bench.py --workload query --steps 2 --warmup 1 --no-cpu > $O/serial.log 2>&1 || { tail -20 $O/serial.log; exit 1; }
python3 tools/kstats.py $O/serial/run_kernel_stats.csv > $O/serial_stats.txt 2>&1; head -24 $O/serial_stats.txt
