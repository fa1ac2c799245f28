#!/bin/bash
# GPU (round 3): QueryIdentity(80) parity (tests/test_gpu_query.py) + the register tests (shared SMT / BJJ code),
# then the query bench line (with its CPU baseline) and a config-3 line.
set -o pipefail
O=gpurun_out/r3q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_query.py tests/test_gpu_register.py -x -v --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 400 python -u bench.py --workload query --steps 5 > $O/bench_query.json 2> $O/bench_query.err \
  || { tail -20 $O/bench_query.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_query.json')); print('query', d['value'], d['roofline'], d.get('cpu_baseline',{}).get('value'))"
timeout -k 10 400 python -u bench.py --no-cpu --no-host --steps 10 > $O/bench_config3.json 2> $O/bench_config3.err \
  || { tail -20 $O/bench_config3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_config3.json')); print('config3', d['value'], d['roofline']['frac'])"
