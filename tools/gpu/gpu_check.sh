#!/bin/bash
# GPU (round 4): selected -m gpu tests (or all with ALL=1), smoke(), the default bench line.
# usage: tools/gpu/gpu_check.sh TAG [pytest -k expression]
set -o pipefail
TAG=${1:-r4}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "$K" \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
else
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
fi
tail -2 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('config3', d['value'], d['roofline']['frac'], d['cpu_baseline']['value'])"
