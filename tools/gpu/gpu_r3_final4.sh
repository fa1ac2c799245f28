#!/bin/bash
# GPU (round 3, late): the whole -m gpu suite, smoke(), the default bench line (CPU baseline, host delivery,
# input side) and its rocprof kernel stats, then the query and mixed lines.
set -o pipefail
O=gpurun_out/r3_final4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('config3', d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], d['host_delivered']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- \
  python bench.py --steps 4 --warmup 1 --no-cpu --no-host > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/kstats.py $O/prof/run_kernel_stats.csv > $O/prof_stats.txt 2>&1; head -4 $O/prof_stats.txt
timeout -k 10 300 python -u bench.py --workload query --steps 10 > $O/bench_query.json 2> $O/bench_query.err || { tail -20 $O/bench_query.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_query.json')); print('query', d['value'], d['cpu_baseline']['value'])"
timeout -k 10 300 python -u bench.py --workload query-td1 --steps 10 --no-cpu > $O/bench_query_td1.json 2> $O/bench_query_td1.err || { tail -20 $O/bench_query_td1.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_query_td1.json')); print('query-td1', d['value'])"
timeout -k 10 400 python -u bench.py --workload mixed --steps 3 --warmup 1 > $O/bench_mixed.json 2> $O/bench_mixed.err || { tail -20 $O/bench_mixed.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_mixed.json')); print('mixed', d['value'])"
