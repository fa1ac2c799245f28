#!/bin/bash
# GPU (round 3, last): sliding-window inversions in k_bjj_core / k_smt_prep / k_smt_chain. The whole -m gpu suite,
# smoke(), the default bench line, the query line and its serialized kernel stats.
set -o pipefail
O=gpurun_out/r3_final5
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('config3', d['value'], d['roofline']['frac'], d['cpu_baseline']['value'], d['host_delivered']['value'])"
timeout -k 10 300 python -u bench.py --workload query --steps 10 --no-cpu > $O/bench_query.json 2> $O/bench_query.err || { tail -20 $O/bench_query.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_query.json')); print('query', d['value'], {k: v['ms_per_launch'] for k, v in d['phases'].items()})"
PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- \
  python bench.py --workload query --steps 2 --warmup 1 --no-cpu > $O/serial.log 2>&1 || { tail -20 $O/serial.log; exit 1; }
python3 tools/kstats.py $O/serial/run_kernel_stats.csv > $O/serial_stats.txt 2>&1; head -12 $O/serial_stats.txt
