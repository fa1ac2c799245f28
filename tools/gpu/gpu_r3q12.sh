#!/bin/bash
# GPU (round 3): sliding-window inversion in k_qry_prep: query, register, Poseidon and full-size parity,
# then the query line, query serialized stats and a config-3 line.
set -o pipefail
O=gpurun_out/r3q12
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_query.py tests/test_gpu_register.py tests/test_gpu_small_circuits.py tests/test_gpu_fullsize.py -x -v --timeout 400 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --workload query --steps 10 --no-cpu > $O/bench_query.json 2> $O/bench_query.err || { tail -20 $O/bench_query.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_query.json')); print('query', d['value'], {k: v['ms_per_launch'] for k, v in d['phases'].items()})"
PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- \
  python bench.py --workload query --steps 2 --warmup 1 --no-cpu > $O/serial.log 2>&1 || { tail -20 $O/serial.log; exit 1; }
python3 tools/kstats.py $O/serial/run_kernel_stats.csv > $O/serial_stats.txt 2>&1; head -6 $O/serial_stats.txt
timeout -k 10 300 python -u bench.py --no-cpu --no-host --steps 10 > $O/bench_config3.json 2> $O/bench_config3.err || { tail -20 $O/bench_config3.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_config3.json')); print('config3', d['value'], d['roofline']['frac'])"
