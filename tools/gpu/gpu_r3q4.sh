#!/bin/bash
# GPU (round 3): 4-product partial rounds in pos_core_group: query + register + Poseidon parity, then the query
# chain-stream A/B (2 / 3 chains, 4 / 8 hardware queues) and serialized query kernel stats.
set -o pipefail
O=gpurun_out/r3q4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_query.py tests/test_gpu_register.py tests/test_gpu_small_circuits.py -x -v --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload query --steps 10 --no-cpu > $O/bench_$tag.json 2> $O/bench_$tag.err \
    || { tail -20 $O/bench_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('$O/bench_$tag.json')); print('$tag', d['value'], d['ms_per_step'], {k: v['ms_per_launch'] for k, v in d['phases'].items()})"
}
run c2 PZK_QRY_CHAINS=2 && run c3 PZK_QRY_CHAINS=3 && run c3q8 PZK_QRY_CHAINS=3 GPU_MAX_HW_QUEUES=8 || exit 1
PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- \
  python bench.py --workload query --steps 2 --warmup 1 --no-cpu > $O/serial.log 2>&1 || { tail -20 $O/serial.log; exit 1; }
python3 tools/kstats.py $O/serial/run_kernel_stats.csv > $O/serial_stats.txt 2>&1; head -8 $O/serial_stats.txt
