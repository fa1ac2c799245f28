#!/bin/bash
# GPU (round 3, after the k_emit_mm / k_emit_pos rewrite): default config-3 bench line, serialized kernel stats
# (standalone kernel times), then the three PMC passes (instruction mix, HBM read / write) and their summary.
set -o pipefail
O=gpurun_out/r3c
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_default.json 2> $O/bench_default.err \
  || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('config3', d['value'], d['roofline']['frac'], d['phases']['emit_mm'], d['phases']['emit_pos'])"
PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial -o run -- \
  python bench.py --steps 2 --warmup 1 --no-cpu --no-host > $O/serial.log 2>&1 || { tail -20 $O/serial.log; exit 1; }
python3 tools/kstats.py $O/serial/run_kernel_stats.csv > $O/serial_stats.txt 2>&1; head -26 $O/serial_stats.txt || true
bash tools/gpu/gpu_pmc.sh pmc_r3c || exit 1
python tools/pmc_summary.py gpurun_out/pmc_r3c > $O/summary.txt &&
python tools/pmc_summary.py gpurun_out/pmc_r3c --json 2048 $O/traffic.json \
  "RegisterIdentityBuilder(1,256,3,4,600,248,1,1496,3,256) synthetic passports (config 3)" || exit 1
head -30 $O/summary.txt | cut -c1-130
