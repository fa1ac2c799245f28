#!/bin/bash
# GPU (round 3): PMC passes of config 3 (instruction mix, HBM read / write bytes per kernel), then the SIG 20 and
# mixed config-5 bench lines on the same tree.
set -o pipefail
O=gpurun_out/r3_pmc
mkdir -p $O
export TMPDIR=/tmp
bash tools/gpu/gpu_pmc.sh pmc_r3 || exit 1
python tools/pmc_summary.py gpurun_out/pmc_r3 > $O/summary.txt &&
python tools/pmc_summary.py gpurun_out/pmc_r3 --json 2048 $O/traffic.json \
  "RegisterIdentityBuilder(1,256,3,4,600,248,1,1496,3,256) synthetic passports (config 3)" || exit 1
head -30 $O/summary.txt | cut -c1-130
timeout -k 10 300 python -u bench.py --workload register-ecdsa --steps 3 --warmup 1 --no-cpu --no-host > $O/bench_sig20.json 2> $O/bench_sig20.err \
  || { tail -20 $O/bench_sig20.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_sig20.json')); print('sig20', d['value'], d['roofline']['achieved'], d['phases']['emit_ect'])"
timeout -k 10 400 python -u bench.py --workload mixed --steps 3 --warmup 1 > $O/bench_mixed.json 2> $O/bench_mixed.err \
  || { tail -20 $O/bench_mixed.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_mixed.json')); print('mixed', d['value'])"
