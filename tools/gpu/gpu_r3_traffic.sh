#!/bin/bash
# GPU (round 3, traffic cuts): the whole -m gpu suite, the PMC passes of config 3 (instruction mix, HBM read / write
# bytes per kernel), then the default config-3 bench line on the same tree.
set -o pipefail
TAG=${1:-r3t}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu/gpu_pmc.sh pmc_$TAG || exit 1
python tools/pmc_summary.py gpurun_out/pmc_$TAG > $O/summary.txt &&
python tools/pmc_summary.py gpurun_out/pmc_$TAG --json 2048 $O/traffic.json \
  "RegisterIdentityBuilder(1,256,3,4,600,248,1,1496,3,256) synthetic passports (config 3)" || exit 1
head -26 $O/summary.txt | cut -c1-120
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err \
  || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('config3', d['value'], d['roofline']['frac'], d['job_hbm'])"
