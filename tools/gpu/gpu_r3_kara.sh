#!/bin/bash
# GPU (round 3): the whole -m gpu suite on the table-driven Karatsuba emitter, then the section clocks of the
# profiling build (gpu_r3_prof.sh) and the default config-3 line.
set -o pipefail
O=gpurun_out/r3_kara
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
bash tools/gpu/gpu_r3_prof.sh || exit 1
timeout -k 10 400 python -u bench.py --no-cpu > $O/bench_default.json 2> $O/bench_default.err \
  || { tail -20 $O/bench_default.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_default.json')); print('config3', d['value'], d['roofline']['frac'], d['phases']['emit_mm'])"
