#!/bin/bash
# GPU (round 3): the whole -m gpu suite, then the mixed config-5 bench and the default config-3 bench line.
set -o pipefail
mkdir -p gpurun_out/r3_all
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3_all/pytest.log 2>&1 || { tail -40 gpurun_out/r3_all/pytest.log; exit 1; }
tail -3 gpurun_out/r3_all/pytest.log
timeout -k 10 400 python -u bench.py --workload mixed --steps 3 --warmup 1 > gpurun_out/r3_all/bench_mixed.json 2> gpurun_out/r3_all/bench_mixed.err \
  || { tail -20 gpurun_out/r3_all/bench_mixed.err; exit 1; }
cat gpurun_out/r3_all/bench_mixed.json
timeout -k 10 400 python -u bench.py > gpurun_out/r3_all/bench_default.json 2> gpurun_out/r3_all/bench_default.err \
  || { tail -20 gpurun_out/r3_all/bench_default.err; exit 1; }
cat gpurun_out/r3_all/bench_default.json
