#!/bin/bash
# GPU (round 3): whole -m gpu suite (mapsink touched every emitter; direct .sym emission, streaming), then
# the config-3 line with host_delivered, the --sym synthetic:4 line (direct) and its staging+gather A/B,
# and a rocprof kernel trace of the mapped line.
set -o pipefail
mkdir -p gpurun_out/r3_sym
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3_sym/pytest.log 2>&1 || { tail -40 gpurun_out/r3_sym/pytest.log; exit 1; }
tail -3 gpurun_out/r3_sym/pytest.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/r3_sym/bench_o0.json 2> gpurun_out/r3_sym/bench_o0.err \
  || { tail -20 gpurun_out/r3_sym/bench_o0.err; exit 1; }
cat gpurun_out/r3_sym/bench_o0.json
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --no-cpu --sym synthetic:4 > gpurun_out/r3_sym/bench_sym4.json 2> gpurun_out/r3_sym/bench_sym4.err \
  || { tail -20 gpurun_out/r3_sym/bench_sym4.err; exit 1; }
cat gpurun_out/r3_sym/bench_sym4.json
PZK_SYM_GATHER=1 timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-host --sym synthetic:4 > gpurun_out/r3_sym/bench_sym4_gather.json 2> gpurun_out/r3_sym/bench_sym4_gather.err \
  || { tail -20 gpurun_out/r3_sym/bench_sym4_gather.err; exit 1; }
cat gpurun_out/r3_sym/bench_sym4_gather.json
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_sym/prof_sym4 -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu --no-host --sym synthetic:4 > $GRAFT_REPO_ROOT/gpurun_out/r3_sym/prof_sym4.log 2>&1
echo prof rc=$?
