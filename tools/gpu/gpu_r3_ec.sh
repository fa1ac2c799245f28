#!/bin/bash
# GPU (round 3): ECDSA parity with the FIPS product in the inlined EC table walker (SIG 20, 21, mixed),
# then the SIG 20 / 21 bench lines with rocprof kernel stats (k_ec_table time).
set -o pipefail
mkdir -p gpurun_out/r3_ec
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ecdsa.py tests/test_gpu_mixed.py -x -v --timeout 150 --timeout-method thread \
  > gpurun_out/r3_ec/pytest.log 2>&1 || { tail -30 gpurun_out/r3_ec/pytest.log; exit 1; }
tail -3 gpurun_out/r3_ec/pytest.log
for wl in register-ecdsa register-brainpool; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu > gpurun_out/r3_ec/bench_$wl.json 2> gpurun_out/r3_ec/bench_$wl.err \
    || { tail -20 gpurun_out/r3_ec/bench_$wl.err; exit 1; }
  cat gpurun_out/r3_ec/bench_$wl.json
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r3_ec/prof -o run -- \
  python $GRAFT_REPO_ROOT/bench.py --workload register-ecdsa --steps 1 --warmup 1 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/r3_ec/prof.log 2>&1
echo prof rc=$?
