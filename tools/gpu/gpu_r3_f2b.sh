#!/bin/bash
# GPU (round 3, f2): SOD -> witness for SIG 25, then the SIG 24 / 25 bench lines and their kernel profiles.
set -o pipefail
O=gpurun_out/r3_f2b
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_passport.py -x -v --timeout 240 --timeout-method thread \
  > $O/passport.log 2>&1 || { tail -40 $O/passport.log; exit 1; }
tail -4 $O/passport.log
for s in 24 25; do
  timeout -k 10 420 python -u bench.py --workload register-ecdsa --sig $s --steps 3 --warmup 1 --cpu-sample 256 --no-host \
    > $O/bench_sig$s.json 2> $O/bench_sig$s.err || { tail -20 $O/bench_sig$s.err; exit 1; }
  cat $O/bench_sig$s.json
done
for s in 24 25; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sig$s -o run -- python3 bench.py --workload register-ecdsa \
    --sig $s --steps 2 --warmup 1 --no-cpu --no-host > $O/prof_sig$s.json 2> $O/prof_sig$s.err || { tail -20 $O/prof_sig$s.err; exit 1; }
done
find $O -name "*kernel_stats.csv" | head
