#!/bin/bash
# round-2 refresh of the other workloads' bench lines (no CPU baseline): ECDSA P-256 (SIG 20), brainpool
# (SIG 21), RSA-PSS (SIG 11), SHA-1 (SIG 3), the mixed config-5 batch and config 2 (Sha256HashChunks(6))
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # tag, bench args
  local tag=$1; shift
  timeout -k 10 400 python -u bench.py "$@" --no-cpu > gpurun_out/bench_wl2_$tag.json 2> gpurun_out/bench_wl2_$tag.err || { tail -20 gpurun_out/bench_wl2_$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_wl2_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['config']['workload'][:60], d['config']['invalid_lanes'])"
}
run sig20 --sig 20 --steps 3 --warmup 1 &&
run sig21 --sig 21 --steps 3 --warmup 1 &&
run sig11 --sig 11 --steps 5 --warmup 1 &&
run sig3 --sig 3 --steps 5 --warmup 1 &&
run mixed --workload mixed --steps 2 --warmup 1 &&
run sha256 --workload sha256 --steps 5 --warmup 1
