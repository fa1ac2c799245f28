#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --workload sha256 --steps 3 --warmup 1 > gpurun_out/bench_sha.json 2> gpurun_out/bench_sha.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sha -o run -- python bench.py --workload sha256 --steps 2 --warmup 1 --no-cpu > gpurun_out/prof_sha.log 2>&1
echo rc=$?
