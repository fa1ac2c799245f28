#!/bin/bash
# HBM traffic of one RegisterIdentityBuilder instance: FETCH_SIZE and WRITE_SIZE passes (one counter
# group per run) over one bench step of BATCH witnesses in a single launch, reduced by
# tools/pmc_summary.py to profiles/pmc_r1_sigSIG/traffic.json (keyed by bench.py's config.workload),
# then the default bench line of the same instance, which picks that file up as roofline.traffic.
# usage: tools/gpu/gpu_pmc_wl.sh SIG BATCH
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SIG=$1; B=$2; TAG=pmc_sig$SIG
ARGS="--sig $SIG --steps 1 --warmup 1 --batch $B --sub $B --no-cpu"
timeout -k 10 400 rocprofv3 --kernel-trace --pmc FETCH_SIZE \
  --output-format csv -d gpurun_out/${TAG}_rd -o run -- python bench.py $ARGS > gpurun_out/${TAG}_rd.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --pmc WRITE_SIZE \
  --output-format csv -d gpurun_out/${TAG}_wr -o run -- python bench.py $ARGS > gpurun_out/${TAG}_wr.log 2>&1 &&
WL=$(python -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['config']['workload'])" gpurun_out/${TAG}_wr.log) &&
mkdir -p profiles/pmc_r1_sig$SIG &&
python tools/pmc_summary.py gpurun_out/$TAG --json $B profiles/pmc_r1_sig$SIG/traffic.json "$WL" &&
cp profiles/pmc_r1_sig$SIG/traffic.json gpurun_out/${TAG}_traffic.json &&
timeout -k 10 400 python bench.py --sig $SIG > gpurun_out/bench_sig$SIG.json 2> gpurun_out/bench_sig$SIG.log
rc=$?; echo "sig $SIG rc=$rc"; exit $rc
