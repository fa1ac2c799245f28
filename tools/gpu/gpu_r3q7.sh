#!/bin/bash
# GPU (round 3): PMC passes of the QueryIdentity workload (one call of 4096 witnesses): instruction mix and HBM
# bytes per kernel, then a query line on the current tree.
set -o pipefail
O=gpurun_out/r3q7
mkdir -p $O
export TMPDIR=/tmp
ARGS="--workload query --steps 1 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/pmcq_sq -o run -- python bench.py $ARGS > $O/sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmcq_rd -o run -- python bench.py $ARGS > $O/rd.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE \
  --output-format csv -d gpurun_out/pmcq_wr -o run -- python bench.py $ARGS > $O/wr.log 2>&1 || { tail -20 $O/sq.log $O/rd.log $O/wr.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmcq > $O/summary.txt && head -30 $O/summary.txt | cut -c1-130
timeout -k 10 300 python -u bench.py --workload query --steps 10 --no-cpu > $O/bench_query.json 2> $O/bench_query.err || { tail -20 $O/bench_query.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench_query.json')); print('query', d['value'], {k: v['ms_per_launch'] for k, v in d['phases'].items()})"
