#!/bin/bash
# PMC passes of one bench workload (rocprofv3 serialises dispatches while it collects counters): instruction mix
# (SQ_*), HBM read bytes (FETCH_SIZE), HBM write bytes (WRITE_SIZE), one counter group per run, then
# tools/pmc_summary.py: per-kernel table + traffic.json (traffic and VALU instructions per witness, keyed by the
# bench line's config.workload).
# usage: tools/gpu/gpu_pmc_line.sh TAG BATCH "bench args"
set -o pipefail
TAG=$1; B=$2; EXTRA=$3
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --batch $B --sub $B --no-cpu --no-host --no-config4 $EXTRA"
timeout -s KILL 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d $O/p_sq -o run -- python bench.py $ARGS > $O/p_sq.log 2>&1 &&
timeout -s KILL 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  --output-format csv -d $O/p_rd -o run -- python bench.py $ARGS > $O/p_rd.log 2>&1 &&
timeout -s KILL 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE \
  --output-format csv -d $O/p_wr -o run -- python bench.py $ARGS > $O/p_wr.log 2>&1 || { echo "pmc pass failed"; tail -5 $O/p_*.log; exit 1; }
WL=$(python3 -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['config']['workload'])" $O/p_wr.log) &&
LK=$(python3 -c "import json,sys; print([json.loads(l) for l in open(sys.argv[1]) if l.startswith('{')][-1]['config'].get('layout_key', 'O0'))" $O/p_wr.log) &&
python3 tools/pmc_summary.py $O/p > $O/summary.txt &&
python3 tools/pmc_summary.py $O/p --json $B $O/traffic.json "$WL" "$LK" || exit 1
head -16 $O/summary.txt | cut -c1-130
python3 -c "import json; d=json.load(open('$O/traffic.json')); print('valu/witness', d.get('valu_insts_per_witness'), 'traffic/witness', sum(k['traffic_bytes_per_witness'] for k in d['kernels'].values()))"
# the scratch CSVs are large: keep the reduced files only
rm -rf $O/p_sq $O/p_rd $O/p_wr
