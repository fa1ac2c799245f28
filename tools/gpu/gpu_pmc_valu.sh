#!/bin/bash
# One PMC pass per bench line for VALU issue cycles (SQ_ACTIVE_INST_VALU beside SQ_INSTS_VALU and its int32 /
# int64 split), then tools/pmc_valu.py. rocprofv3 serialises dispatches while it collects counters: the figures
# are per-kernel costs, not the concurrent schedule.
# usage: tools/gpu/gpu_pmc_valu.sh TAG "name:BATCH:RATE:bench args" ...   (RATE: the line's witnesses/s, or -)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; B=${rest%%:*}; rest=${rest#*:}; RATE=${rest%%:*}; args=${rest#*:}
  timeout -s KILL 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 \
    --output-format csv -d $O/v_$name -o run -- \
    python bench.py --steps 1 --warmup 1 --batch $B --sub $B --no-cpu --no-host --no-config4 $args \
    > $O/v_$name.log 2>&1 || { echo "pmc pass $name failed"; tail -5 $O/v_$name.log; exit 1; }
  python3 tools/pmc_valu.py $O/v_$name/run_counter_collection.csv $B $RATE $O/valu_$name.json > $O/valu_$name.txt || exit 1
  echo "== $name"; head -14 $O/valu_$name.txt; tail -2 $O/valu_$name.txt
  rm -rf $O/v_$name
done
