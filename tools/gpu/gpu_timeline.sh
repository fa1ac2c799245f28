#!/bin/bash
# GPU: rocprofv3 --kernel-trace --stats of bench lines (concurrent schedule, as bench runs it), then a timeline
# window and per-queue busy fractions (tools/timeline.py) of each.
# usage: tools/gpu/gpu_timeline.sh TAG "name:bench args" ...
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$name -o run -- \
    python bench.py $args > $O/bench_$name.json 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  python3 tools/kstats.py $O/tr_$name/run_kernel_stats.csv > $O/stats_$name.txt 2>&1
  python3 tools/timeline_csv.py $O/tr_$name/run_kernel_trace.csv k_load_values -3 60 > $O/timeline_$name.txt 2>&1
  python3 tools/queue_busy.py $O/tr_$name/run_kernel_trace.csv > $O/queues_$name.txt 2>&1 || true
  echo "== $name"; head -3 $O/bench_$name.json | cut -c1-200; head -12 $O/stats_$name.txt; cat $O/queues_$name.txt | head -20
done
