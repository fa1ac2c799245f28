#!/bin/bash
# GPU (round 3): config-3 bench + kernel trace with k_emit_pos's witnesses-per-workgroup A/B (PZK_POS_WPB 1 / 4 / 8)
set -o pipefail
O=gpurun_out/r3_ab_pos
mkdir -p $O
export TMPDIR=/tmp
for wpb in 1 4 8; do
  PZK_POS_WPB=$wpb timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --no-host > $O/bench_wpb$wpb.json 2> $O/bench_wpb$wpb.err \
    || { tail -20 $O/bench_wpb$wpb.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench_wpb$wpb.json')); print($wpb, d['value'], d['ms_per_step'], d['phases']['emit_pos'])"
done
for wpb in 1 4; do
  cd /tmp && PZK_POS_WPB=$wpb timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_wpb$wpb -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu --no-host > $GRAFT_REPO_ROOT/$O/prof_wpb$wpb.json 2> $GRAFT_REPO_ROOT/$O/prof_wpb$wpb.err \
    || { tail -20 $GRAFT_REPO_ROOT/$O/prof_wpb$wpb.err; exit 1; }
  cd $GRAFT_REPO_ROOT
done
find $O -name "*kernel_stats.csv" | while read f; do echo $f; head -12 $f | cut -c1-160; done
