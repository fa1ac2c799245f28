#!/bin/bash
# GPU (round 3): isolated k_emit_ect times (PZK_SERIAL=1) over descriptor batch size PZK_ECT_U x prefetch, SIG 20.
set -o pipefail
O=gpurun_out/r3_ect2
mkdir -p $O
export TMPDIR=/tmp
for cfg in "8 0" "8 1" "16 0" "16 1" "32 0"; do
  set -- $cfg
  tag=u$1_pf$2
  cd /tmp && PZK_SERIAL=1 PZK_ECT_U=$1 PZK_ECT_PREFETCH=$2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $GRAFT_REPO_ROOT/$O/$tag -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload register-ecdsa --steps 1 --warmup 1 --batch 1024 \
    --no-cpu --no-host > /dev/null 2> $GRAFT_REPO_ROOT/$O/$tag.err || { tail -20 $GRAFT_REPO_ROOT/$O/$tag.err; exit 1; }
  cd $GRAFT_REPO_ROOT
  python3 -c "
import csv
for r in csv.DictReader(open('$O/$tag/run_kernel_stats.csv')):
    if 'k_emit_ect' in r['Name']: print('$tag', round(float(r['AverageNs'])/1e6, 3))"
done
