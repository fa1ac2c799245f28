#!/bin/bash
# GPU (round 3): k_emit_ect descriptor prefetch A/B on SIG 20 / 24 (PZK_ECT_PREFETCH 1 / 0), isolated kernel times
# under PZK_SERIAL=1 rocprof, then the ECDSA parity tests.
set -o pipefail
O=gpurun_out/r3_ect
mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, sig, prefetch
  PZK_ECT_PREFETCH=$3 timeout -k 10 300 python -u bench.py --workload register-ecdsa --sig $2 --steps 3 --warmup 1 --no-cpu --no-host \
    > $O/$1.json 2> $O/$1.err || { tail -20 $O/$1.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$1.json')); ph=d['phases']
print('$1', d['value'], d['roofline']['achieved'], {k: ph[k]['ms_per_launch'] for k in ('emit_gen','emit_ecr','emit_ect') if k in ph})"
}
run s20_pf1 20 1
run s20_pf0 20 0
run s20_pf1b 20 1
run s24_pf1 24 1
run s24_pf0 24 0
for pf in 1 0; do
  cd /tmp && PZK_SERIAL=1 PZK_ECT_PREFETCH=$pf timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_pf$pf -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload register-ecdsa --steps 1 --warmup 1 --batch 1024 --no-cpu --no-host > /dev/null 2> $GRAFT_REPO_ROOT/$O/prof_pf$pf.err \
    || { tail -20 $GRAFT_REPO_ROOT/$O/prof_pf$pf.err; exit 1; }
  cd $GRAFT_REPO_ROOT
  grep -h "k_emit_ect\|k_emit_ecr\|k_emit_gen" $O/prof_pf$pf/run_kernel_stats.csv | cut -d, -f1-4 | cut -c1-40,200-
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_ecdsa.py -x -q --timeout 240 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
