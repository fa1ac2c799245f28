#!/bin/bash
# GPU (round 3, last): query-line A/B of the chain-stream count and the one-emitter-stream switch on the final tree.
set -o pipefail
O=gpurun_out/r3_qab
mkdir -p $O
for cfg in "PZK_QRY_CHAINS=3" "PZK_QRY_CHAINS=2" "PZK_QRY_CHAINS=1" "PZK_QRY_EMIT1=1" "PZK_QRY_CHAINS=3"; do
  f=$O/$(echo $cfg | tr '=' '_').json
  env $cfg timeout -k 10 200 python -u bench.py --workload query --steps 20 --no-cpu > $f.tmp 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$f.tmp')); print('$cfg', d['value'], d['ms_per_step'])" | tee -a $O/summary.txt
  mv $f.tmp $f
done
