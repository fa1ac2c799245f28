#!/bin/bash
# GPU (round 3): k_emit_ecr (EC selection tables) — ECDSA parity (4 curves + .sym-mapped), then same-box A/B against
# the pre-rewrite library (lib/ab/libpzkwit_old.so) on SIG 20 and config 3.
set -o pipefail
O=gpurun_out/r3_ecr
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ecdsa.py tests/test_gpu_symmap.py -x -v --timeout 300 --timeout-method thread \
  > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
run() {  # tag, workload, lib
  local tag=$1 wl=$2 lib=$3
  PZK_DATA_DIR=$GRAFT_REPO_ROOT/passport-zk-circuits_amd/data PZK_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl \
    --steps 3 --warmup 1 --no-cpu --no-host > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$tag.json')); ph=d['phases']
print('$tag', d['value'], {k: ph[k]['ms_per_launch'] for k in ('emit_gen','emit_ecr','ec_core','ec_table','emit_ect') if k in ph})"
}
NEW=passport-zk-circuits_amd/lib/libpzkwit.so
OLD=passport-zk-circuits_amd/lib/ab/libpzkwit_old.so
run sig20_new register-ecdsa $NEW
run sig20_old register-ecdsa $OLD
run sig20_new2 register-ecdsa $NEW
run cfg3_new register $NEW
run cfg3_old register $OLD
run cfg3_new2 register $NEW
