#!/bin/bash
# GPU (round 3): same-box A/B of the library before the generic-chunk EC rewrite (commit 0dfb197, built into
# lib/ab/libpzkwit_old.so) against the current one: SIG 20 and config 3, alternating.
set -o pipefail
O=gpurun_out/r3_ab_old
mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, workload, lib
  local tag=$1 wl=$2 lib=$3
  PZK_DATA_DIR=$GRAFT_REPO_ROOT/passport-zk-circuits_amd/data PZK_LIB=$lib timeout -k 10 300 python -u bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --no-host > $O/$tag.json 2> $O/$tag.err \
    || { tail -20 $O/$tag.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/$tag.json')); ph=d['phases']
print('$tag', d['value'], {k: ph[k]['ms_per_launch'] for k in ('emit_gen','ec_core','ec_table','emit_ect') if k in ph})"
}
NEW=passport-zk-circuits_amd/lib/libpzkwit.so
OLD=passport-zk-circuits_amd/lib/ab/libpzkwit_old.so
run sig20_new register-ecdsa $NEW
run sig20_old register-ecdsa $OLD
run sig20_new2 register-ecdsa $NEW
run sig20_old2 register-ecdsa $OLD
run cfg3_new register $NEW
run cfg3_old register $OLD
