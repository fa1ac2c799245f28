#!/bin/bash
# k_emit_ect A/B builds (ab/lib_<name>.so, PZK_LIB): serialized per-kernel times of SIG 20 (rocprofv3 stats) for
# every build, then the concurrent SIG 20 line for the given ones.
# usage: tools/gpu/gpu_r4_ectab.sh TAG "base wpe4 ..." "base wpe4 ..."
set -o pipefail
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
lib() { if [ "$1" = base ]; then echo ""; else echo "$PWD/passport-zk-circuits_amd/ab/lib_$1.so"; fi; }
for n in $2; do
  PZK_LIB=$(lib $n) PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s_$n -o run \
    -- python3 bench.py --sig 20 --steps 1 --warmup 1 --batch 1024 --no-cpu --no-host > $O/s_$n.log 2>&1 || { tail -20 $O/s_$n.log; exit 1; }
  f=$(find $O/s_$n -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    if "k_emit_ect" in r["Name"] or "k_ec_table" in r["Name"] or "k_emit_sha<" in r["Name"]:
        print(sys.argv[2], r["Name"][:40], r["Calls"], "avg_ms", round(float(r["AverageNs"]) / 1e6, 3))
PY
done
for n in $3; do
  PZK_LIB=$(lib $n) timeout -k 10 300 python3 bench.py --sig 20 --steps 6 --warmup 2 --no-cpu --no-host > $O/b_$n.json 2> $O/b_$n.err || { tail -20 $O/b_$n.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'job_hbm', d['job_hbm']['frac'], {k: v['ms_per_launch'] for k, v in d['phases'].items()})" $O/b_$n.json $n
done
echo EXIT 0
