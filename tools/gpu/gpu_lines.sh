#!/bin/bash
# GPU: optional parity tests, then bench lines.
# usage: TESTS="<pytest -k expr>|all|none" SMOKE=1 tools/gpu/gpu_lines.sh TAG "name:[VAR=v ...|]bench args" ...
# (a spec may start with environment assignments for that line, separated from the bench args by '|')
# Each line runs `python bench.py <args>` under its own timeout into gpurun_out/TAG/bench_<name>.json and prints
# value / job HBM / per-phase ms; the script stops at the first failure.
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
T=${TESTS:-none}
if [ "$T" = all ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
elif [ "$T" != none ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread -k "$T" \
    > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -1 $O/pytest.log
fi
if [ -n "$SMOKE" ]; then
  timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}; envs=""
  if [[ "$args" == *"|"* ]]; then envs=${args%%|*}; args=${args#*|}; fi
  f=$O/bench_$name.json
  env $envs timeout -k 10 600 python -u bench.py $args > $f 2> $O/bench_$name.err || { tail -20 $O/bench_$name.err; exit 1; }
  python3 - "$f" "$name" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
ph = {k: v["ms_per_launch"] for k, v in d.get("phases", {}).items()}
print(sys.argv[2], d["value"], "job_hbm", d.get("job_hbm", {}).get("frac"), "roof", d.get("roofline", {}).get("frac"), ph)
PY
done
