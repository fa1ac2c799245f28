#!/bin/bash
# Round end: the whole -m gpu suite, smoke(), the default bench line (the command the driver runs), then
# rocprofv3 --kernel-trace --stats of the same bench command (without the CPU legs), reduced to a per-kernel summary.
# usage: tools/gpu/gpu_r4_final.sh TAG
set -o pipefail
TAG=${1:-r4_final}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 - "$O/bench_default.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("default bench", d["value"], "job_hbm", d["job_hbm"]["frac"], "roof", r["kernel"], r["frac"], r["avg_launch_ms"], "ms",
      "valu", (r.get("valu") or {}).get("frac"), "cpu", d["cpu_baseline"]["value"])
PY
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python3 bench.py --no-cpu --no-host > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python3 tools/kstats.py "$f" > $O/kernel_stats.txt 2>&1
head -16 $O/kernel_stats.txt
python3 -c "import json; d=json.load(open('$O/prof_bench.json')); print('profiled bench', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], 'ms')"
echo EXIT 0
