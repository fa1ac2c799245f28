#!/bin/bash
# Round end: the whole -m gpu suite, smoke(), the driver's default bench command, rocprofv3 --kernel-trace --stats
# of the same bench command (without the CPU legs), then the other lines.
# usage: tools/gpu/gpu_final.sh TAG
set -o pipefail
TAG=${1:-final}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
T0=$(date +%s)
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo "elapsed $(( $(date +%s) - T0 ))s"
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python3 - "$O/bench_default.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["roofline"]
print("default bench", d["value"], "job_hbm", d["job_hbm"]["frac"], "roof", r["kernel"], r["frac"], r["avg_launch_ms"], "ms",
      "valu", (r.get("valu") or {}).get("frac"), "cpu", d["cpu_baseline"]["value"], "config4", d["config4"]["value"],
      d["config4"]["job_hbm"]["frac"])
PY
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
  -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-host > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python3 tools/kstats.py "$f" > $O/kernel_stats.txt 2>&1
head -16 $O/kernel_stats.txt
python3 -c "import json; d=json.load(open('$O/prof_bench.json')); print('profiled bench', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'], 'ms')"
cp "$f" $O/run_kernel_stats.csv
rm -rf $O/prof
echo "elapsed $(( $(date +%s) - T0 ))s"
tools/gpu/gpu_lines.sh $TAG "query:--workload query --steps 20 --warmup 5" \
  "querytd1:--workload query-td1 --steps 20 --warmup 5 --no-cpu" \
  "o2:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o1:--sym o1shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "sha256:--workload sha256 --steps 20 --warmup 5" \
  "poseidon:--workload poseidon --steps 20 --warmup 5" \
  "sig20:--sig 20 --steps 10 --warmup 2 --no-host --no-cpu" \
  "mixed:--workload mixed --steps 6 --warmup 2" &&
echo "elapsed $(( $(date +%s) - T0 ))s" && echo EXIT 0
