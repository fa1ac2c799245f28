#!/bin/bash
# signature-emitter placement A/B on the ECDSA, RSA-4096 and mixed workloads (PZK_SIGEMIT=emit puts
# emit_mm / emit_ect on the emit stream instead of behind the signature chain on the RSA stream)
set -o pipefail
mkdir -p gpurun_out
run() {  # tag, env value, bench args
  local tag=$1 se=$2; shift 2
  PZK_SIGEMIT=$se timeout -k 10 400 python -u bench.py "$@" --no-cpu > gpurun_out/bench_se_$tag.json 2> gpurun_out/bench_se_$tag.err || { tail -20 gpurun_out/bench_se_$tag.err; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_se_$tag.json')); print('$tag', d['value'], d['ms_per_step'], d['config']['invalid_lanes'])"
}
run sig20_emit emit --sig 20 --steps 3 --warmup 1 &&
run sig20_rsa rsa --sig 20 --steps 3 --warmup 1 &&
run sig2_emit emit --sig 2 --steps 3 --warmup 1 &&
run sig2_rsa rsa --sig 2 --steps 3 --warmup 1 &&
run mixed_emit emit --workload mixed --steps 2 --warmup 1 &&
run mixed_rsa rsa --workload mixed --steps 2 --warmup 1
