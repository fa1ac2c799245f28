#!/bin/bash
# GPU (round 3): config-3 bench under stream-placement variants: PZK_TAIL (split = tail on the SHA stream; own = a
# fifth stream) x GPU_MAX_HW_QUEUES (4 = HIP's default; 8)
set -o pipefail
O=gpurun_out/r3_ab_streams
mkdir -p $O
export TMPDIR=/tmp
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 4 --warmup 1 --no-cpu --no-host > $O/$tag.json 2> $O/$tag.err \
    || { tail -20 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', d['value'], d['ms_per_step'])"
}
run split_q4 PZK_TAIL=split GPU_MAX_HW_QUEUES=4
run own_q4 PZK_TAIL=own GPU_MAX_HW_QUEUES=4
run split_q8 PZK_TAIL=split GPU_MAX_HW_QUEUES=8
run own_q8 PZK_TAIL=own GPU_MAX_HW_QUEUES=8
run emit_q8 PZK_TAIL=emit GPU_MAX_HW_QUEUES=8
run own_q8_wpb4 PZK_TAIL=own GPU_MAX_HW_QUEUES=8 PZK_POS_WPB=4
run split_q4_again PZK_TAIL=split GPU_MAX_HW_QUEUES=4
