#!/bin/bash
# Round 5: the signature emitters (k_emit_mm) on a stream of their own (PZK_SIGEMIT=own, PZK_MM_PRIO=hi|lo) against
# the RSA stream, on configs 3 / 4 and the O2-shaped line; register + mapped parity under the switch first
set -o pipefail
T0=$(date +%s)
O=gpurun_out/r5n
mkdir -p $O
PZK_SIGEMIT=own timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "register or symmap" > $O/pytest_own.log 2>&1 || { tail -30 $O/pytest_own.log; exit 1; }
tail -1 $O/pytest_own.log
tools/gpu/gpu_lines.sh r5n "c3:--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3own:PZK_SIGEMIT=own|--steps 20 --warmup 5 --no-cpu --no-host" \
  "c3ownhi:PZK_SIGEMIT=own PZK_MM_PRIO=hi|--steps 20 --warmup 5 --no-cpu --no-host" \
  "o2:--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2own:PZK_SIGEMIT=own|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "o2ownhi:PZK_SIGEMIT=own PZK_MM_PRIO=hi|--sym o2shape --steps 20 --warmup 5 --no-host --no-cpu" \
  "c3b:--steps 20 --warmup 5 --no-cpu --no-host" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
