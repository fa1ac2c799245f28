#!/bin/bash
# GPU (round 3): serialized QueryIdentity kernel times at 2048 vs 4096 witnesses per call (k_emit_bits scaling).
set -o pipefail
O=gpurun_out/r3q8
mkdir -p $O
export TMPDIR=/tmp
for b in 2048 4096; do
  PZK_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/serial_$b -o run -- \
    python bench.py --workload query --steps 2 --warmup 1 --no-cpu --batch $b > $O/serial_$b.log 2>&1 || { tail -20 $O/serial_$b.log; exit 1; }
  python3 tools/kstats.py $O/serial_$b/run_kernel_stats.csv > $O/serial_$b.txt 2>&1; grep -E "emit_bits|emit_gen|emit_qry|smt_chain|emit_pos<3" $O/serial_$b.txt
done
