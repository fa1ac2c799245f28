#!/bin/bash
# emit_mm section-cost probe (serialized): PZK_MM_SKIP bit s = section s emits zeros
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
# sections: 0 Q 1 R 2 XYN 3 MOUT 4 MCOPY 5 KARA 6 MODCHK 7 GT0 8 GTIN 9 LE0 10 LEIN 11 LERES 12 LT 13 M2OUT 14 M2IN 15 TMPM 16 TMPR 17 ISZIN 18 CARRY 19 RANGE
for m in 0 0x20 0x10000 0x1000 0x80040 0x8000 0xe0000 0xfffff; do
  PZK_SERIAL=1 PZK_MM_SKIP=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mmp_$m -o run -- python bench.py --steps 1 --warmup 1 --batch 2048 --no-cpu > gpurun_out/mmp_$m.log 2>&1 || exit $?
done
echo done
