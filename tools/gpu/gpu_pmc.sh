#!/bin/bash
# PMC passes over one bench step (config 3, batch 2048): instruction mix, then HBM read bytes,
# then HBM write bytes (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-pmc}
ARGS="--steps 1 --warmup 1 --batch 2048 --no-cpu --no-host"
timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  --output-format csv -d gpurun_out/${TAG}_sq -o run -- python bench.py $ARGS > gpurun_out/${TAG}_sq.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/${TAG}_rd -o run -- python bench.py $ARGS > gpurun_out/${TAG}_rd.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace --pmc WRITE_SIZE \
  --output-format csv -d gpurun_out/${TAG}_wr -o run -- python bench.py $ARGS > gpurun_out/${TAG}_wr.log 2>&1
echo rc=$?
