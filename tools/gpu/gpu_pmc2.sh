#!/bin/bash
# stall breakdown per kernel (serialized phases): issue vs wait counters
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 1 --batch 2048 --no-cpu"
PZK_SERIAL=1 timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
  --output-format csv -d gpurun_out/pmcw_sq -o run -- python bench.py $ARGS > gpurun_out/pmcw_sq.log 2>&1 &&
PZK_SERIAL=1 timeout -k 10 600 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmcw_b -o run -- python bench.py $ARGS > gpurun_out/pmcw_b.log 2>&1
echo rc=$?
