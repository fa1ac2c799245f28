#!/bin/bash
# GPU (round 3): section clocks of k_emit_mm / k_emit_pos from the profiling build (make EXTRA=-DPZK_MM_PROF into
# lib/ab/libpzkwit_prof.so): config 3, kernels serialized (PZK_SERIAL=1) and concurrent.
set -o pipefail
O=gpurun_out/r3_prof
mkdir -p $O
export TMPDIR=/tmp
LIB=passport-zk-circuits_amd/lib/ab/libpzkwit_prof.so
export PZK_DATA_DIR=$GRAFT_REPO_ROOT/passport-zk-circuits_amd/data
PZK_SERIAL=1 PZK_LIB=$LIB timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-host > $O/serial.json 2> $O/serial.err \
  || { tail -20 $O/serial.err; exit 1; }
grep "_prof" $O/serial.err | tail -2
PZK_LIB=$LIB timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-host > $O/conc.json 2> $O/conc.err \
  || { tail -20 $O/conc.err; exit 1; }
grep "_prof" $O/conc.err | tail -2
