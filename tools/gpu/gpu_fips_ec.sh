#!/bin/bash
# GPU: the ECDSA parity tests against the PZK_FR_FIPS_ALL build (FIPS Fr product in every kernel,
# including the EC table walker), under a short time limit. LOG=1: serialised launches with the HIP
# runtime's dispatch log, so a hang names its kernel (the last dispatch logged).
set -o pipefail
mkdir -p gpurun_out/fips_ec
export TMPDIR=/tmp
export PZK_LIB=$PWD/passport-zk-circuits_amd/${VARIANT:-lib_x/fips}/libpzkwit.so
export PZK_DATA_DIR=$PWD/passport-zk-circuits_amd/data
if [ -n "$LOG" ]; then export PZK_SERIAL=1 HIP_LAUNCH_BLOCKING=1 AMD_LOG_LEVEL=3; fi
timeout -k 10 ${TLIM:-240} python -u -m pytest tests/test_gpu_ecdsa.py -x -v --timeout ${PTLIM:-150} --timeout-method thread ${TESTK:+-k $TESTK} \
  > gpurun_out/fips_ec/pytest.log 2> gpurun_out/fips_ec/stderr.log
rc=$?
grep -a "ShaderName" gpurun_out/fips_ec/stderr.log | tail -20 > gpurun_out/fips_ec/last_dispatch.txt
tail -5 gpurun_out/fips_ec/last_dispatch.txt
grep -v "^\s*$" gpurun_out/fips_ec/pytest.log | grep -E "PASS|FAIL|Timeout|Error|passed|failed" | head -20
rm -f gpurun_out/fips_ec/stderr.log
exit $rc
