#!/bin/bash
# GPU (round 3): compile-time store modes — mapped + register parity, O0 and mapped bench lines (with host_delivered)
set -o pipefail
mkdir -p gpurun_out/r3_sym2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_symmap.py tests/test_gpu_stream.py tests/test_gpu_register.py tests/test_gpu_pss.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r3_sym2/pytest.log 2>&1 || { tail -40 gpurun_out/r3_sym2/pytest.log; exit 1; }
tail -3 gpurun_out/r3_sym2/pytest.log
for k in 1 2; do
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu --no-host > gpurun_out/r3_sym2/bench_o0_$k.json 2> gpurun_out/r3_sym2/bench_o0_$k.err \
  || { tail -20 gpurun_out/r3_sym2/bench_o0_$k.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3_sym2/bench_o0_$k.json'));print('o0',d['value'],d['roofline']['avg_launch_ms'])"
done
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 --no-cpu --sym synthetic:4 > gpurun_out/r3_sym2/bench_sym4.json 2> gpurun_out/r3_sym2/bench_sym4.err \
  || { tail -20 gpurun_out/r3_sym2/bench_sym4.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/r3_sym2/bench_sym4.json'));print('sym4',d['value'],d['roofline'],d['host_delivered'])"
