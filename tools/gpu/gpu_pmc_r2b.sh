#!/bin/bash
# PMC passes of the final round-2 kernels (config 3, one bench step of 2048 witnesses) and their
# summary / per-witness traffic (profiles/pmc_r2b), so roofline.traffic and the per-kernel table
# describe the kernels the bench times
set -o pipefail
bash tools/gpu/gpu_pmc.sh pmc_r2b || exit 1
python tools/pmc_summary.py gpurun_out/pmc_r2b > gpurun_out/pmc_r2b_summary.txt &&
python tools/pmc_summary.py gpurun_out/pmc_r2b --json 2048 gpurun_out/pmc_r2b_traffic.json \
  "RegisterIdentityBuilder(1,256,3,4,600,248,1,1496,3,256) synthetic passports (config 3)" &&
cat gpurun_out/pmc_r2b_summary.txt | cut -c1-120
