#!/bin/bash
# GPU (round 4): PMC passes (instruction mix, FETCH_SIZE, WRITE_SIZE) of config 3, QueryIdentity and SIG 20 on this tree
set -o pipefail
tools/gpu/gpu_pmc_r4.sh pmc_r4c 2048 "" && tools/gpu/gpu_pmc_r4.sh pmc_r4q 4096 "--workload query" &&
  tools/gpu/gpu_pmc_r4.sh pmc_r4e 1024 "--sig 20"
