#!/bin/bash
# Round 5: RSA tests after the k_rsa_inv store change, config 1 (PoseidonHash(2)) line with its CPU baselines, PMC
# passes of config 3 (traffic), the O2-shaped line and QueryIdentity, and a kernel-trace timeline of the O2 line
set -o pipefail
T0=$(date +%s)
tools/gpu/gpu_lines.sh r5g "poseidon:--workload poseidon --steps 20 --warmup 5" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5c3b 2048 "" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5o2 2048 "--sym o2shape" &&
tools/gpu/gpu_pmc_r4.sh pmc_r5q 4096 "--workload query" &&
echo "elapsed $(( $(date +%s) - T0 ))s" &&
tools/gpu/gpu_timeline.sh r5g "o2tl:--sym o2shape --steps 6 --warmup 2 --no-host --no-cpu" &&
echo "elapsed $(( $(date +%s) - T0 ))s"
