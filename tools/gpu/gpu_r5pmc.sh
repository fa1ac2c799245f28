#!/bin/bash
# Round 5, last tree: config-3 PMC passes (512-thread k_emit_mm)
set -o pipefail
tools/gpu/gpu_pmc_r4.sh pmc_r5c3e 2048 ""
