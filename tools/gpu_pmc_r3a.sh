#!/bin/bash
# round 3: PMC of the current build for config 4 (STD128_MKNTRU_3, B=8192) and
# config 5 (50-bit Q, FP64 wide kernels); one rocprofv3 pass per counter set
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_pmc.sh r3_c4 STD128_MKNTRU_3 --batch 8192 --stage evalacc > gpurun_out/pmc_r3_c4.txt 2>&1 || { cat gpurun_out/pmc_r3_c4.txt; exit 1; }
bash tools/gpu_pmc.sh r3_c5 STD100_MKNTRU --q-bits 50 --stage evalacc > gpurun_out/pmc_r3_c5.txt 2>&1 || { cat gpurun_out/pmc_r3_c5.txt; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmc_r3_c5 step_kernel
