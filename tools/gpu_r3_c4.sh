#!/bin/bash
# round 3, config 4 (k=8, STD128_MKNTRU_3, B=8192): d_i scratch on/off A/B, then
# the PMC of both (HBM traffic against the accumulator bytes)
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--paramset STD128_MKNTRU_3 --batch 8192" bash tools/gpu_ab_matrix.sh c4 \
  "dscr1|mkfhe_amd/lib/libmkfhe_amd.so|MKACC_DSCR=1" "dscr0|mkfhe_amd/lib/libmkfhe_amd.so|MKACC_DSCR=0" || exit 1
MKACC_DSCR=0 bash tools/gpu_pmc.sh r3_c4_dscr0 STD128_MKNTRU_3 --batch 8192 --stage evalacc \
  > gpurun_out/pmc_r3_c4_dscr0.txt 2>&1 || { cat gpurun_out/pmc_r3_c4_dscr0.txt; exit 1; }
cat gpurun_out/pmc_r3_c4_dscr0.txt
