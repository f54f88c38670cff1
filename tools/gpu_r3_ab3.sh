#!/bin/bash
# round 3: index-party store policy A/B (headline), and step kernels at k = 4 (STD128_MKNTRU_2: v2 against v1 with its d_i scratch)
export TMPDIR=/tmp
bash tools/gpu_ab_matrix.sh s2i "v1|mkfhe_amd/lib/libmkfhe_amd.so|MKACC_STEP=1" "def|mkfhe_amd/lib/libmkfhe_amd.so|" "idx|mkfhe_amd/lib/variants/idx.so|" || exit 1
BENCH_ARGS="--paramset STD128_MKNTRU_2" bash tools/gpu_ab_matrix.sh k4 "v1|mkfhe_amd/lib/libmkfhe_amd.so|MKACC_STEP=1" "v2|mkfhe_amd/lib/libmkfhe_amd.so|"
