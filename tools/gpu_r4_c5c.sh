#!/bin/bash
# round 4: config 5 widereg scheduler / register-pressure A/B, then PMC of the default build
export TMPDIR=/tmp
BENCH_ARGS="--paramset STD100_MKNTRU --q-bits 50" bash tools/gpu_ab_matrix.sh c5c_$TAG "pf4|mkfhe_amd/lib/libmkfhe_amd.so|" "ilp|mkfhe_amd/lib/variants/wr_max-ilp.so|" "mmc|mkfhe_amd/lib/variants/wr_max-memory-clause.so|" "mn0pf4|mkfhe_amd/lib/variants/mn0pf4.so|" "mn0ilp|mkfhe_amd/lib/variants/mn0ilp.so|" || exit 1
TAG=$TAG bash tools/gpu_r4_pmc_c5.sh
