#!/bin/bash
# round 4: config 5 register-resident FP64 kernel with pipelined key stream -- parity, then A/B
# (default pf4, pf2, pf8 variants, and the LDS-tile kernel MKACC_WFP_REG=0)
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_wide.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_wide_parity.txt 2>&1 || { tail -40 $O/${TAG}_wide_parity.txt; exit 1; }
tail -1 $O/${TAG}_wide_parity.txt
BENCH_ARGS="--paramset STD100_MKNTRU --q-bits 50" bash tools/gpu_ab_matrix.sh c5_$TAG "pf4|mkfhe_amd/lib/libmkfhe_amd.so|" "pf2|mkfhe_amd/lib/variants/pf2.so|" "pf8|mkfhe_amd/lib/variants/pf8.so|" "mn0pf8|mkfhe_amd/lib/variants/mn0.so|" "lds|mkfhe_amd/lib/libmkfhe_amd.so|MKACC_WFP_REG=0"
# headline: twiddle / modulus operands of the pinned multiply-adds from VGPRs (MKACC_PIN_VB=1) vs SGPRs
bash tools/gpu_ab_matrix.sh hl_$TAG "def|mkfhe_amd/lib/libmkfhe_amd.so|" "pinvb|mkfhe_amd/lib/variants/pinvb.so|"
