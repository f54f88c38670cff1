#!/bin/bash
# round 4: config 4 -- mk_step2_kernel at dg = 4 in two halves (MKACC_STEP=2; default 2-slot groups, 2 ahead;
# variants h40 = 4-slot groups no prefetch, h21 = 2-slot groups 1 ahead) against mk_step_kernel + d_i scratch
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "step_kernels" --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $O/${TAG}_c4_parity.txt 2>&1 || { tail -40 $O/${TAG}_c4_parity.txt; exit 1; }
tail -1 $O/${TAG}_c4_parity.txt
BENCH_ARGS="--paramset STD128_MKNTRU_3 --batch 8192" bash tools/gpu_ab_matrix.sh c4_$TAG "v1|mkfhe_amd/lib/libmkfhe_amd.so|MKACC_STEP=1" "h22|mkfhe_amd/lib/libmkfhe_amd.so|MKACC_STEP=2" "h40|mkfhe_amd/lib/variants/h40.so|MKACC_STEP=2" "h21|mkfhe_amd/lib/variants/h21.so|MKACC_STEP=2"
