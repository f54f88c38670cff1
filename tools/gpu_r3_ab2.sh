#!/bin/bash
# round 3: wide-path parity of the padded FP64 tile, then headline (party order) and config-5 (tile padding) A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_wide.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r3/wide_parity.txt 2>&1 || { tail -30 gpurun_out/r3/wide_parity.txt; exit 1; }
tail -1 gpurun_out/r3/wide_parity.txt
bash tools/gpu_ab_matrix.sh s2g "v1|mkfhe_amd/lib/libmkfhe_amd.so|MKACC_STEP=1" "def|mkfhe_amd/lib/libmkfhe_amd.so|" "ord0|mkfhe_amd/lib/variants/ord0.so|" || exit 1
BENCH_ARGS="--paramset STD100_MKNTRU --q-bits 50" bash tools/gpu_ab_matrix.sh c5a "pad1|mkfhe_amd/lib/libmkfhe_amd.so|" "pad0|mkfhe_amd/lib/variants/pad0.so|"
