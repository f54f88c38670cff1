#!/bin/bash
# round 3: FP64 wide kernel with register-fed transforms -- parity, then config-5 A/B
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
timeout -k 10 600 python -u -m pytest tests/test_wide.py tests/test_device_entry.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/r3/wfp2_parity.txt 2>&1 || { tail -30 gpurun_out/r3/wfp2_parity.txt; exit 1; }
tail -1 gpurun_out/r3/wfp2_parity.txt
BENCH_ARGS="--paramset STD100_MKNTRU --q-bits 50" bash tools/gpu_ab_matrix.sh c5b "new4|mkfhe_amd/lib/libmkfhe_amd.so|" "old|mkfhe_amd/lib/variants/wfpold.so|" "new3|mkfhe_amd/lib/variants/wg3.so|" "new5|mkfhe_amd/lib/variants/wg5.so|"
