#!/bin/bash
# FP64 wide kernel A/B: parity of the new layouts, then config-5 benches
export TMPDIR=/tmp
mkdir -p gpurun_out/r3
MKFHE_LIB=$PWD/mkfhe_amd/lib/variants/wfpnv.so timeout -k 10 600 python -u -m pytest tests/test_wide.py tests/test_device_entry.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "wide" > gpurun_out/r3/wfp_parity.txt 2>&1 || { tail -30 gpurun_out/r3/wfp_parity.txt; exit 1; }
tail -2 gpurun_out/r3/wfp_parity.txt
BENCH_ARGS="--paramset STD100_MKNTRU --q-bits 50" bash tools/gpu_ab_matrix.sh wfp1 "old|mkfhe_amd/lib/variants/wfpold.so|" "nv|mkfhe_amd/lib/variants/wfpnv.so|" "vol|mkfhe_amd/lib/variants/wfpnew.so|"
