#!/bin/bash
# usage: tools/gpu_wide.sh TAG -- 64-bit word path: parity tests + the 50-bit config-5 stress bench
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wide.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_$TAG.txt 2>&1
rc=$?; tail -3 gpurun_out/pytest_$TAG.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --paramset STD100_MKNTRU --q-bits 50 --steps 1 --warmup 1 --cpu-baseline 0 "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; tail -2 gpurun_out/bench_$TAG.err; cat gpurun_out/bench_$TAG.json
exit $rc
