#!/bin/bash
# usage: tools/gpu_ab3.sh TAG LIB.so [LIB.so ...]
#   headline EvalAcc bench per engine build (its in-bench oracle parity check
#   of 16 gates included), ABAB order to expose drift
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_$TAG
for rep in 1 2; do
for L in "$@"; do
  n=$(basename $L .so)
  MKFHE_LIB=$PWD/$L timeout -k 10 300 python bench.py --stage evalacc --steps 2 --warmup 1 --cpu-threads 16 \
     > gpurun_out/ab_$TAG/$n.$rep.json 2> gpurun_out/ab_$TAG/$n.$rep.err || { echo "$n: bench failed"; tail -5 gpurun_out/ab_$TAG/$n.$rep.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$TAG/$n.$rep.json')); print('$n', round(d['value'],1), 'us/launch', round(d['roofline']['per_launch_us'],2), 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
done
done
