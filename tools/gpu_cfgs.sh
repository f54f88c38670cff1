#!/bin/bash
# bench lines for the other BASELINE configs (one short run each)
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for PS in STD100_MKNTRU STD100_MKNTRU_LWE_2 STD128_MKNTRU_3; do
  timeout -k 10 300 python bench.py --paramset $PS --steps 1 --warmup 1 --cpu-baseline 0 "$@" > gpurun_out/cfg_${TAG}_$PS.json 2> gpurun_out/cfg_${TAG}_$PS.err || { echo "$PS failed"; tail -3 gpurun_out/cfg_${TAG}_$PS.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/cfg_${TAG}_$PS.json')); print('$PS', round(d['value'],1), d['unit'], 'per_launch_us', round(d['roofline']['per_launch_us'],1))"
done
