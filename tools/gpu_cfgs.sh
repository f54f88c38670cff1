#!/bin/bash
# bench lines for the other BASELINE configs (one short run each)
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
# per-GPU batch: 4096, 8192 for config 4 (65536 gates over 8 GPUs)
for PS in STD100_MKNTRU STD100_MKNTRU_LWE_2 STD128_MKNTRU_3; do
  B=4096; [ $PS = STD128_MKNTRU_3 ] && B=8192
  timeout -k 10 300 python bench.py --paramset $PS --batch $B --steps 1 --warmup 1 --cpu-baseline 0 "$@" > gpurun_out/cfg_${TAG}_$PS.json 2> gpurun_out/cfg_${TAG}_$PS.err || { echo "$PS failed"; tail -3 gpurun_out/cfg_${TAG}_$PS.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/cfg_${TAG}_$PS.json')); print('$PS', round(d['value'],1), d['unit'], 'per_launch_us', round(d['roofline']['per_launch_us'],1))"
done
# config 5 stress: STD100_MKNTRU shape with the 50-bit Q (64-bit word path), with its rocprof summary
timeout -k 10 300 python bench.py --paramset STD100_MKNTRU --q-bits 50 --steps 1 --warmup 1 "$@" > gpurun_out/cfg_${TAG}_cfg5_q50.json 2> gpurun_out/cfg_${TAG}_cfg5_q50.err || { echo "cfg5 failed"; tail -3 gpurun_out/cfg_${TAG}_cfg5_q50.err; exit 1; }
python3 -c "import json,sys; d=json.load(open('gpurun_out/cfg_${TAG}_cfg5_q50.json')); print('cfg5_q50', round(d['value'],1), d['unit'], 'per_launch_us', round(d['roofline']['per_launch_us'],1), 'valu frac', round(d['roofline_valu']['frac'],3))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${TAG}_cfg5 -o run --output-format csv -- \
    python3 bench.py --paramset STD100_MKNTRU --q-bits 50 --steps 1 --warmup 0 --cpu-baseline 0 > gpurun_out/prof_${TAG}_cfg5.log 2>&1 || { echo "cfg5 rocprof failed"; exit 1; }
