#!/bin/bash
# round 4: the other BASELINE configs with batch slices (defaults)
export TMPDIR=/tmp
O=gpurun_out/r4
mkdir -p $O
run() {  # name, env, bench args
  env $2 timeout -k 10 400 python bench.py $3 > $O/${TAG}_$1.json 2> $O/${TAG}_$1.err || { echo "$1 failed"; tail -5 $O/${TAG}_$1.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/${TAG}_$1.json')); print('$1', round(d['value'],1), round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['per_launch_us'],2), 'us/step', d['roofline']['kernel'], 'parity', d.get('parity_checked'), d.get('parity_mismatches'))"
}
run std100 "" "--steps 3 --warmup 1 --cpu-threads 16 --paramset STD100_MKNTRU"
run std100lwe2 "" "--steps 3 --warmup 1 --cpu-threads 16 --paramset STD100_MKNTRU_LWE_2"
run std100_s1 "MKACC_STREAMS=1" "--steps 3 --warmup 1 --cpu-threads 16 --paramset STD100_MKNTRU"
run std100lwe2_s1 "MKACC_STREAMS=1" "--steps 3 --warmup 1 --cpu-threads 16 --paramset STD100_MKNTRU_LWE_2"
